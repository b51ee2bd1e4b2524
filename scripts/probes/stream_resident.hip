// Probe: temporal blocking of the headline update.
//
// k_batch_stream (pqp_kernels.hip) streams each problem's 4 MiB of Qd from HBM
// once per iteration of a launch (10 iterations per launch in the bench).
// Here part of each problem's Qd stays on the CU across the launch's
// iterations, so only the first iteration reads it from HBM:
//   RA blocks (16 k x 1024 rows each, 64 KiB) in registers (AGPR-backed:
//      the stream buffers already take the 256 arch VGPRs),
//   RL blocks in LDS (beside the 8 KiB iterate ping-pong),
//   R further blocks loaded with the default cache policy instead of `nt`
//      (reuse from L2 / the Infinity Cache, if the nt stream leaves them there).
// The arithmetic and its order are the hot kernel's (same bits: the output of
// every variant is compared with the (0,0,0) variant's).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off stream_resident.hip -o stream_resident
// Run:   ./stream_resident [B=4096] [reps=5]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#pragma clang fp contract(off)

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

__device__ __forceinline__ float max_ref(float a, float b) { return (a > b) ? a : b; }

typedef float f32x4 __attribute__((ext_vector_type(4)));
template <bool NTL>
__device__ __forceinline__ float4 ldq4(const float* p) {
    if constexpr (NTL) {
        const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *reinterpret_cast<const float4*>(p);
    }
}

struct Acc4 {
    float p[4], n[4];
};
__device__ __forceinline__ void lean4(Acc4& a, float4 q, float y) {
    const float z = 0.0f * y;
    float p;
    p = q.x * y; a.p[0] += (q.x < 0.0f) ? z : p; a.n[0] += (q.x > 0.0f) ? z : -p;
    p = q.y * y; a.p[1] += (q.y < 0.0f) ? z : p; a.n[1] += (q.y > 0.0f) ? z : -p;
    p = q.z * y; a.p[2] += (q.z < 0.0f) ? z : p; a.n[2] += (q.z > 0.0f) ? z : -p;
    p = q.w * y; a.p[3] += (q.w < 0.0f) ? z : p; a.n[3] += (q.w > 0.0f) ? z : -p;
}
__device__ __forceinline__ void literal1(float& ap, float& an, float q, float y, float t) {
    const float qp = max_ref(0.0f, q) + t;
    const float qn = max_ref(0.0f, -q) + t;
    ap += qp * y;
    an += qn * y;
}
__device__ __forceinline__ void literal4(Acc4& a, float4 q, float y, int k, int row, const float th[4]) {
    literal1(a.p[0], a.n[0], q.x, y, (k == row + 0) ? th[0] : 0.0f);
    literal1(a.p[1], a.n[1], q.y, y, (k == row + 1) ? th[1] : 0.0f);
    literal1(a.p[2], a.n[2], q.z, y, (k == row + 2) ? th[2] : 0.0f);
    literal1(a.p[3], a.n[3], q.w, y, (k == row + 3) ? th[3] : 0.0f);
}
template <int U, bool NTL>
__device__ __forceinline__ void stream_load(float4 (&q)[U], const float* __restrict__ src, int ldq) {
#pragma unroll
    for (int j = 0; j < U; ++j) q[j] = ldq4<NTL>(src + (size_t)j * ldq);
}
template <int U>
__device__ __forceinline__ void block_load(float4 (&q)[U], const float* __restrict__ src, int ldq, bool keep) {
    if (keep)
        stream_load<U, false>(q, src, ldq);
    else
        stream_load<U, true>(q, src, ldq);
}
// the same block through a buffer descriptor: one VGPR offset (the lane's
// rows) for all U loads, the k offset in SGPRs (aux 2 = nt)
template <int U>
__device__ __forceinline__ void block_load_buf(float4 (&q)[U], __amdgpu_buffer_rsrc_t rs, int voff, int kb, int ldq,
                                               bool keep) {
    const int s0 = kb * U * ldq * 4;
    if (keep) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, s0 + j * ldq * 4, 0);
            q[j] = make_float4(v.x, v.y, v.z, v.w);
        }
    } else {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, s0 + j * ldq * 4, 2);
            q[j] = make_float4(v.x, v.y, v.z, v.w);
        }
    }
}
template <int U>
__device__ __forceinline__ void stream_block(Acc4& a, const float4 (&q)[U], int k0, bool literal,
                                             const float* __restrict__ y, int row, const float th[4]) {
    if (literal) {
#pragma unroll
        for (int j = 0; j < U; j += 4) {
            const float4 yv = *reinterpret_cast<const float4*>(y + k0 + j);
            literal4(a, q[j + 0], yv.x, k0 + j + 0, row, th);
            literal4(a, q[j + 1], yv.y, k0 + j + 1, row, th);
            literal4(a, q[j + 2], yv.z, k0 + j + 2, row, th);
            literal4(a, q[j + 3], yv.w, k0 + j + 3, row, th);
        }
    } else {
#pragma unroll
        for (int j = 0; j < U; j += 4) {
            const float4 yv = *reinterpret_cast<const float4*>(y + k0 + j);
            lean4(a, q[j + 0], yv.x);
            lean4(a, q[j + 1], yv.y);
            lean4(a, q[j + 2], yv.z);
            lean4(a, q[j + 3], yv.w);
        }
    }
}

// N == 1024 (one row pass: 256 lanes x 4 rows).  Blocks 0..P-1 (P = RA + RL)
// are resident: in iteration 0 they are loaded from HBM (all RA register
// blocks at once, the LDS blocks one at a time through qb) and summed from
// their resident copy; from iteration 1 on they are summed from the copy while
// block P -- the first streamed block, prefetched at the end of the previous
// iteration -- is in flight.  Blocks P..63 stream as in k_batch_stream; the
// first R of them with default-policy loads.
template <int U, int RA, int RL, bool BUF>
__global__ void __launch_bounds__(256) k_stream_res(const float* __restrict__ QdT, long long qstride, int ldq,
                                                    const float* __restrict__ theta, const float* __restrict__ Fd,
                                                    int ldv, float* Y, int updates, int R) {
    constexpr int N = 1024, P = RA + RL, nb = N / U;
    static_assert((nb - P) % 2 == 0, "streamed blocks come in pairs");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* ya = lds;
    float* yb = lds + ldq;
    float4* res = reinterpret_cast<float4*>(lds + 2 * ldq);  // [RL][U][256]
    const int b = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6;
    const float* Q = QdT + (size_t)b * (size_t)qstride;
    const float* th_g = theta + (size_t)b * ldv;
    const float* fd_g = Fd + (size_t)b * ldv;
    for (int i = tid; i < ldq; i += 256) {
        ya[i] = (i < N) ? 1000.0f : 0.0f;
        yb[i] = 0.0f;
    }
    const int row = 4 * tid;
    const int wa = 256 * wave, wbd = wa + 256;
    const float* col = Q + row;
    float th[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) th[r] = th_g[row + r];
    float4 qa[U], qb[U];
    float4 rr[RA > 0 ? RA * U : 1];
    const unsigned long long qaddr = (unsigned long long)Q;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(qaddr >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)qaddr)),
        (short)0, __builtin_amdgcn_readfirstlane((int)(qstride * 4)), 0x00020000);
    auto ld = [&](float4(&q)[U], int kb, bool keep) {
        if constexpr (BUF)
            block_load_buf<U>(q, rs, 16 * tid, kb, ldq, keep);
        else
            block_load<U>(q, col + (size_t)kb * U * ldq, ldq, keep);
    };
    // iteration 0's resident register blocks, and the first streamed block
    if constexpr (RA > 0) {
#pragma unroll
        for (int j = 0; j < RA * U; ++j) rr[j] = ldq4<true>(col + (size_t)j * ldq);
    }
    if (updates > 0) ld(qa, P, 0 < R);
    __syncthreads();
    for (int u = 0; u < updates; ++u) {
        const float* cur = (u & 1) ? yb : ya;
        float* nxt = (u & 1) ? ya : yb;
        // the register blocks are pinned to AGPRs at the top of each iteration
        // (an "a" constraint): left to itself the compiler keeps them in the
        // arch VGPRs the stream needs and spills to scratch (2 blocks: 532 B)
        if constexpr (RA > 0) {
#pragma unroll
            for (int j = 0; j < RA * U; ++j) {
                asm volatile("" : "+a"(rr[j].x));
                asm volatile("" : "+a"(rr[j].y));
                asm volatile("" : "+a"(rr[j].z));
                asm volatile("" : "+a"(rr[j].w));
            }
        }
        Acc4 a;
#pragma unroll
        for (int r = 0; r < 4; ++r) a.p[r] = a.n[r] = 0.0f;
        // resident blocks: registers first, then LDS
        if constexpr (RA > 0) {
#pragma unroll
            for (int rb = 0; rb < RA; ++rb) {
                float4 q[U];
#pragma unroll
                for (int j = 0; j < U; ++j) q[j] = rr[rb * U + j];
                const int k0 = rb * U;
                stream_block<U>(a, q, k0, k0 >= wa && k0 < wbd, cur, row, th);
            }
        }
        if constexpr (RL > 0) {
#pragma unroll
            for (int lb = 0; lb < RL; ++lb) {
                float4* slot = res + (size_t)lb * U * 256 + tid;
                if (u == 0) {
                    ld(qb, RA + lb, false);
#pragma unroll
                    for (int j = 0; j < U; ++j) slot[j * 256] = qb[j];
                } else {
#pragma unroll
                    for (int j = 0; j < U; ++j) qb[j] = slot[j * 256];
                }
                const int k0 = (RA + lb) * U;
                stream_block<U>(a, qb, k0, k0 >= wa && k0 < wbd, cur, row, th);
            }
        }
        for (int kb = P; kb < nb; kb += 2) {
            ld(qb, kb + 1, kb + 1 - P < R);
            int k0 = kb * U;
            stream_block<U>(a, qa, k0, k0 >= wa && k0 < wbd, cur, row, th);
            if (kb + 2 < nb)
                ld(qa, kb + 2, kb + 2 - P < R);
            else if (u + 1 < updates)
                ld(qa, P, 0 < R);
            k0 += U;
            stream_block<U>(a, qb, k0, k0 >= wa && k0 < wbd, cur, row, th);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = row + r;
            const float f = fd_g[i];
            const float num = a.n[r] + 1.0f * max_ref(0.0f, -f);
            const float den = a.p[r] + 1.0f * max_ref(0.0f, f);
            nxt[i] = num / den * cur[i];
        }
        __syncthreads();
    }
    const float* fin = (updates & 1) ? yb : ya;
    for (int i = tid; i < N; i += 256) Y[(size_t)b * ldv + i] = fin[i];
}

__global__ void k_fill(float* q, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        q[i] = ((int)(x % 2001u) - 1000) * 1e-3f;  // [-1, 1], zeros included
    }
}

struct Variant {
    const char* name;
    void (*launch)(int B, const float*, long long, int, const float*, const float*, int, float*, int, int, hipStream_t);
    int RA, RL;
};

template <int RA, int RL, bool BUF>
void launch(int B, const float* Q, long long qs, int ldq, const float* th, const float* fd, int ldv, float* Y,
            int updates, int R, hipStream_t s) {
    const size_t lds = (size_t)2 * ldq * 4 + (size_t)RL * 16 * 256 * 16;
    static bool attr = false;
    if (!attr) {
        CK(hipFuncSetAttribute((const void*)k_stream_res<16, RA, RL, BUF>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
        attr = true;
    }
    hipLaunchKernelGGL((k_stream_res<16, RA, RL, BUF>), dim3(B), dim3(256), lds, s, Q, qs, ldq, th, fd, ldv, Y, updates, R);
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 4096;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const int N = 1024, ldq = 1024, ldv = 1024, C = 10;
    const long long qs = (long long)N * ldq;
    float *Q, *th, *fd, *Y;
    CK(hipMalloc(&Q, (size_t)B * qs * 4));
    CK(hipMalloc(&th, (size_t)B * ldv * 4));
    CK(hipMalloc(&fd, (size_t)B * ldv * 4));
    CK(hipMalloc(&Y, (size_t)B * ldv * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, Q, (size_t)B * qs, 1u);
    hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, fd, (size_t)B * ldv, 7u);
    std::vector<float> h(B * (size_t)ldv, 5.0f);
    CK(hipMemcpy(th, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    const Variant vs[] = {
        {"base", launch<0, 0, false>, 0, 0},         {"lds2", launch<0, 2, false>, 0, 2},
        {"buf_lds2", launch<0, 2, true>, 0, 2},      {"buf_reg2lds2", launch<2, 2, true>, 2, 2},
        {"buf_reg2", launch<2, 0, true>, 2, 0},
    };
    const int Rs[] = {0, 1, 2};
    std::vector<float> ref(h.size()), got(h.size());
    bool have_ref = false;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double alg = (4.0 * N * N + 16.0 * N) * B * C;
    for (int round = 0; round < 2; ++round) {
        for (const Variant& v : vs) {
            for (int R : Rs) {

                v.launch(B, Q, qs, ldq, th, fd, ldv, Y, C, R, 0);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(got.data(), Y, got.size() * 4, hipMemcpyDeviceToHost));
                if (!have_ref) {
                    ref = got;
                    have_ref = true;
                }
                const bool same = memcmp(ref.data(), got.data(), got.size() * 4) == 0;
                CK(hipEventRecord(e0, 0));
                for (int r = 0; r < reps; ++r) v.launch(B, Q, qs, ldq, th, fd, ldv, Y, C, R, 0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                ms /= reps;
                printf("{\"variant\": \"%s\", \"RA\": %d, \"RL\": %d, \"R\": %d, \"ms_per_launch\": %.3f, "
                       "\"alg_TBps\": %.3f, \"same_bits\": %s}\n",
                       v.name, v.RA, v.RL, R, ms, alg / (ms * 1e-3) / 1e12, same ? "true" : "false");
                fflush(stdout);
            }
        }
    }
    return 0;
}
