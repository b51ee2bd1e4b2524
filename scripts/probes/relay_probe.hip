// Probe: in-kernel timeline of the relay update (k_split_relay's structure)
// for one n_dual = 1024 problem: s_memtime stamps per wave and segment.
// Build: hipcc --offload-arch=gfx950 -O3 relay_probe.hip -o relay_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#pragma clang fp contract(off)
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int W = 8;

// EARLY: 0 = every wave loads its first segment before y is staged (shipped);
//        1 = y loads first, wave 0 loads its segment before the barrier, the
//            other waves after it
// BATCH: products read y for 4 packets before multiplying (vs one at a time)
template <int S, int EARLY, int BATCH, int NOSTAGE = 0>
__global__ void __launch_bounds__(64 * W) k_relay(const float* __restrict__ SP, int N, int lw, const float* __restrict__ Yin,
                                                  float* __restrict__ Yout, unsigned long long* stamps) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    unsigned long long* slot = reinterpret_cast<unsigned long long*>(lds);
    float* ys = lds + 128;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const int KB = (N + 3) / 4;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ll = lane % lw;
    const int G = (KB + S - 1) / S;
    const float* region = SP + (size_t)blockIdx.x * KB * lw * 4;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(region), (short)0, KB * lw * 16, 0x00020000);
    const int vo = ll * 16, kstride = lw * 16;
    f4v q[S];
    auto load_seg = [&](int g) {
        const int nj = KB - g * S;
#pragma unroll
        for (int j = 0; j < S; ++j)
            q[j] = (j < nj && lane < lw) ? __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (g * S + j) * kstride, 0)
                                         : f4v{0, 0, 0, 0};
    };
    if (NOSTAGE) {
        // no y in LDS: every wave reads its own segment's y with uniform
        // (scalar) loads; only the hand-off words are initialised first
        if (w == 0) slot[lane] = 0ull;
        __syncthreads();
        if (w < G) load_seg(w);
    }
    if (!NOSTAGE && !EARLY && w < G) load_seg(w);
    if (!NOSTAGE) {
        const int t = threadIdx.x, n_lds = 4 * G * S;
        for (int b = 0; b < n_lds; b += 64 * W * 8) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = b + 64 * W * j + t;
                v[j] = (k < N) ? Yin[k] : 0.0f;
            }
            if (EARLY && b == 0 && w == 0 && G > 0) load_seg(0);  // after the y loads: vmcnt waits for y only
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = b + 64 * W * j + t;
                if (k < n_lds) ys[k] = v[j];
            }
        }
        if (w == 0) slot[lane] = 0ull;
        __syncthreads();
    }
    if (!NOSTAGE && EARLY && w > 0 && w < G) load_seg(w);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long* my = stamps + ((size_t)blockIdx.x * W + w) * 64;  // [0] t0 [1] t1 then 4 per round
    if (lane == 0) {
        my[0] = t0;
        my[1] = t1;
    }
    float acc = 0.0f;
    int round = 0;
    for (int g = w; g < G; g += W, ++round) {
        const unsigned long long ta = __builtin_amdgcn_s_memtime();
        if (BATCH) {
            const float* ysrc = NOSTAGE ? Yin : ys;
            const int nk = N - g * S * 4;  // wave-uniform: y past N is 0 (NOSTAGE reads Yin directly)
#pragma unroll
            for (int j0 = 0; j0 < S; j0 += 4) {
                f4v y[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (NOSTAGE) {
                        const int k = (j0 + u) * 4;
                        y[u] = f4v{k < nk ? ysrc[g * S * 4 + k] : 0.0f, k + 1 < nk ? ysrc[g * S * 4 + k + 1] : 0.0f,
                                   k + 2 < nk ? ysrc[g * S * 4 + k + 2] : 0.0f, k + 3 < nk ? ysrc[g * S * 4 + k + 3] : 0.0f};
                    } else {
                        y[u] = *reinterpret_cast<const f4v*>(ys + 4 * (g * S + j0 + u));
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int j = j0 + u;
                    f2v lo = f2v{q[j].x, q[j].y} * f2v{y[u].x, y[u].y};
                    f2v hi = f2v{q[j].z, q[j].w} * f2v{y[u].z, y[u].w};
                    q[j] = f4v{lo.x, lo.y, hi.x, hi.y};
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) asm volatile("" : "+v"(q[j0 + u]));
            }
        } else {
#pragma unroll
            for (int j = 0; j < S; ++j) {
                const f4v y = *reinterpret_cast<const f4v*>(ys + 4 * (g * S + j));
                f2v lo = f2v{q[j].x, q[j].y} * f2v{y.x, y.y};
                f2v hi = f2v{q[j].z, q[j].w} * f2v{y.z, y.w};
                q[j] = f4v{lo.x, lo.y, hi.x, hi.y};
                asm volatile("" : "+v"(q[j]));
            }
        }
        const unsigned long long tb = __builtin_amdgcn_s_memtime();
        unsigned long long h;
        for (int spin = 0;; ++spin) {
            h = __hip_atomic_load(slot + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (__all((int)(h >> 32) == g) || spin > (1 << 20)) break;
        }
        const unsigned long long tc = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_setprio(3);
        acc = __uint_as_float((unsigned)h);
#pragma unroll
        for (int j = 0; j < S; ++j) {
            acc += q[j].x;
            acc += q[j].y;
            acc += q[j].z;
            acc += q[j].w;
        }
        __hip_atomic_store(slot + lane, ((unsigned long long)(g + 1) << 32) | __float_as_uint(acc), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_s_setprio(0);
        const unsigned long long td = __builtin_amdgcn_s_memtime();
        if (lane == 0 && round < 14) {
            my[2 + 4 * round] = ta;
            my[3 + 4 * round] = tb;
            my[4 + 4 * round] = tc;
            my[5 + 4 * round] = td;
        }
        if (g + W < G) load_seg(g + W);
    }
    if (w == (G - 1) % W) {
        const float v = acc;
        const float den = __shfl_xor(v, 1);
        const int p = blockIdx.x * lw + ll;
        if (!(p & 1) && lane < lw && p < 2 * N) Yout[p >> 1] = v / den * Yin[p >> 1];
    }
    if (lane == 0 && w == 0) stamps[(size_t)gridDim.x * W * 64 + blockIdx.x] = __builtin_amdgcn_s_memtime();
}

template <int S, int EARLY, int BATCH, int NOSTAGE = 0>
void run(const char* name, int lw) {
    const int N = 1024, KB = N / 4;
    const int wgs = 2 * N / lw;
    const size_t nsp = (size_t)wgs * KB * lw * 4;
    std::vector<float> h(nsp);
    for (size_t i = 0; i < nsp; ++i) h[i] = 0.001f * (float)((i * 2654435761u) % 1000);
    float *SP, *Y, *Yo;
    unsigned long long* st;
    (void)hipMalloc(&SP, nsp * 4);
    (void)hipMemcpy(SP, h.data(), nsp * 4, hipMemcpyHostToDevice);
    (void)hipMalloc(&Y, N * 4);
    (void)hipMalloc(&Yo, N * 4);
    std::vector<float> y(N, 1000.0f);
    (void)hipMemcpy(Y, y.data(), N * 4, hipMemcpyHostToDevice);
    const size_t nst = (size_t)wgs * W * 64 + wgs;
    (void)hipMalloc(&st, nst * 8);
    (void)hipMemset(st, 0, nst * 8);
    const int G = (KB + S - 1) / S;
    const size_t lds = sizeof(float) * (4 * G * S + 128);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL((k_relay<S, EARLY, BATCH, NOSTAGE>), dim3(wgs), dim3(64 * W), lds, 0, SP, N, lw, Y, Yo, st);
    (void)hipEventRecord(e0);
    for (int rep = 0; rep < 200; ++rep)  // alternate y buffers like the real update
        hipLaunchKernelGGL((k_relay<S, EARLY, BATCH, NOSTAGE>), dim3(wgs), dim3(64 * W), lds, 0, SP, N, lw, (rep & 1) ? Yo : Y,
                           (rep & 1) ? Y : Yo, st);
    (void)hipEventRecord(e1);
    (void)hipDeviceSynchronize();
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> hs(nst);
    (void)hipMemcpy(hs.data(), st, nst * 8, hipMemcpyDeviceToHost);
    unsigned long long base = ~0ull, staged = 0, first_turn = 0, last_done = 0, prod0 = 0;
    for (int w = 0; w < W; ++w) base = std::min(base, hs[(size_t)w * 64]);
    for (int w = 0; w < W; ++w) {
        const unsigned long long* m = &hs[(size_t)w * 64];
        staged = std::max(staged, m[1] - base);
        for (int r = 0; r < 14; ++r)
            if (m[5 + 4 * r]) last_done = std::max(last_done, m[5 + 4 * r] - base);
    }
    prod0 = hs[3] - hs[2];
    first_turn = hs[4] - base;
    printf("{\"variant\": \"%s\", \"lw\": %d, \"us_per_launch\": %.3f, \"staged\": %llu, \"seg0_products\": %llu, "
           "\"first_turn\": %llu, \"last_done\": %llu}\n",
           name, lw, ms * 1e3 / 200, staged, prod0, first_turn, last_done);
    (void)hipFree(SP);
    (void)hipFree(Y);
    (void)hipFree(Yo);
    (void)hipFree(st);
}

int main() {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    for (int lw : {64, 8}) {
        run<16, 0, 0>("S16 shipped", lw);
        run<16, 0, 1>("S16 batch", lw);
        run<16, 0, 1, 1>("S16 batch nostage", lw);
        run<32, 0, 1, 1>("S32 batch nostage", lw);
        run<8, 0, 1, 1>("S8 batch nostage", lw);
    }
    return 0;
}
