// pqp_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the PQP dual update.
//
// Hot path: the reference's updateY2
// (PQP_CPU.c:603-618) is two N x N mat-vecs over the stored split matrices
//   num = (max(0,-Qd)+Theta) Y + max(0,-Fd)      den = (max(0,Qd)+Theta) Y + max(0,Fd)
//   Y_next[i] = num[i] / den[i] * Y[i]                                  (updY, :590-596)
// Here one pass streams Qd ONCE (4 N^2 bytes instead of 8 N^2), derives both
// split entries in registers, and applies the update in the epilogue.
//
// Bit-exactness with PQP_CPU.c: every row keeps the reference's sequential
// k = 0..N-1 fp32 accumulation (one lane owns a row, no reduction tree), each
// product is rounded before it is added (-ffp-contract=off), and the
// +0.0/Theta additions of the stored matrices are reproduced literally inside
// the diagonal window.  Off the diagonal the "lean" form is used:
//   den += (q < 0) ? 0*y : q*y ;   num += (q > 0) ? 0*y : -(q*y)
// which is bit-identical to (max(0,+-q) + 0.0f) * y for every q (incl. +-0,
// NaN) and every y (incl. inf/NaN): see DESIGN.md "Lean form".
//
// Layout: Qd is stored column-major per problem (QdT, element (i,k) at
// k*ldq + i) so that at a fixed k a wave's 64 lanes x 4 rows read 1 KiB of
// contiguous HBM with one global_load_dwordx4 each (fully coalesced), while
// y[k] is a wave-uniform LDS broadcast.
#include <atomic>
#include <type_traits>

#include "pqp_device.h"
#include "pqp_launch.h"

namespace pqp {

static inline unsigned cdiv(long long a, long long b) { return (unsigned)((a + b - 1) / b); }
static bool aligned16(const void* p);

// <hot-kernel> (bench.py hashes the text up to </hot-kernel>: PMC traffic records are keyed by it)
// ---------------------------------------------------------------------------
// Row-update building blocks
// ---------------------------------------------------------------------------
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
// streamed-once Qd: optionally non-temporal (global_load_dwordx4 ... nt)
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
    float p[4];  // den accumulators (Qd+ side)
    float n[4];  // num accumulators (Qd- side)
};

// lean step for one k and this lane's 4 rows (off-diagonal entries only)
__device__ __forceinline__ void lean4(Acc4& a, float4 q, float y) {
    const float z = 0.0f * y;  // (+0)*y: +0 for finite y >= 0, NaN for inf/NaN y
    float p;
    p = q.x * y; a.p[0] += (q.x < 0.0f) ? z : p; a.n[0] += (q.x > 0.0f) ? z : -p;
    p = q.y * y; a.p[1] += (q.y < 0.0f) ? z : p; a.n[1] += (q.y > 0.0f) ? z : -p;
    p = q.z * y; a.p[2] += (q.z < 0.0f) ? z : p; a.n[2] += (q.z > 0.0f) ? z : -p;
    p = q.w * y; a.p[3] += (q.w < 0.0f) ? z : p; a.n[3] += (q.w > 0.0f) ? z : -p;
}

// literal step: (max(0,+-q) + (k==i ? theta_i : +0)) * y, PQP_CPU.c:524-537 + :608-609
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

// Stream k in [ka, kb) with the lean form.  ka % 4 == 0.  `col` points at
// QdT + row (this lane's 4 rows), y is the iterate (LDS).
template <int U, bool NTL>
__device__ __forceinline__ void lean_segment(Acc4& a, const float* __restrict__ col, int ldq, int ka, int kb,
                                             const float* __restrict__ y) {
    static_assert(U % 4 == 0, "unroll must be a multiple of 4 (one float4 of y per 4 k)");
    int k = ka;
    const float* src = col + (size_t)k * ldq;
    for (; k + U <= kb; k += U) {
        float4 q[U];
#pragma unroll
        for (int j = 0; j < U; ++j) q[j] = ldq4<NTL>(src + (size_t)j * ldq);
        src += (size_t)U * ldq;
#pragma unroll
        for (int j = 0; j < U; j += 4) {
            const float4 yv = *reinterpret_cast<const float4*>(y + k + j);
            lean4(a, q[j + 0], yv.x);
            lean4(a, q[j + 1], yv.y);
            lean4(a, q[j + 2], yv.z);
            lean4(a, q[j + 3], yv.w);
        }
    }
    for (; k < kb; ++k) {
        lean4(a, ldq4<NTL>(src), y[k]);
        src += ldq;
    }
}

template <bool NTL>
__device__ __forceinline__ void literal_segment(Acc4& a, const float* __restrict__ col, int ldq, int ka, int kb,
                                                const float* __restrict__ y, int row, const float th[4]) {
    int k = ka;
    const float* src = col + (size_t)k * ldq;
    for (; k + 4 <= kb; k += 4) {
        float4 q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = ldq4<NTL>(src + (size_t)j * ldq);
        src += (size_t)4 * ldq;
        const float4 y0 = *reinterpret_cast<const float4*>(y + k);
        literal4(a, q[0], y0.x, k + 0, row, th);
        literal4(a, q[1], y0.y, k + 1, row, th);
        literal4(a, q[2], y0.z, k + 2, row, th);
        literal4(a, q[3], y0.w, k + 3, row, th);
    }
    for (; k < kb; ++k) {
        literal4(a, ldq4<NTL>(src), y[k], k, row, th);
        src += ldq;
    }
}

// One lane: num/den for rows [row,row+4) of one problem, then
// out[i] = num/den * y[i] for the rows < N.  w0 = first row of this lane's
// wave (wave-uniform): the diagonal of the wave's 256 rows lies in
// k in [w0, w0+256) and only that window needs the literal form.
template <int U, bool NTL, typename OutPtr>
__device__ __forceinline__ void update_rows4(const float* __restrict__ Q, int ldq, int N, int row, int w0,
                                             const float* __restrict__ th_g, const float* __restrict__ fd_g,
                                             const float* __restrict__ y, OutPtr out) {
    Acc4 a;
#pragma unroll
    for (int r = 0; r < 4; ++r) a.p[r] = a.n[r] = 0.0f;
    float th[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) th[r] = (row + r < N) ? th_g[row + r] : 0.0f;
    const float* col = Q + row;
    const int wa = w0 < N ? w0 : N;
    const int wb = (w0 + 256) < N ? (w0 + 256) : N;
    lean_segment<U, NTL>(a, col, ldq, 0, wa, y);
    literal_segment<NTL>(a, col, ldq, wa, wb, y, row, th);
    lean_segment<U, NTL>(a, col, ldq, wb, N, y);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = row + r;
        if (i < N) {
            const float f = fd_g[i];
            const float num = a.n[r] + 1.0f * max_ref(0.0f, -f);  // matrixAdd(num, Fdn, 1) :611
            const float den = a.p[r] + 1.0f * max_ref(0.0f, f);   // matrixAdd(den, Fdp, 1) :612
            out[i] = num / den * y[i];                            // updY :594
        }
    }
}

// ---------------------------------------------------------------------------
// k_batch_iterate: `updates` fixed-mode iterations of every problem in ONE
// launch.  One workgroup owns one problem; its iterate ping-pongs between two
// LDS buffers, so the only HBM traffic per iteration is Qd (streamed once).
// ---------------------------------------------------------------------------
template <int NT, int U = 8, bool NTL = false>
__global__ void __launch_bounds__(NT) k_batch_iterate(const float* __restrict__ QdT, long long qstride, int ldq,
                                                      int N, const float* __restrict__ theta,
                                                      const float* __restrict__ Fd, int ldv,
                                                      const float* Y0, float* Y, int updates) {
    // Y0 may alias Y (chained launches): each workgroup reads its problem's
    // Y0 into LDS before the loop and writes Y only after it
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* ya = lds;
    float* yb = lds + ldq;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const float* Q = QdT + (size_t)b * (size_t)qstride;
    const float* th = theta + (size_t)b * ldv;
    const float* fd = Fd + (size_t)b * ldv;
    for (int i = tid; i < ldq; i += NT) {
        ya[i] = (i < N) ? (Y0 ? Y0[(size_t)b * ldv + i] : 1000.0f) : 0.0f;  // initMat(Y,1000) :710
        yb[i] = 0.0f;
    }
    __syncthreads();
    const int wave = tid >> 6;
    for (int u = 0; u < updates; ++u) {
        float* cur = (u & 1) ? yb : ya;
        float* nxt = (u & 1) ? ya : yb;
        for (int r0 = 0; r0 < N; r0 += 4 * NT) {
            const int row = r0 + 4 * tid;
            const int w0 = r0 + 256 * wave;
            if (row < N) update_rows4<U, NTL, float*>(Q, ldq, N, row, w0, th, fd, cur, nxt);
        }
        __syncthreads();
    }
    const float* fin = (updates & 1) ? yb : ya;
    for (int i = tid; i < N; i += NT) Y[(size_t)b * ldv + i] = fin[i];
}

// ---------------------------------------------------------------------------
// k_batch_stream: k_batch_iterate's arithmetic (the same lean / literal terms
// in the same k order per row) with Qd's loads kept in flight continuously:
// two register buffers of U float4 per lane, the block b + 1 loaded while
// block b is summed, and the next row pass's (or the next iteration's) first
// block loaded before the pass ends -- Qd does not depend on y, so only the
// sums wait at the iteration's barrier.  N % 1024 == 0 (256 lanes x 4 rows
// per pass, whole blocks of U k, block-aligned diagonal windows).
// ---------------------------------------------------------------------------
template <int U, bool NTL>
__device__ __forceinline__ void stream_load(float4 (&q)[U], const float* __restrict__ src, int ldq) {
#pragma unroll
    for (int j = 0; j < U; ++j) q[j] = ldq4<NTL>(src + (size_t)j * ldq);
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
template <int U, bool NTL>
__global__ void __launch_bounds__(256) k_batch_stream(const float* __restrict__ QdT, long long qstride, int ldq,
                                                      int N, const float* __restrict__ theta,
                                                      const float* __restrict__ Fd, int ldv,
                                                      const float* Y0, float* Y, int updates) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* ya = lds;
    float* yb = lds + ldq;
    const int b = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6;
    const float* Q = QdT + (size_t)b * (size_t)qstride;
    const float* th_g = theta + (size_t)b * ldv;
    const float* fd_g = Fd + (size_t)b * ldv;
    for (int i = tid; i < ldq; i += 256) {
        ya[i] = (i < N) ? (Y0 ? Y0[(size_t)b * ldv + i] : 1000.0f) : 0.0f;  // initMat(Y,1000) :710
        yb[i] = 0.0f;
    }
    const int nb = N / U, npass = N / 1024;
    float4 qa[U], qb[U];
    if (updates > 0) stream_load<U, NTL>(qa, Q + 4 * tid, ldq);
    __syncthreads();
    for (int u = 0; u < updates; ++u) {
        const float* cur = (u & 1) ? yb : ya;
        float* nxt = (u & 1) ? ya : yb;
        for (int pass = 0; pass < npass; ++pass) {
            const int row = pass * 1024 + 4 * tid;
            const int wa = pass * 1024 + 256 * wave, wbd = wa + 256;  // this wave's diagonal window
            Acc4 a;
#pragma unroll
            for (int r = 0; r < 4; ++r) a.p[r] = a.n[r] = 0.0f;
            float th[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) th[r] = th_g[row + r];
            const float* col = Q + row;
            for (int kb = 0; kb < nb; kb += 2) {
                stream_load<U, NTL>(qb, col + (size_t)(kb + 1) * U * ldq, ldq);
                int k0 = kb * U;
                stream_block<U>(a, qa, k0, k0 >= wa && k0 < wbd, cur, row, th);
                // one block ahead: this pass's next, else the next pass's (or
                // the next iteration's) first
                if (kb + 2 < nb) stream_load<U, NTL>(qa, col + (size_t)(kb + 2) * U * ldq, ldq);
                else if (pass + 1 < npass) stream_load<U, NTL>(qa, Q + (pass + 1) * 1024 + 4 * tid, ldq);
                else if (u + 1 < updates) stream_load<U, NTL>(qa, Q + 4 * tid, ldq);
                k0 += U;
                stream_block<U>(a, qb, k0, k0 >= wa && k0 < wbd, cur, row, th);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = row + r;
                const float f = fd_g[i];
                const float num = a.n[r] + 1.0f * max_ref(0.0f, -f);  // matrixAdd(num, Fdn, 1) :611
                const float den = a.p[r] + 1.0f * max_ref(0.0f, f);   // matrixAdd(den, Fdp, 1) :612
                nxt[i] = num / den * cur[i];                           // updY :594
            }
        }
        __syncthreads();
    }
    const float* fin = (updates & 1) ? yb : ya;
    for (int i = tid; i < N; i += 256) Y[(size_t)b * ldv + i] = fin[i];
}

// ---------------------------------------------------------------------------
// k_batch_resident (n_dual 1024, the bench shape): k_batch_stream with part of
// each problem's Qd kept on the CU across the launch's iterations (temporal
// blocking; one workgroup per CU, so the CU's LDS and registers are this
// problem's):
//   blocks 0 .. RA-1 (U k each, 64 KiB per block over the workgroup) in
//     registers: loaded from HBM in the first iteration and pinned to AGPRs
//     (the stream buffers take the arch VGPRs);
//   blocks RA .. P-1 (P = RA + RL) copied into LDS in the first iteration and
//     summed from there afterwards;
//   block P -- the first streamed block, loaded at the end of each iteration
//     for the next one while the resident blocks are summed -- uses the
//     default cache policy: 64 KiB per CU = 2 MiB per XCD, which stays in the
//     XCD's L2 between iterations while the nt stream passes through;
//   blocks P+1 .. 63 stream non-temporally as in k_batch_stream.
// RA > 0 reads Qd through a buffer descriptor (one VGPR offset for all U loads
// of a block, the k offset in SGPRs): the 64-bit per-load addresses of the
// global form leave no room for the pinned blocks.  Every row sums the same
// terms in the same k order as k_batch_stream (only where q comes from
// differs), so the bits are the same.
// ---------------------------------------------------------------------------
template <int U, int RL, int RA = 0>
__global__ void __launch_bounds__(256) k_batch_resident(const float* __restrict__ QdT, long long qstride, int ldq,
                                                        const float* __restrict__ theta,
                                                        const float* __restrict__ Fd, int ldv, const float* Y0,
                                                        float* Y, int updates) {
    constexpr int N = 1024, nb = N / U, P = RA + RL;
    static_assert((nb - P) % 2 == 0, "the streamed blocks come in pairs");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* ya = lds;
    float* yb = lds + ldq;
    float4* res = reinterpret_cast<float4*>(lds + 2 * ldq);  // [RL][U][256 lanes]
    const int b = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6;
    const float* Q = QdT + (size_t)b * (size_t)qstride;
    const float* th_g = theta + (size_t)b * ldv;
    const float* fd_g = Fd + (size_t)b * ldv;
    for (int i = tid; i < ldq; i += 256) {
        ya[i] = (i < N) ? (Y0 ? Y0[(size_t)b * ldv + i] : 1000.0f) : 0.0f;  // initMat(Y,1000) :710
        yb[i] = 0.0f;
    }
    const int row = 4 * tid;
    const int wa = 256 * wave, wbd = wa + 256;  // this wave's diagonal window
    const float* col = Q + row;
    float th[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) th[r] = th_g[row + r];
    // block kb's U float4 of this lane (nt: non-temporal)
    const unsigned long long qaddr = (unsigned long long)Q;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(qaddr >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)qaddr)),
        (short)0, __builtin_amdgcn_readfirstlane((int)(qstride * 4)), 0x00020000);
    auto ld = [&](float4(&q)[U], int kb, bool nt) {
        if constexpr (RA > 0) {
            const int s0 = kb * U * ldq * 4;
            if (nt) {
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * tid, s0 + j * ldq * 4, 2);
                    q[j] = make_float4(v.x, v.y, v.z, v.w);
                }
            } else {
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * tid, s0 + j * ldq * 4, 0);
                    q[j] = make_float4(v.x, v.y, v.z, v.w);
                }
            }
        } else {
            if (nt) stream_load<U, true>(q, col + (size_t)kb * U * ldq, ldq);
            else stream_load<U, false>(q, col + (size_t)kb * U * ldq, ldq);
        }
    };
    float4 qa[U], qb[U];
    float4 rr[RA > 0 ? RA * U : 1];
    if (updates > 0) {
#pragma unroll
        for (int rb = 0; rb < RA; ++rb) {
            float4 t[U];
            ld(t, rb, true);
#pragma unroll
            for (int j = 0; j < U; ++j) rr[rb * U + j] = t[j];
        }
        ld(qa, P, false);
    }
    __syncthreads();
    for (int u = 0; u < updates; ++u) {
        const float* cur = (u & 1) ? yb : ya;
        float* nxt = (u & 1) ? ya : yb;
        // the register blocks pinned to AGPRs here (an "a" constraint): left to
        // itself the compiler keeps them in the arch VGPRs the stream needs and
        // spills to scratch (scripts/probes/stream_resident.hip)
#pragma unroll
        for (int j = 0; j < RA * U; ++j) {
            asm volatile("" : "+a"(rr[j].x));
            asm volatile("" : "+a"(rr[j].y));
            asm volatile("" : "+a"(rr[j].z));
            asm volatile("" : "+a"(rr[j].w));
        }
        Acc4 a;
#pragma unroll
        for (int r = 0; r < 4; ++r) a.p[r] = a.n[r] = 0.0f;
#pragma unroll
        for (int rb = 0; rb < RA; ++rb) {
            float4 q[U];
#pragma unroll
            for (int j = 0; j < U; ++j) q[j] = rr[rb * U + j];
            const int k0 = rb * U;
            stream_block<U>(a, q, k0, k0 >= wa && k0 < wbd, cur, row, th);
        }
#pragma unroll
        for (int lb = 0; lb < RL; ++lb) {
            float4* slot = res + (size_t)lb * U * 256 + tid;  // lane-private: no barrier needed
            if (u == 0) {
                ld(qb, RA + lb, true);
#pragma unroll
                for (int j = 0; j < U; ++j) slot[j * 256] = qb[j];
            } else {
#pragma unroll
                for (int j = 0; j < U; ++j) qb[j] = slot[j * 256];
            }
            const int k0 = (RA + lb) * U;
            stream_block<U>(a, qb, k0, k0 >= wa && k0 < wbd, cur, row, th);
        }
        for (int kb = P; kb < nb; kb += 2) {
            ld(qb, kb + 1, true);
            int k0 = kb * U;
            stream_block<U>(a, qa, k0, k0 >= wa && k0 < wbd, cur, row, th);
            if (kb + 2 < nb)
                ld(qa, kb + 2, true);
            else if (u + 1 < updates)  // the next iteration's first streamed block (L2-kept)
                ld(qa, P, false);
            k0 += U;
            stream_block<U>(a, qb, k0, k0 >= wa && k0 < wbd, cur, row, th);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = row + r;
            const float f = fd_g[i];
            const float num = a.n[r] + 1.0f * max_ref(0.0f, -f);  // matrixAdd(num, Fdn, 1) :611
            const float den = a.p[r] + 1.0f * max_ref(0.0f, f);   // matrixAdd(den, Fdp, 1) :612
            nxt[i] = num / den * cur[i];                           // updY :594
        }
        __syncthreads();
    }
    const float* fin = (updates & 1) ? yb : ya;
    for (int i = tid; i < N; i += 256) Y[(size_t)b * ldv + i] = fin[i];
}
// </hot-kernel>

// ---------------------------------------------------------------------------
// k_batch_update: one iteration; grid = (row blocks, problems).  The iterate
// is staged into LDS once per workgroup; Y_next goes straight to HBM.
// ---------------------------------------------------------------------------
template <int NT, int U = 8, bool NTL = false>
__global__ void __launch_bounds__(NT) k_batch_update(const float* __restrict__ QdT, long long qstride, int ldq,
                                                     int N, const float* __restrict__ theta,
                                                     const float* __restrict__ Fd, int ldv,
                                                     const float* __restrict__ Yin, float* __restrict__ Yout) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int b = blockIdx.y;
    const int tid = threadIdx.x;
    const float* yg = Yin + (size_t)b * ldv;
    for (int i = tid; i < ldq; i += NT) lds[i] = (i < N) ? yg[i] : 0.0f;
    __syncthreads();
    const int r0 = blockIdx.x * 4 * NT;
    const int row = r0 + 4 * tid;
    const int w0 = r0 + 256 * (tid >> 6);
    if (row < N)
        update_rows4<U, NTL>(QdT + (size_t)b * (size_t)qstride, ldq, N, row, w0, theta + (size_t)b * ldv,
                     Fd + (size_t)b * ldv, lds, Yout + (size_t)b * ldv);
}

// ---------------------------------------------------------------------------
// k_update_split: the reference's own updateY2 interface -- two STORED split
// matrices (column-major here), Fdp/Fdn given.  PQP_CPU.c:603-618.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_update_split(const float* __restrict__ QpT, const float* __restrict__ QnT,
                                                      int ldq, int N, const float* __restrict__ Fdp,
                                                      const float* __restrict__ Fdn, const float* __restrict__ Y,
                                                      float* __restrict__ Ynext) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    float num = 0.0f, den = 0.0f;
    for (int k = 0; k < N; ++k) num += QnT[(size_t)k * ldq + i] * Y[k];
    for (int k = 0; k < N; ++k) den += QpT[(size_t)k * ldq + i] * Y[k];
    num = num + 1.0f * Fdn[i];
    den = den + 1.0f * Fdp[i];
    Ynext[i] = num / den * Y[i];
}

// ---------------------------------------------------------------------------
// Single large problem, fixed mode, spread over many workgroups (BASELINE
// configs[2]), and the row blocks of a row-sharded problem.
// The reference's two stored split matrices are kept (8 B per entry): lane
// p = 2i + side owns local row i's numerator (side 0, Qdn_theta) or
// denominator (side 1, Qdp_theta).  A block of `rows` rows starting at global
// row `row0` is spread over ceil(2 rows / 64) single-wave workgroups.
// Layout: workgroup-major 4-k packets, SP[wg][kb][lane < lw][4] = the entries
// for k = 4kb..4kb+3, so each workgroup streams its own contiguous region
// (KB * lw * 16 B) with one dwordx4 per lane per four k, and a wave reads
// lw * 16 B contiguous per load.  k >= N is padded with +0 (an exact no-op) and the
// padding lanes of the last workgroup hold zeros.  The per-update floor is
// one lane's N-long mul/add chain plus the bytes one CU can pull.
// ---------------------------------------------------------------------------
// lw = lanes (row sides) per workgroup: 64, 32, 16 or 8.  Fewer rows per
// workgroup spread a block over more CUs (each CU then pulls fewer bytes per
// update; the per-CU fetch rate, not HBM, bounds a single small problem).
__host__ __device__ inline int split_wgs(int rows, int lw) { return (2 * rows + lw - 1) / lw; }

// Qd: the block's rows, row-major with leading dimension ld (row i local =
// global row row0 + i); theta: the block's Theta_ii (rows); Fd: full N-vector.
__global__ void __launch_bounds__(256) k_build_split(const float* __restrict__ Qd, int ld,
                                                     const float* __restrict__ theta, const float* __restrict__ Fd,
                                                     int N, int rows, int row0, int lw, float* __restrict__ SP,
                                                     float* __restrict__ fdpn) {
    const int KB = split_kblocks(N);
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;  // (i, k) with k < 4*KB
    if (e < (long long)rows * 4 * KB) {
        const int i = (int)(e / (4 * KB)), k = (int)(e % (4 * KB));
        float qn = 0.0f, qp = 0.0f;
        if (k < N) {
            const float q = Qd[(size_t)i * ld + k];
            const float t = (row0 + i == k) ? theta[i] : 0.0f;
            qn = max_ref(0.0f, -q) + 1.0f * t;  // computeQdn_theta :533-537
            qp = max_ref(0.0f, q) + 1.0f * t;   // computeQdp_theta :524-528
        }
        const int p = 2 * i;  // even, so lane p + 1 is in the same workgroup
        const size_t base = (((size_t)(p / lw) * KB + (k >> 2)) * lw + (p % lw)) * 4 + (k & 3);
        SP[base] = qn;      // lane 2i
        SP[base + 4] = qp;  // lane 2i + 1
    }
    if (e < rows) {
        const float fd = Fd[row0 + e];
        fdpn[2 * e + 0] = max_ref(0.0f, -fd);  // Fdn :704
        fdpn[2 * e + 1] = max_ref(0.0f, fd);   // Fdp :703
    }
}

// Theta_ii = max(sum_k max(0, -Qd_ik) * 1.0, 5) for the block's rows
// (computeTheta, PQP_CPU.c:503-519; k sequential).
__global__ void __launch_bounds__(256) k_theta_rows(const float* __restrict__ Qd, int ld, int N, int rows,
                                                    float* __restrict__ theta) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= rows) return;
    float s = 0.0f;
    for (int k = 0; k < N; ++k) s += max_ref(0.0f, -Qd[(size_t)i * ld + k]) * 1.0f;
    theta[i] = max_ref(s, 5.0f);
}

// Stage y[0..N) (zero-padded to n_lds) in LDS with one wave.  Each batch
// issues all of its loads before the LDS stores, so their latencies overlap;
// a plain load-store loop would pay one L2 round trip per 64 elements, which
// dominated the single-problem update.
__device__ inline void stage_y_lds(const float* __restrict__ Y, int N, int n_lds, float* ys) {
    const int t = threadIdx.x;
    int done = 0;
    if ((reinterpret_cast<uintptr_t>(Y) & 15) == 0) {
        const int N4 = N >> 2;
        const float4* Y4 = reinterpret_cast<const float4*>(Y);
        for (int b = 0; b < N4; b += 64 * 8) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = b + 64 * j + t;
                v[j] = (i < N4) ? Y4[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = b + 64 * j + t;
                if (i < N4) reinterpret_cast<float4*>(ys)[i] = v[j];
            }
        }
        done = 4 * N4;
    }
    for (int b = done; b < n_lds; b += 64 * 16) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int k = b + 64 * j + t;
            v[j] = (k < N) ? Y[k] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int k = b + 64 * j + t;
            if (k < n_lds) ys[k] = v[j];
        }
    }
    __syncthreads();
}

// One update of a row block over its stored split matrices: W waves per
// workgroup share the workgroup's 32 rows (lanes 2i + side: one side of row
// i each, the SP layout of k_build_split) and split the k range
// into segments of S packets (4S values of k).  Segment g belongs to wave
// g % W.  A wave loads its segment into registers as early as it can and
// multiplies it by y while earlier segments are being summed; only the
// additions form the sequential chain, and they run segment after segment,
// the running sums handed from wave to wave through LDS (a turn counter
// orders the hand-off).  Each row's sum therefore still runs over k = 0..N-1
// in order from +0.0f, bit-identical to the reference, while a workgroup
// keeps W*S KiB of packets in flight, and the chain issues 4 cycles per k (an
// add) instead of 8 (a multiply and an add).  (A streaming one-wave form and
// relay shapes W x S = 4 x 64, 8 x 32, 16 x 16 were measured slower and
// removed in round 4: profiles/r01/split_sweep.txt.)
template <int W, int S>
__global__ void __launch_bounds__(64 * W) k_split_relay(const float* __restrict__ SP, const float* __restrict__ fdpn,
                                                        int N, int rows, int row0, int lw,
                                                        const float* __restrict__ Yin, float* __restrict__ Yout,
                                                        const int* __restrict__ gate, int* __restrict__ err,
                                                        int spin_max) {
    if (gate && *gate != kStatusContinue) return;  // converge-mode solve already finished
    // LDS: [64] hand-off words, then y [4*KB]
    extern __shared__ __attribute__((aligned(16))) float lds[];
    unsigned long long* slot = reinterpret_cast<unsigned long long*>(lds);  // per lane: (seq << 32) | bits(sum)
    float* ys = lds + 128;
    const int KB = split_kblocks(N);
    // w is wave-uniform; readfirstlane tells the compiler so (segment offsets
    // then live in SGPRs instead of forcing waterfall loops around the loads)
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // lanes >= lw repeat lane % lw's loads (same cache lines) and are discarded
    const int ll = lane % lw;
    const int p = blockIdx.x * lw + ll;
    const bool live = lane < lw && p < 2 * rows;
    const int G = (KB + S - 1) / S;  // segments
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef float f2v __attribute__((ext_vector_type(2)));
    const float* region = SP + (size_t)blockIdx.x * KB * lw * 4;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(region), (short)0, KB * lw * 16, 0x00020000);
    const int vo = ll * 16, kstride = lw * 16;
    f4v q[S];
    const bool lane_loads = lane < lw;  // lanes >= lw would only repeat lane % lw's requests
    auto load_seg = [&](int g) {
        // packets past KB (the last segment's tail) are +0, an exact no-op;
        // they are not loaded (the SGPR offset is not range-checked)
        const int nj = KB - g * S;  // wave-uniform
#pragma unroll
        for (int j = 0; j < S; ++j)
            q[j] = (j < nj && lane_loads) ? __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (g * S + j) * kstride, 0)
                                          : f4v{0.0f, 0.0f, 0.0f, 0.0f};
    };
    if (w < G) load_seg(w);  // independent of y: in flight while y is staged
    const float fd = live ? fdpn[p] : 0.0f;
    // y staged by all W waves (loads issued before the LDS stores), zeroed up
    // to the end of the last segment: the products of the tail packets read
    // it, and LDS is not cleared between launches (0 * stale NaN = NaN)
    {
        const int t = threadIdx.x, n_lds = 4 * G * S;
        for (int b = 0; b < n_lds; b += 64 * W * 8) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = b + 64 * W * j + t;
                v[j] = (k < N) ? Yin[k] : 0.0f;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = b + 64 * W * j + t;
                if (k < n_lds) ys[k] = v[j];
            }
        }
        if (w == 0) slot[lane] = 0ull;  // segment 0 starts from +0.0f
    }
    __syncthreads();
    float acc = 0.0f;
    bool stale = false;
    for (int g = w; g < G; g += W) {
        // products of this segment (packed multiplies, each product rounded
        // exactly as q * y), overwriting the packets; y is read from LDS four
        // packets at a time so the reads overlap (one at a time, the first
        // segment's products took twice as long on the critical path)
#pragma unroll
        for (int j0 = 0; j0 < S; j0 += 4) {
            f4v y[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) y[u] = *reinterpret_cast<const f4v*>(ys + 4 * (g * S + j0 + u));
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j = j0 + u;
                const f2v lo = f2v{q[j].x, q[j].y} * f2v{y[u].x, y[u].y};
                const f2v hi = f2v{q[j].z, q[j].w} * f2v{y[u].z, y[u].w};
                q[j] = f4v{lo.x, lo.y, hi.x, hi.y};
            }
            // pin the products here, before the wait below: otherwise the
            // compiler sinks the multiplies into the add chain
#pragma unroll
            for (int u = 0; u < 4; ++u) asm volatile("" : "+v"(q[j0 + u]));
        }
        // wait until every lane's hand-off word carries sequence g (the sum
        // and its sequence number travel in one 64-bit LDS word).  Bounded:
        // an expired wait is reported through *err at exit, not hung on.
        const unsigned long long h = relay_wait(slot, lane, g, spin_max, stale);
        __builtin_amdgcn_s_setprio(3);
        acc = __uint_as_float((unsigned)h);
#pragma unroll
        for (int j = 0; j < S; ++j) {
            acc += q[j].x;  // :608-609, k in order
            acc += q[j].y;
            acc += q[j].z;
            acc += q[j].w;
        }
        __hip_atomic_store(slot + lane, ((unsigned long long)(g + 1) << 32) | __float_as_uint(acc), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_s_setprio(0);
        if (g + W < G) load_seg(g + W);
    }
    if (w == (G - 1) % W) {  // the wave that summed the last segment
        const float v = acc + 1.0f * fd;     // even lane: num (:611), odd lane: den (:612)
        const float den = __shfl_xor(v, 1);  // the whole wave is here
        if (!(p & 1) && live) {
            const int i = p >> 1;
            Yout[i] = v / den * ys[row0 + i];  // :594
        }
    }
    relay_report(stale, err, lane);
}

// ---------------------------------------------------------------------------
// k_lean_relay<W,S>: the relay update over Qd itself (4 B per entry) instead of
// the stored split matrices (8 B): half the bytes, for blocks whose update the
// bytes bound (rows x N >= 4096^2; below that the three instructions per k of
// forming the terms cost more than the bytes saved).  Lanes 2i + side hold one
// side of row i, as for the split matrices: both read row i's Qd packet (one
// cache line), num negates q, and each lane sums one side with one add per k.  One lane owns one ROW and keeps both sums, num
// and den, as the two halves of one packed accumulator: the chain is one
// v_pk_add_f32 per k (each half rounds exactly like the scalar add), so it
// issues like the split form's single add.  The terms are formed ahead of the
// turn: off the diagonal the lean form
//   den += (q < 0) ? 0*y : q*y ;   num += (q > 0) ? 0*y : -(q*y)
// (bit-identical to (max(0,+-q) + 0.0f) * y, DESIGN.md "Lean form"); in the
// one or two segments that hold this workgroup's diagonal, the reference's
// literal (max(0,+-q) + (k == i ? Theta_i : +0)) * y for every k.
// Layout LP[wg][kb][lw] packets of 4 k of row wg*lw + lane; aux[row] =
// {Fdn, Fdp, Theta, 0}.
// ---------------------------------------------------------------------------
constexpr int kLeanS = 16;  // packets per k_lean_relay segment (the builder flags NaN per segment)
__global__ void __launch_bounds__(256) k_build_lean(const float* __restrict__ Qd, int ld,
                                                    const float* __restrict__ theta, const float* __restrict__ Fd,
                                                    int N, int rows, int row0, int lw, float* __restrict__ LP,
                                                    float* __restrict__ aux) {
    const int KB = split_kblocks(N);
    const int rp = lw >> 1;  // rows per workgroup
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;  // (i, k), k fastest
    if (e < (long long)rows * 4 * KB) {
        const int i = (int)(e / (4 * KB)), k = (int)(e % (4 * KB));
        const size_t at = (((size_t)(i / rp) * KB + (k >> 2)) * rp + (i % rp)) * 4 + (k & 3);
        const float q = k < N ? Qd[(size_t)i * ld + k] : 0.0f;
        LP[at] = q;
        if (q != q) {  // this (workgroup, segment) needs the compare/select form
            const int G = (KB + kLeanS - 1) / kLeanS, nwg = (rows + rp - 1) / rp;
            int* segnan = reinterpret_cast<int*>(aux + 4 * (size_t)nwg * rp);
            atomicOr(segnan + (size_t)(i / rp) * G + (k >> 2) / kLeanS, 1);
        }
    }
    if (e < rows) {
        const float fd = Fd[row0 + e];
        aux[4 * e + 0] = max_ref(0.0f, -fd);  // Fdn :704
        aux[4 * e + 1] = max_ref(0.0f, fd);   // Fdp :703
        aux[4 * e + 2] = theta[e];            // computeTheta :503-519
        aux[4 * e + 3] = 0.0f;
    }
}

template <int W, int S>
__global__ void __launch_bounds__(64 * W) k_lean_relay(const float* __restrict__ LP, const float* __restrict__ aux,
                                                       int N, int rows, int row0, int lw,
                                                       const float* __restrict__ Yin, float* __restrict__ Yout,
                                                       const int* __restrict__ gate, int* __restrict__ err,
                                                       int spin_max) {
    if (gate && *gate != kStatusContinue) return;  // converge-mode solve already finished
    // LDS: [64] hand-off words, then y [4*G*S]
    extern __shared__ __attribute__((aligned(16))) float lds[];
    unsigned long long* slot = reinterpret_cast<unsigned long long*>(lds);
    float* ys = lds + 128;
    const int KB = split_kblocks(N);
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ll = lane % lw;  // lanes >= lw repeat lane % lw's requests and are discarded
    const int rp = lw >> 1;    // rows per workgroup: lane 2i + side holds one side of row i
    const int side = ll & 1;   // 0: num (Qdn_theta), 1: den (Qdp_theta)
    const int r = blockIdx.x * rp + (ll >> 1);
    const bool live = lane < lw && r < rows;
    const int G = (KB + S - 1) / S;
    typedef float f4v __attribute__((ext_vector_type(4)));
    const float* region = LP + (size_t)blockIdx.x * KB * rp * 4;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(region), (short)0, KB * rp * 16, 0x00020000);
    const int vo = (ll >> 1) * 16, kstride = rp * 16;  // both lanes of a row read its packet (one cache line)
    f4v q[S];
    const bool lane_loads = lane < lw;
    auto load_seg = [&](int g) {
        const int nj = KB - g * S;  // wave-uniform; packets past KB are +0 and not loaded
#pragma unroll
        for (int j = 0; j < S; ++j)
            q[j] = (j < nj && lane_loads) ? __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (g * S + j) * kstride, 0)
                                          : f4v{0.0f, 0.0f, 0.0f, 0.0f};
    };
    if (w < G) load_seg(w);
    const f4v ax = live ? *reinterpret_cast<const f4v*>(aux + 4 * (size_t)r) : f4v{0.0f, 0.0f, 0.0f, 0.0f};
    const int* segnan = reinterpret_cast<const int*>(aux + 4 * (size_t)gridDim.x * rp);  // [wg][G] NaN flags
    {
        const int t = threadIdx.x, n_lds = 4 * G * S;
        for (int b = 0; b < n_lds; b += 64 * W * 8) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = b + 64 * W * j + t;
                v[j] = (k < N) ? Yin[k] : 0.0f;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = b + 64 * W * j + t;
                if (k < n_lds) ys[k] = v[j];
            }
        }
        if (w == 0) slot[lane] = 0ull;  // segment 0 starts from +0.0f
    }
    __syncthreads();
    const int d0 = row0 + blockIdx.x * rp;  // the workgroup's first diagonal k (wave-uniform)
    const int diag = row0 + r;              // this lane's diagonal k
    const float th = ax.z;
    const float fd = side ? ax.y : ax.x;    // Fdp / Fdn (:703-704)
    // this lane's side of the split entry: den uses q, num uses -q (negation is
    // exact), so every form below is the den formula on qs
    const unsigned sgn = side ? 0u : 0x80000000u;
    float acc = 0.0f;
    bool stale = false;
    for (int g = w; g < G; g += W) {
        const int kbase = 4 * g * S;
        const bool lit = kbase < d0 + rp && kbase + 4 * S > d0;  // a diagonal of this workgroup is in here
        const bool nan_seg = !lit && segnan[(size_t)blockIdx.x * G + g] != 0;  // a NaN of Qd is in here
        // the terms replace the packets in place; the branch is per segment,
        // each side one straight-line unrolled loop (2: literal, 1: lean with
        // compares, 0: lean by max)
        auto form = [&](auto kind) {
            constexpr int KIND = decltype(kind)::value;
            // distinct volatile markers keep the sides from being merged back
            // into a branch per k
            if constexpr (KIND == 2)
                asm volatile("; literal terms");
            else if constexpr (KIND == 1)
                asm volatile("; lean terms, compare/select");
            else
                asm volatile("; lean terms, max");
#pragma unroll
            for (int j0 = 0; j0 < S; j0 += 4) {
                f4v y[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) y[u] = *reinterpret_cast<const f4v*>(ys + 4 * (g * S + j0 + u));
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int j = j0 + u;
                    float qv[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
                    const float yv[4] = {y[u].x, y[u].y, y[u].z, y[u].w};
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float qs = __uint_as_float(__float_as_uint(qv[c]) ^ sgn);
                        const float yy = yv[c];
                        if constexpr (KIND == 0) {
                            // no NaN in this segment's q: max(qs, 0) * y is the
                            // reference's (max(0, qs) + 0.0f) * y up to the sign of
                            // a zero term, which adds nothing to a sum that is never
                            // -0 (0 * inf / NaN y still gives NaN).  v_max_f32
                            // directly: fmaxf would first quiet a NaN (one more
                            // instruction), and there is none here
                            float m;
                            asm("v_max_f32_e64 %0, 0, %1" : "=v"(m) : "v"(qs));
                            qv[c] = m * yy;
                        } else if constexpr (KIND == 1) {
                            const float p = qs * yy;
                            const float z = 0.0f * yy;  // (+0)*y: NaN for inf/NaN y
                            qv[c] = qs < 0.0f ? z : p;
                        } else {  // computeQdp/Qdn_theta :524-537, then :608-609
                            const float t = (kbase + 4 * j + c == diag) ? th : 0.0f;
                            qv[c] = (max_ref(0.0f, qs) + t) * yy;
                        }
                    }
                    q[j] = f4v{qv[0], qv[1], qv[2], qv[3]};
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) asm volatile("" : "+v"(q[j0 + u]));
            }
            if constexpr (KIND == 2)
                asm volatile("; literal terms end");
            else if constexpr (KIND == 1)
                asm volatile("; lean terms, compare/select, end");
            else
                asm volatile("; lean terms, max, end");
        };
        if (lit)
            form(std::integral_constant<int, 2>{});
        else if (nan_seg)
            form(std::integral_constant<int, 1>{});
        else
            form(std::integral_constant<int, 0>{});
        const unsigned long long h = relay_wait(slot, lane, g, spin_max, stale);
        __builtin_amdgcn_s_setprio(3);
        acc = __uint_as_float((unsigned)h);
#pragma unroll
        for (int j = 0; j < S; ++j) {
            acc += q[j].x;  // :608-609, k in order
            acc += q[j].y;
            acc += q[j].z;
            acc += q[j].w;
        }
        __hip_atomic_store(slot + lane, ((unsigned long long)(g + 1) << 32) | __float_as_uint(acc), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_s_setprio(0);
        if (g + W < G) load_seg(g + W);
    }
    if (w == (G - 1) % W) {  // the wave that summed the last segment
        const float v = acc + 1.0f * fd;     // even lane: num (:611), odd lane: den (:612)
        const float den = __shfl_xor(v, 1);  // the whole wave is here
        if (!side && live) Yout[r] = v / den * ys[row0 + r];  // updY :594
    }
    relay_report(stale, err, lane);
}

bool use_lean(int N, int rows) {
    return g_tune.lean_min_n > 0 && (long long)rows * N >= (long long)g_tune.lean_min_n * g_tune.lean_min_n;
}
// lw = row SIDES per workgroup (as for the split matrices): lw / 2 rows
size_t lean_floats(int N, int rows, int lw) { return (size_t)cdiv(2LL * rows, lw) * split_kblocks(N) * (lw / 2) * 4; }
size_t lean_aux_floats(int N, int rows, int lw) {  // per-row words, then the [wg][segment] NaN flags
    const size_t nwg = cdiv(2LL * rows, lw);
    return nwg * (lw / 2) * 4 + nwg * cdiv(split_kblocks(N), kLeanS);
}
int lean_pick_lw(int rows) { return split_pick_lw(rows); }
hipError_t launch_build_lean(const float* Qd, int ld, const float* theta, const float* Fd, int N, int rows, int row0,
                             int lw, float* LP, float* aux, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    const size_t nwg = cdiv(2LL * rows, lw), nflag = nwg * cdiv(split_kblocks(N), kLeanS);
    hipError_t e = hipMemsetAsync(aux + 4 * nwg * (lw / 2), 0, sizeof(int) * nflag, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_build_lean, dim3(cdiv((long long)rows * 4 * split_kblocks(N), 256)), dim3(256), 0, s, Qd,
                       ld, theta, Fd, N, rows, row0, lw, LP, aux);
    return hipGetLastError();
}
hipError_t launch_lean_update(const float* LP, const float* aux, int N, int rows, int row0, int lw, const float* Yin,
                              float* Yout, hipStream_t s, const int* gate, int* err) {
    if (rows <= 0) return hipSuccess;
    constexpr int W = 8, S = kLeanS;
    const int G = (split_kblocks(N) + S - 1) / S;
    const size_t lds = sizeof(float) * ((size_t)4 * G * S + 128);
    hipLaunchKernelGGL((k_lean_relay<W, S>), dim3(cdiv(2LL * rows, lw)), dim3(64 * W), lds, s, LP, aux, N, rows, row0,
                       lw, Yin, Yout, gate, err, g_tune.relay_spin_max);
    return hipGetLastError();
}

size_t split_floats(int N, int rows, int lw) { return (size_t)split_wgs(rows, lw) * split_kblocks(N) * lw * 4; }
// LDS of the split updates (the full y, padded to a whole relay segment of up
// to 64 packets, plus the relay's hand-off words)
size_t split_lds_bytes(int N) { return sizeof(float) * ((size_t)4 * (split_kblocks(N) + 64) + 128); }

int split_pick_lw(int rows) {
    if (g_tune.split_lw == 8 || g_tune.split_lw == 16 || g_tune.split_lw == 32 || g_tune.split_lw == 64) return g_tune.split_lw;
    // about one workgroup per CU: 2 rows / lw ~ 256
    int lw = 8;
    while (lw < 64 && 2LL * rows > 256LL * lw) lw *= 2;
    return lw;
}

hipError_t launch_build_split(const float* Qd, int ld, const float* theta, const float* Fd, int N, int rows,
                              int row0, int lw, float* SP, float* fdpn, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_build_split, dim3(cdiv((long long)rows * 4 * split_kblocks(N), 256)), dim3(256), 0, s, Qd,
                       ld, theta, Fd, N, rows, row0, lw, SP, fdpn);
    return hipGetLastError();
}

hipError_t launch_theta_rows(const float* Qd, int ld, int N, int rows, float* theta, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_theta_rows, dim3(cdiv(rows, 256)), dim3(256), 0, s, Qd, ld, N, rows, theta);
    return hipGetLastError();
}


template <int W, int S>
static void launch_relay(const float* SP, const float* fdpn, int N, int rows, int row0, int lw, const float* Yin,
                         float* Yout, hipStream_t s, const int* gate, int* err) {
    const int G = (split_kblocks(N) + S - 1) / S;
    const size_t lds = sizeof(float) * ((size_t)4 * G * S + 128);  // y to the end of the last segment
    hipLaunchKernelGGL((k_split_relay<W, S>), dim3(split_wgs(rows, lw)), dim3(64 * W), lds, s, SP, fdpn, N, rows,
                       row0, lw, Yin, Yout, gate, err, g_tune.relay_spin_max);
}

hipError_t launch_split_update(const float* SP, const float* fdpn, int N, int rows, int row0, int lw,
                               const float* Yin, float* Yout, hipStream_t s, const int* gate, int* err) {
    if (rows <= 0) return hipSuccess;
    launch_relay<8, 16>(SP, fdpn, N, rows, row0, lw, Yin, Yout, s, gate, err);
    return hipGetLastError();
}

__global__ void k_fill(float* __restrict__ a, float v, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) a[i] = v;
}
hipError_t launch_fill(float* a, float v, int n, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_fill, dim3(cdiv(n, 256)), dim3(256), 0, s, a, v, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Setup kernels
// ---------------------------------------------------------------------------
// Row-major N x N (contiguous per problem) -> column-major QdT with padding.
__global__ void __launch_bounds__(256) k_pack_colmajor(const float* __restrict__ Qd, int N, long long in_stride,
                                                       float* __restrict__ QdT, int ldq, long long qstride) {
    __shared__ float tile[32][33];
    const int b = blockIdx.z;
    const int k0 = blockIdx.x * 32, i0 = blockIdx.y * 32;  // output column k, rows i
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    const float* src = Qd + (size_t)b * in_stride;
    float* dst = QdT + (size_t)b * qstride;
    for (int r = ty; r < 32; r += 8) {
        const int i = i0 + r, k = k0 + tx;
        tile[r][tx] = (i < N && k < N) ? src[(size_t)i * N + k] : 0.0f;
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int k = k0 + r, i = i0 + tx;
        if (k < N && i < ldq) dst[(size_t)k * ldq + i] = tile[tx][r];
    }
}

// theta_i = max( sum_k max(0,-Qd[i][k]) * 1.0f , 5 )   computeTheta + diagonalAdd
// (PQP_CPU.c:503-519, 235-242), sequential k; one lane per row, coalesced.
__global__ void __launch_bounds__(256) k_theta(const float* __restrict__ QdT, int ldq, long long qstride, int N,
                                               float* __restrict__ theta, int ldv) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const float* col = QdT + (size_t)b * (size_t)qstride + i;
    float s = 0.0f;
    for (int k = 0; k < N; ++k) s += max_ref(0.0f, -col[(size_t)k * ldq]) * 1.0f;
    theta[(size_t)b * ldv + i] = max_ref(s, 5.0f);
}

// The same, four adjacent rows per lane with 16-byte loads, 8 columns of
// loads in flight (ldq, qstride multiples of 4, QdT 16-byte aligned).
__global__ void __launch_bounds__(256) k_theta4(const float* __restrict__ QdT, int ldq, long long qstride, int N,
                                                float* __restrict__ theta, int ldv) {
    typedef float tf4 __attribute__((ext_vector_type(4)));
    const int b = blockIdx.y;
    const int i0 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (i0 >= N) return;
    const float* col = QdT + (size_t)b * (size_t)qstride + i0;
    float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    int k = 0;
    for (; k + 8 <= N; k += 8) {
        tf4 q[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = *reinterpret_cast<const tf4*>(col + (size_t)(k + j) * ldq);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[r] += max_ref(0.0f, -q[j][r]) * 1.0f;
    }
    for (; k < N; ++k) {
        const tf4 q = *reinterpret_cast<const tf4*>(col + (size_t)k * ldq);
#pragma unroll
        for (int r = 0; r < 4; ++r) s[r] += max_ref(0.0f, -q[r]) * 1.0f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (i0 + r < N) theta[(size_t)b * ldv + i0 + r] = max_ref(s[r], 5.0f);
}

// Synthetic dual: Qd(i,j) = sum_k (Gp(i,k) q_k) Gp(j,k), k sequential.  The
// convertToDual products Gp.Qp_inv are exact for a diagonal Qp_inv (all other
// terms are +-0), so (Gp Qp_inv)(i,k) = Gp(i,k)*q_k bit for bit.  64x64 output
// tile per 256-thread workgroup, 4x4 per thread, Gp regenerated from the
// counter hash into LDS per 32-deep k chunk.
constexpr int SYN_T = 64, SYN_K = 32;
__global__ void __launch_bounds__(256) k_synth_qd(uint32_t seed, long long inst0, int N, int M,
                                                  float* __restrict__ QdT, int ldq, long long qstride, int c0,
                                                  int cols) {
    __shared__ float gq[SYN_K][SYN_T + 4];  // (Gp Qinv)(i0+ii, k0+kk) stored [kk][ii]
    __shared__ float gj[SYN_K][SYN_T + 4];  // Gp(j0+jj, k0+kk) stored [kk][jj]
    const int b = blockIdx.z;
    const SynthKeys K = synth_keys(seed, (uint32_t)(inst0 + b));
    // columns j in [c0, c0 + cols) only (stored at column j - c0): a column
    // block of the exactly symmetric Qd is the row-major block of its rows
    const int i0 = blockIdx.x * SYN_T, j0 = c0 + blockIdx.y * SYN_T;
    const int jend = (c0 + cols < N) ? c0 + cols : N;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    float acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = 0.0f;
    for (int k0 = 0; k0 < M; k0 += SYN_K) {
        // fill: 64 x 32 each; thread covers (kk = tid & 31, rows (tid >> 5) + 8*s)
        {
            const int kk = tid & 31, k = k0 + kk;
            const float q = (k < M) ? synth_qinv(K, k) : 0.0f;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int rr = (tid >> 5) + 8 * s;
                const int i = i0 + rr, j = j0 + rr;
                gq[kk][rr] = (k < M && i < N) ? synth_gp(K, i, k, M) * q : 0.0f;
                gj[kk][rr] = (k < M && j < jend) ? synth_gp(K, j, k, M) : 0.0f;
            }
        }
        __syncthreads();
        const int kend = (M - k0) < SYN_K ? (M - k0) : SYN_K;
        for (int kk = 0; kk < kend; ++kk) {
            float a[4], g[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] = gq[kk][tx + 16 * r];
#pragma unroll
            for (int c = 0; c < 4; ++c) g[c] = gj[kk][ty + 16 * c];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] += a[r] * g[c];
        }
        __syncthreads();
    }
    float* dst = QdT + (size_t)b * (size_t)qstride;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int j = j0 + ty + 16 * c;
        if (j >= jend) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + tx + 16 * r;
            if (i < ldq) dst[(size_t)(j - c0) * ldq + i] = (i < N) ? acc[r][c] : 0.0f;  // Qd(i,j) at col j
        }
    }
}

// Synthetic Fd(i) = sum_k (Gp(i,k) q_k) Fp_k + Kp_i  and  Md = sum_j (Fp_j q_j) Fp_j - Mp
// (computeFd / computeMd, PQP_CPU.c:456-479).
__global__ void __launch_bounds__(256) k_synth_fd(uint32_t seed, long long inst0, int N, int M,
                                                  float* __restrict__ Fd, int ldv, float* __restrict__ Md) {
    const int b = blockIdx.y;
    const SynthKeys K = synth_keys(seed, (uint32_t)(inst0 + b));
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < N) {
        float s = 0.0f;
        for (int k = 0; k < M; ++k) s += (synth_gp(K, i, k, M) * synth_qinv(K, k)) * synth_fp(K, k);
        Fd[(size_t)b * ldv + i] = s + 1.0f * synth_kp(K, i);
    }
    for (int i2 = N + i; i2 < ldv; i2 += gridDim.x * 256) Fd[(size_t)b * ldv + i2] = 0.0f;
    if (Md && blockIdx.x == 0 && threadIdx.x == 0) {
        float s = 0.0f;
        for (int j = 0; j < M; ++j) {
            const float f = synth_fp(K, j);
            s += (f * synth_qinv(K, j)) * f;
        }
        Md[b] = s - 1.0f;  // Md[0] -= Mp[0], Mp = 1
    }
}

// Synthetic primal problem (the generator behind pqp_batch_generate's duals):
// Qp_inv = diag(0.1 + u), Gp in {-1, 0, +1}, Kp = 10u, Fp = 20u - 10, Mp = 1.
__global__ void __launch_bounds__(256) k_synth_primal(uint32_t seed, long long inst0, int N, int M,
                                                      float* __restrict__ Qinv, float* __restrict__ Gp,
                                                      float* __restrict__ Kp, float* __restrict__ Fp,
                                                      float* __restrict__ Mp) {
    const int b = blockIdx.y;
    const SynthKeys K = synth_keys(seed, (uint32_t)(inst0 + b));
    const long long nG = (long long)N * M, nQ = (long long)M * M;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < nG + nQ + N + M + 1;
         e += (long long)gridDim.x * 256) {
        if (e < nG) {
            Gp[(size_t)b * nG + e] = synth_gp(K, (int)(e / M), (int)(e % M), M);
        } else if (e < nG + nQ) {
            const long long q = e - nG;
            const int r = (int)(q / M), c = (int)(q % M);
            Qinv[(size_t)b * nQ + q] = (r == c) ? synth_qinv(K, r) : 0.0f;
        } else if (e < nG + nQ + N) {
            const int i = (int)(e - nG - nQ);
            Kp[(size_t)b * N + i] = synth_kp(K, i);
        } else if (e < nG + nQ + N + M) {
            const int j = (int)(e - nG - nQ - N);
            Fp[(size_t)b * M + j] = synth_fp(K, j);
        } else {
            Mp[b] = 1.0f;
        }
    }
}

hipError_t launch_synth_primal(uint32_t seed, long long inst0, int B, int N, int M, float* Qinv, float* Gp, float* Kp,
                               float* Fp, float* Mp, hipStream_t s) {
    for (int b0 = 0; b0 < B; b0 += 65535) {
        const int nb = (B - b0) < 65535 ? (B - b0) : 65535;
        const long long n = (long long)N * M + (long long)M * M + N + M + 1;
        const int gx = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
        hipLaunchKernelGGL(k_synth_primal, dim3(gx, nb), dim3(256), 0, s, seed, inst0 + b0, N, M,
                           Qinv + (size_t)b0 * M * M, Gp + (size_t)b0 * N * M, Kp + (size_t)b0 * N,
                           Fp + (size_t)b0 * M, Mp + b0);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
typedef float sf4 __attribute__((ext_vector_type(4)));  // (repeated, same type, in the solve-single region)

// Generic sequential-k product: out[a x c] = op(A)[a x b] op(B)[b x c]
// (matrixMultiply, PQP_CPU.c:84-147).  One thread per output element; used
// for setup and for the drop-in helpers, not on the iteration path.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_matmul_seq(float* __restrict__ out, const float* __restrict__ A, int tA,
                                                    const float* __restrict__ B, int tB, int a, int bdim, int c,
                                                    long long sA = 0, long long sB = 0, long long sO = 0) {
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long long)a * c) return;
    A += blockIdx.y * sA;  // problem blockIdx.y of a batch (strides 0 = shared operand)
    B += blockIdx.y * sB;
    out += blockIdx.y * sO;
    const int i = (int)(e / c), j = (int)(e % c);
    float s = 0.0f;
    for (int k = 0; k < bdim; ++k) {
        const float x = tA ? A[(size_t)k * a + i] : A[(size_t)i * bdim + k];
        const float y = tB ? B[(size_t)j * bdim + k] : B[(size_t)k * c + j];
        s += x * y;
    }
    out[e] = s;
}

// The same product, LDS-tiled (setup GEMMs of convertToDual at scale: Qd =
// (Gp Qp_inv) Gp', PQP_CPU.c:440-498).  A 64 x 64 output tile per 256-thread
// workgroup, 4 x 4 outputs per thread; op(A) and op(B) are staged 32 k at a
// time into LDS with coalesced reads in whichever layout the transpose flags
// give, and every output still sums k = 0..b-1 in order from +0.0f with the
// product rounded before each add (no FMA: -ffp-contract=off), exactly as
// matrixMultiply (:88-146) and k_matmul_seq.  grid = (ceil(c/64), ceil(a/64),
// problems); strides sA/sB/sO per problem (0 = shared operand).
constexpr int MMT = 64, MMK = 32;
__global__ void __launch_bounds__(256) k_matmul_tiled(float* __restrict__ out, const float* __restrict__ A, int tA,
                                                      const float* __restrict__ B, int tB, int a, int bdim, int c,
                                                      long long sA, long long sB, long long sO) {
    __shared__ __attribute__((aligned(16))) float As[MMK][MMT + 4];  // op(A)(i0 + ii, k0 + kk) at [kk][ii]
    __shared__ __attribute__((aligned(16))) float Bs[MMK][MMT + 4];  // op(B)(k0 + kk, j0 + jj) at [kk][jj]
    const int z = blockIdx.z;
    A += z * sA;
    B += z * sB;
    out += z * sO;
    const int j0 = blockIdx.x * MMT, i0 = blockIdx.y * MMT;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    float acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[r][q] = 0.0f;
    for (int k0 = 0; k0 < bdim; k0 += MMK) {
        // stage 64 x 32 of each operand (8 elements per thread), the fastest
        // thread index along the operand's contiguous dimension
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int e = tid + 256 * s;
            int ii, kk;
            if (tA) {  // A stored b x a: A(i,k) = A[k*a + i], i contiguous
                ii = e & 63;
                kk = e >> 6;
            } else {  // A stored a x b: A(i,k) = A[i*b + k], k contiguous
                kk = e & 31;
                ii = e >> 5;
            }
            const int i = i0 + ii, k = k0 + kk;
            float v = 0.0f;
            if (i < a && k < bdim) v = tA ? A[(size_t)k * a + i] : A[(size_t)i * bdim + k];
            As[kk][ii] = v;
            int jj, kb;
            if (tB) {  // B stored c x b: B(k,j) = B[j*b + k], k contiguous
                kb = e & 31;
                jj = e >> 5;
            } else {  // B stored b x c: B(k,j) = B[k*c + j], j contiguous
                jj = e & 63;
                kb = e >> 6;
            }
            const int j = j0 + jj, k2 = k0 + kb;
            float w = 0.0f;
            if (j < c && k2 < bdim) w = tB ? B[(size_t)j * bdim + k2] : B[(size_t)k2 * c + j];
            Bs[kb][jj] = w;
        }
        __syncthreads();
        const int kend = (bdim - k0) < MMK ? (bdim - k0) : MMK;
        for (int kk = 0; kk < kend; ++kk) {
            const float4 av = *reinterpret_cast<const float4*>(&As[kk][4 * tx]);
            const float4 bv = *reinterpret_cast<const float4*>(&Bs[kk][4 * ty]);
            const float ar[4] = {av.x, av.y, av.z, av.w}, br[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[r][q] += ar[r] * br[q];  // :88-100, k in order
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = i0 + 4 * tx + r;
        if (i >= a) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = j0 + 4 * ty + q;
            if (j < c) out[(size_t)i * c + j] = acc[r][q];
        }
    }
}

// The mat-vec form out[i] = sum_k A[i][k] x[k] (row-major A, c = 1; the Fd =
// (Gp Qp_inv) Fp of convertToDual, PQP_CPU.c:456-460, and computeUfromY's
// products, :352-360) at scale: 256 rows per workgroup, one lane per row
// summing k = 0..b-1 in order from +0.0f, the rows staged 32 k at a time
// through LDS with coalesced loads (32 lanes per 128-byte row segment)
// instead of each lane walking its own row at a stride of b floats.  k past
// b adds 0*0 = +0.0f to a sum that is never -0.0f.
__global__ void __launch_bounds__(256) k_matvec_rows(float* __restrict__ out, const float* __restrict__ A,
                                                     const float* __restrict__ x, int a, int bdim, long long sA,
                                                     long long sB, long long sO) {
    __shared__ float T[256][33];
    __shared__ float xs[32];
    const int z = blockIdx.y;
    A += z * sA;
    x += z * sB;
    out += z * sO;
    const int tid = threadIdx.x, row0 = blockIdx.x * 256, i = row0 + tid;
    float acc = 0.0f;
    for (int k0 = 0; k0 < bdim; k0 += 32) {
#pragma unroll 8
        for (int q = 0; q < 32; ++q) {
            const int e = q * 256 + tid, r = e >> 5, kk = e & 31;
            T[r][kk] = (row0 + r < a && k0 + kk < bdim) ? A[(size_t)(row0 + r) * bdim + k0 + kk] : 0.0f;
        }
        if (tid < 32) xs[tid] = (k0 + tid < bdim) ? x[k0 + tid] : 0.0f;
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 32; ++kk) acc += T[tid][kk] * xs[kk];  // :88-100, k in order
        __syncthreads();
    }
    if (i < a) out[i] = acc;
}

// The same mat-vec with one lane per row and no LDS: each lane walks its own
// row 16 bytes at a time, 16 loads in flight (a row's 128-byte lines are
// fetched once and re-read from the vector cache), x[k] wave-uniform
// (scalar loads).  One wave per 64 rows, so a batch of problems fills the
// chip (convertToDual's Fd = (Gp Qp_inv) Fp of 64 problems of n_dual 1024:
// 16 x 64 waves).  Needs bdim % 4 == 0 and 16-byte-aligned rows.
__global__ void __launch_bounds__(64) k_matvec_lane(float* __restrict__ out, const float* __restrict__ A,
                                                    const float* __restrict__ x, int a, int bdim, long long sA,
                                                    long long sB, long long sO) {
    const int z = blockIdx.y;
    A += z * sA;
    x += z * sB;
    out += z * sO;
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a) return;
    const float* row = A + (size_t)i * bdim;
    float acc = 0.0f;
    int k0 = 0;
    for (; k0 + 64 <= bdim; k0 += 64) {
        float4 v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = *reinterpret_cast<const float4*>(row + k0 + 4 * e);
#pragma unroll
        for (int e = 0; e < 16; ++e) {  // :88-100, k in order
            const int k = k0 + 4 * e;
            acc += v[e].x * x[k];
            acc += v[e].y * x[k + 1];
            acc += v[e].z * x[k + 2];
            acc += v[e].w * x[k + 3];
        }
    }
    for (; k0 < bdim; k0 += 4) {
        const float4 v = *reinterpret_cast<const float4*>(row + k0);
        acc += v.x * x[k0];
        acc += v.y * x[k0 + 1];
        acc += v.z * x[k0 + 2];
        acc += v.w * x[k0 + 3];
    }
    out[i] = acc;
}

// The row-vector form out[j] = sum_k x[k] B(k, j) (a = 1: convertToDual's
// Fp'Qp_inv and (Fp'Qp_inv) Fp, PQP_CPU.c:472-479, and computeCost-style
// dots): one lane per output j, k = 0..b-1 in order from +0.0f; x[k] is
// wave-uniform (scalar loads) and the k loop issues 8 loads of B ahead of its
// adds, so a lane's chain is not one memory round trip per k.  k past b adds
// 0*0 = +0.0f to a sum that is never -0.0f.
__global__ void __launch_bounds__(256) k_vecmat(float* __restrict__ out, const float* __restrict__ x,
                                                const float* __restrict__ B, int tB, int bdim, int c, long long sA,
                                                long long sB, long long sO) {
    const int z = blockIdx.y;
    x += z * sA;
    B += z * sB;
    out += z * sO;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= c) return;
    const float* col = tB ? B + (size_t)j * bdim : B + j;  // B(k, j) = col[k * step]
    const size_t step = tB ? 1 : (size_t)c;
    float s = 0.0f;
    for (int k0 = 0; k0 < bdim; k0 += 8) {
        float v[8], xv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = k0 + e;
            v[e] = k < bdim ? col[(size_t)k * step] : 0.0f;
            xv[e] = k < bdim ? x[k] : 0.0f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) s += xv[e] * v[e];  // :88-146, k in order
    }
    out[j] = s;
}

// The setup GEMM at scale, on packed fp32: a 128 x 128 output tile per
// 256-thread workgroup, 8 x 8 outputs per thread (rows 4tx+r and 64+4tx+r,
// columns 4ty+q and 64+4ty+q), op(A) and op(B) staged KT8 = 32 k at a time
// through LDS from 16-byte global loads, the next k-slab's loads issued into
// registers before the current slab is summed.  Every output still sums
// k = 0..b-1 in order from +0.0f with the product rounded before the add
// (matrixMultiply, PQP_CPU.c:88-146): the compiler forms the 64 products and
// adds of a k step as v_pk_mul_f32 / v_pk_add_f32, each half of which rounds
// like the scalar op.  The k range is zero-padded to a multiple of KT8: a
// padded step adds 0*0 = +0.0f to a sum that is never -0.0f (it starts at
// +0.0f; round-to-nearest gives +0.0f on exact cancellation), so the bits are
// those of the unpadded sum.  TA / TB: the transpose flags, so every staging
// load is branch-free; needs the contiguous dimension of each operand a
// multiple of 4 and 16-byte-aligned bases (launch_matmul_seq_b checks).
// Workgroups are numbered so that consecutive tiles -- the same problem's --
// run on one XCD (dispatch is round-robin over the 8 XCDs): each problem's
// operands are then fetched into one XCD's L2, not all eight.
constexpr int MM8 = 128, KT8 = 32, MM8P = MM8 + 4;
template <int TA, int TB>
__global__ void __launch_bounds__(256) k_matmul_pk(float* __restrict__ out, const float* __restrict__ A,
                                                   const float* __restrict__ B, int a, int bdim, int c, long long sA,
                                                   long long sB, long long sO, int tiles_x, int tiles_per_problem,
                                                   int problems) {
    __shared__ __attribute__((aligned(16))) float As[KT8][MM8P];  // op(A)(i0 + ii, k0 + kk) at [kk][ii]
    __shared__ __attribute__((aligned(16))) float Bs[KT8][MM8P];  // op(B)(k0 + kk, j0 + jj) at [kk][jj]
    // XCD-grouped numbering: logical tile q of the whole grid
    const int G = tiles_per_problem * problems, L = blockIdx.x;
    const int q = (G % 8 == 0) ? (L % 8) * (G / 8) + L / 8 : L;
    const int z = q / tiles_per_problem, t = q % tiles_per_problem;
    const int j0 = (t % tiles_x) * MM8, i0 = (t / tiles_x) * MM8;
    A += z * sA;
    B += z * sB;
    out += z * sO;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    // staging map: 128 x 32 of each operand = 1024 float4, 4 per thread.
    // k-contiguous operand (A with TA = 0, B with TB = 1): float4 along k,
    // 8 lanes per 128-byte row segment; element e: row e >> 3, k group e & 7.
    // i/j-contiguous operand: float4 along i/j; element e: k row e >> 5,
    // column group e & 31.
    sf4 ra[4], rb[4];
    auto load = [&](int k0) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int e = tid + 256 * s;
            if (TA == 0) {
                const int ii = e >> 3, kk = 4 * (e & 7), i = i0 + ii, k = k0 + kk;
                ra[s] = (i < a && k < bdim) ? *reinterpret_cast<const sf4*>(A + (size_t)i * bdim + k) : sf4{0, 0, 0, 0};
            } else {
                const int kk = e >> 5, ii = 4 * (e & 31), i = i0 + ii, k = k0 + kk;
                ra[s] = (i < a && k < bdim) ? *reinterpret_cast<const sf4*>(A + (size_t)k * a + i) : sf4{0, 0, 0, 0};
            }
            if (TB == 1) {
                const int jj = e >> 3, kk = 4 * (e & 7), j = j0 + jj, k = k0 + kk;
                rb[s] = (j < c && k < bdim) ? *reinterpret_cast<const sf4*>(B + (size_t)j * bdim + k) : sf4{0, 0, 0, 0};
            } else {
                const int kk = e >> 5, jj = 4 * (e & 31), j = j0 + jj, k = k0 + kk;
                rb[s] = (j < c && k < bdim) ? *reinterpret_cast<const sf4*>(B + (size_t)k * c + j) : sf4{0, 0, 0, 0};
            }
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int e = tid + 256 * s;
            if (TA == 0) {
                const int ii = e >> 3, kk = 4 * (e & 7);
#pragma unroll
                for (int x = 0; x < 4; ++x) As[kk + x][ii] = ra[s][x];
            } else {
                *reinterpret_cast<sf4*>(&As[e >> 5][4 * (e & 31)]) = ra[s];
            }
            if (TB == 1) {
                const int jj = e >> 3, kk = 4 * (e & 7);
#pragma unroll
                for (int x = 0; x < 4; ++x) Bs[kk + x][jj] = rb[s][x];
            } else {
                *reinterpret_cast<sf4*>(&Bs[e >> 5][4 * (e & 31)]) = rb[s];
            }
        }
    };
    float acc[8][8];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int x = 0; x < 8; ++x) acc[r][x] = 0.0f;
    load(0);
    for (int k0 = 0; k0 < bdim; k0 += KT8) {
        __syncthreads();  // the previous slab's sums are done with LDS
        store();
        __syncthreads();
        if (k0 + KT8 < bdim) load(k0 + KT8);  // in flight while this slab is summed
#pragma unroll 4
        for (int kk = 0; kk < KT8; ++kk) {
            const sf4 a0 = *reinterpret_cast<const sf4*>(&As[kk][4 * tx]);
            const sf4 a1 = *reinterpret_cast<const sf4*>(&As[kk][64 + 4 * tx]);
            const sf4 b0 = *reinterpret_cast<const sf4*>(&Bs[kk][4 * ty]);
            const sf4 b1 = *reinterpret_cast<const sf4*>(&Bs[kk][64 + 4 * ty]);
            const float ar[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const float br[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int x = 0; x < 8; ++x) acc[r][x] += ar[r] * br[x];  // :88-100, k in order
        }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int i = i0 + (r < 4 ? 4 * tx + r : 64 + 4 * tx + r - 4);
        if (i >= a) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = j0 + 64 * h + 4 * ty;
            float* o = out + (size_t)i * c + j;
            if (j + 3 < c) {
                *reinterpret_cast<sf4*>(o) = sf4{acc[r][4 * h], acc[r][4 * h + 1], acc[r][4 * h + 2], acc[r][4 * h + 3]};
            } else {
#pragma unroll
                for (int x = 0; x < 4; ++x)
                    if (j + x < c) o[x] = acc[r][4 * h + x];
            }
        }
    }
}

// A[i] += sign * B[i]   (matrixAdd, PQP_CPU.c:157-163)
__global__ void k_axpy(float* __restrict__ A, const float* __restrict__ B, float sign, int n, long long sA = 0,
                       long long sB = 0) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    A += blockIdx.y * sA;
    B += blockIdx.y * sB;
    if (i < n) A[i] += sign * B[i];
}
// A[i] = -A[i]   (negateMatrix, PQP_CPU.c:171-177)
__global__ void k_negate(float* __restrict__ A, int n, long long sA = 0) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    A += blockIdx.y * sA;
    if (i < n) A[i] = -A[i];
}
// flag = all(GpU <= Kp + max(erc*Kp, eac))   (compare, PQP_CPU.c:334-343); flag preset to 1
__global__ void k_compare(const float* __restrict__ gu, const float* __restrict__ Kp, int n, int* flag) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        const float kp = Kp[i];
        if (gu[i] > kp + max_ref((float)(kTol * kp), (float)kTol)) atomicAnd(flag, 0);
    }
}
// theta matrix diagonal from a row-major Qd (computeTheta, :503-519): rows in parallel
__global__ void k_theta_rowmajor(const float* __restrict__ Qd, int N, float* __restrict__ theta_mat) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    float s = 0.0f;
    for (int k = 0; k < N; ++k) s += max_ref(0.0f, -Qd[(size_t)i * N + k]) * 1.0f;
    theta_mat[(size_t)i * N + i] = max_ref(s, 5.0f);
}
// computeCost's scalar tail (PQP_CPU.c:655-661): J = 0; J += 0.5*q; J += f; J += M/2
__global__ void k_cost_finish(const float* __restrict__ quad, const float* __restrict__ lin,
                              const float* __restrict__ Mc, float* __restrict__ J) {
    float j = 0.0f;
    j = (float)((double)j + 0.5 * (double)quad[0]);
    j += lin[0];
    j += Mc[0] / 2;
    J[0] = j;
}
// computeMp's accumulation (PQP_CPU.c:397-425): terms t[0..4] then Mp6, each halved
__global__ void k_mp_finish(const float* __restrict__ t, const float* __restrict__ Mp6, float* __restrict__ Mp,
                            long long sMp6 = 0) {
    t += (size_t)blockIdx.x * 5;  // problem blockIdx.x of a batch
    Mp6 += blockIdx.x * sMp6;
    Mp += blockIdx.x;
    float m = 0.0f;
    for (int s = 0; s < 5; ++s) m += t[s] / 2;
    m += Mp6[0] / 2;
    Mp[0] = m;
}

// Gauss_Jordan (PQP_CPU.c:251-326) in one workgroup.  aug is n x 2n scratch
// (global).  Row updates of one pivot are independent (row j reads only rows
// i and j), so computing every factor first and then updating all rows in
// parallel is the reference's arithmetic exactly.
__global__ void __launch_bounds__(256) k_gauss_jordan(const float* __restrict__ A, float* __restrict__ aug,
                                                      float* __restrict__ fac, float* __restrict__ res, int n) {
    const int tid = threadIdx.x, w = 2 * n;
    {  // problem blockIdx.x of a batch
        const size_t b = blockIdx.x;
        A += b * n * n;
        res += b * n * n;
        aug += b * n * w;
        fac += b * n;
    }
    for (int e = tid; e < n * w; e += 256) {
        const int r = e / w, c = e % w;
        aug[e] = (c < n) ? A[(size_t)r * n + c] : ((c == n + r) ? 1.0f : 0.0f);
    }
    __syncthreads();
    __shared__ int do_swap;
    for (int r = n - 1; r > 0; --r) {  // one bubble pass on column 0 (:280-289)
        if (tid == 0) do_swap = aug[(size_t)(r - 1) * w] < aug[(size_t)r * w];
        __syncthreads();
        if (do_swap)
            for (int c = tid; c < w; c += 256) {
                const float t = aug[(size_t)r * w + c];
                aug[(size_t)r * w + c] = aug[(size_t)(r - 1) * w + c];
                aug[(size_t)(r - 1) * w + c] = t;
            }
        __syncthreads();
    }
    for (int p = 0; p < n; ++p) {  // :291-305
        for (int r = tid; r < n; r += 256) fac[r] = aug[(size_t)r * w + p] / aug[(size_t)p * w + p];
        __syncthreads();
        for (int e = tid; e < n * w; e += 256) {
            const int r = e / w, c = e % w;
            if (r != p) aug[e] -= aug[(size_t)p * w + c] * fac[r];
        }
        __syncthreads();
    }
    for (int r = tid; r < n; r += 256) fac[r] = aug[(size_t)r * w + r];  // :307-314
    __syncthreads();
    for (int e = tid; e < n * w; e += 256) {
        const int r = e / w;
        aug[e] = aug[e] / fac[r];
    }
    __syncthreads();
    for (int e = tid; e < n * n; e += 256) {
        const int r = e / n, c = e % n;
        res[e] = aug[(size_t)r * w + n + c];
    }
}

// Problem b of a batched SolveArgs (contiguous per-problem arrays).
__device__ __forceinline__ SolveArgs problem_at(SolveArgs A, int b) {
    const size_t N = A.N, M = A.M;
    A.QdT = A.QdT ? A.QdT + b * N * A.ldq : nullptr;
    A.theta = A.theta ? A.theta + b * N : nullptr;
    A.Qd += b * N * N;
    A.Fd += b * N;
    A.Md = A.Md ? A.Md + b : nullptr;
    A.Qp = A.Qp ? A.Qp + b * M * M : nullptr;
    A.Qinv = A.Qinv ? A.Qinv + b * M * M : nullptr;
    A.Fp = A.Fp ? A.Fp + b * M : nullptr;
    A.Mp = A.Mp ? A.Mp + b : nullptr;
    A.Gp = A.Gp ? A.Gp + b * N * M : nullptr;
    A.GpT = A.GpT ? A.GpT + b * N * M : nullptr;
    A.QinvT = A.QinvT ? A.QinvT + b * M * M : nullptr;
    A.Kp = A.Kp ? A.Kp + b * N : nullptr;
    A.Y += b * N;
    A.U = A.U ? A.U + b * M : nullptr;
    return A;
}

// <solve-single> (bench.py hashes the text up to </solve-single>: k_solve_single PMC records are keyed by it)
// ---------------------------------------------------------------------------
// k_solve_single: the whole solveQuadraticDual (PQP_CPU.c:694-750) in ONE
// persistent workgroup: terminate() before every update, bit-exact, no host
// round trip per iteration.  Resumable in chunks (state in SolveState) so no
// single launch runs unbounded.
// ---------------------------------------------------------------------------
// s = sum_k a[k*astride] * b[k] in the reference's order (k = 0..n-1 from
// +0.0f, product rounded before each add).  The operands of U consecutive
// terms are loaded before any of them is used, so LDS/L2 latency overlaps
// instead of serializing behind the add chain; the add order is unchanged.
template <int U = 8>
__device__ __forceinline__ float seq_dot(const float* a, int astride, const float* b, int n) {
    float s = 0.0f;
    int k = 0;
    for (; k + U <= n; k += U) {
        float av[U], bv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            av[j] = a[(size_t)(k + j) * astride];
            bv[j] = b[k + j];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) s += av[j] * bv[j];
    }
    for (; k < n; ++k) s += a[(size_t)k * astride] * b[k];
    return s;
}

// updateY2 (PQP_CPU.c:603-618) of rows i = tid, tid + NT, ... from `cur`
// into `nxt`, one lane per row over the column-major QdT.  Split entries in
// "max form": (q<0 ? 0 : q)*y and (q>0 ? 0 : -q)*y off the diagonal
// (bit-identical to (max(0,+-q)+0.0f)*y), the stored literal
// (max(0,+-q_ii)+theta_i) on it.  FUSE (Qd bit-symmetric, so QdT's column i
// is also Qd's column i): the same stream also gives tq[i] = sum_k Y_k Qd[k][i]
// in k order -- terminate()'s Y'Qd row (computeCost :648-653, :110) -- with
// a third sequential sum, instead of a second pass over Qd.
constexpr int kSU = 16;  // k per batch of loads in flight (per lane) in k_solve_single's passes
template <int NT, bool FUSE>
__device__ __forceinline__ void single_update(const SolveArgs& A, const float* __restrict__ cur,
                                              float* __restrict__ nxt, float* __restrict__ tq) {
    const int N = A.N, ldq = A.ldq;
    for (int i = threadIdx.x; i < N; i += NT) {
        float ap = 0.0f, an = 0.0f, aq = 0.0f;
        const float thi = A.theta[i];
        const float qii = A.QdT[(size_t)i * ldq + i];
        const float dp = max_ref(0.0f, qii) + 1.0f * thi, dn = max_ref(0.0f, -qii) + 1.0f * thi;
        const float* col = A.QdT + i;
        int k = 0;
        for (; k + kSU <= N; k += kSU) {
            float q[kSU], yv[kSU];
#pragma unroll
            for (int j = 0; j < kSU; ++j) {
                q[j] = col[(size_t)(k + j) * ldq];
                yv[j] = cur[k + j];
            }
#pragma unroll
            for (int j = 0; j < kSU; ++j) {
                const bool d = (k + j == i);
                const float qp = d ? dp : ((q[j] < 0.0f) ? 0.0f : q[j]);
                const float qn = d ? dn : ((q[j] > 0.0f) ? 0.0f : -q[j]);
                ap += qp * yv[j];
                an += qn * yv[j];
                if constexpr (FUSE) aq += yv[j] * q[j];  // Y'Qd :110, k in order
            }
        }
        for (; k < N; ++k) {
            const float q = col[(size_t)k * ldq], yk = cur[k];
            const bool d = (k == i);
            ap += (d ? dp : ((q < 0.0f) ? 0.0f : q)) * yk;
            an += (d ? dn : ((q > 0.0f) ? 0.0f : -q)) * yk;
            if constexpr (FUSE) aq += yk * q;
        }
        const float f = A.Fd[i];
        const float num = an + 1.0f * max_ref(0.0f, -f);
        const float den = ap + 1.0f * max_ref(0.0f, f);
        nxt[i] = num / den * cur[i];
        if constexpr (FUSE) tq[i] = aq;
    }
}

// ---- wide-load forms (VEC: N and M multiples of 4; the arrays 16-byte
// aligned per problem).  Each lane's sums keep the reference's k order; the
// loads are 8 or 16 bytes per lane, so a wave moves 2-4x the bytes per
// instruction and a pass needs 2-4x fewer dependent load batches.
typedef float sf2 __attribute__((ext_vector_type(2)));
typedef float sf4 __attribute__((ext_vector_type(4)));
template <int V> struct SVec;
template <> struct SVec<2> { typedef sf2 t; };
template <> struct SVec<4> { typedef sf4 t; };

// s[c] = sum_k A[k * lda + c] * x[k], c < V (V adjacent columns of a
// row-major matrix), k = 0..n-1 in order, U rows of loads in flight (the
// matrix is streamed once per pass: non-temporal loads)
template <int V, int U>
__device__ __forceinline__ void col_dotv(const float* __restrict__ A, int lda, const float* x, int n, float (&s)[V]) {
    typedef typename SVec<V>::t vt;
#pragma unroll
    for (int c = 0; c < V; ++c) s[c] = 0.0f;
    int k = 0;
    for (; k + U <= n; k += U) {
        vt a[U];
        float xv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            a[j] = __builtin_nontemporal_load(reinterpret_cast<const vt*>(A + (size_t)(k + j) * lda));
            xv[j] = x[k + j];
        }
#pragma unroll
        for (int j = 0; j < U; ++j)
#pragma unroll
            for (int c = 0; c < V; ++c) s[c] += a[j][c] * xv[j];
    }
    for (; k < n; ++k) {
        const vt a = *reinterpret_cast<const vt*>(A + (size_t)k * lda);
#pragma unroll
        for (int c = 0; c < V; ++c) s[c] += a[c] * x[k];
    }
}

// s = sum_k a[k] * x[k] over a contiguous row (16-byte aligned, as is x),
// k in order, 4 terms per load, U loads in flight
template <int U>
__device__ __forceinline__ float row_dot4(const float* __restrict__ a, const float* x, int n) {
    float s = 0.0f;
    int k = 0;
    for (; k + 4 * U <= n; k += 4 * U) {
        sf4 av[U], xv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            av[j] = *reinterpret_cast<const sf4*>(a + k + 4 * j);
            xv[j] = *reinterpret_cast<const sf4*>(x + k + 4 * j);
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            s += av[j].x * xv[j].x;
            s += av[j].y * xv[j].y;
            s += av[j].z * xv[j].z;
            s += av[j].w * xv[j].w;
        }
    }
    for (; k < n; ++k) s += a[k] * x[k];
    return s;
}

// single_update with four adjacent rows per lane (16-byte loads of QdT)
constexpr int kSU4 = 8;
template <int NT, bool FUSE, int SU = kSU4>
__device__ __forceinline__ void single_update4(const SolveArgs& A, const float* __restrict__ cur,
                                               float* __restrict__ nxt, float* __restrict__ tq) {
    const int N = A.N, ldq = A.ldq;
    for (int i0 = 4 * threadIdx.x; i0 < N; i0 += 4 * NT) {
        float ap[4] = {}, an[4] = {}, aq[4] = {}, dp[4], dn[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + r;
            const float thi = i < N ? A.theta[i] : 0.0f;
            const float qii = i < N ? A.QdT[(size_t)i * ldq + i] : 0.0f;
            dp[r] = max_ref(0.0f, qii) + 1.0f * thi;
            dn[r] = max_ref(0.0f, -qii) + 1.0f * thi;
        }
        const float* col = A.QdT + i0;
        int k = 0;
        for (; k + SU <= N; k += SU) {
            sf4 q[SU];
            float yv[SU];
#pragma unroll
            for (int j = 0; j < SU; ++j) {
                q[j] = __builtin_nontemporal_load(reinterpret_cast<const sf4*>(col + (size_t)(k + j) * ldq));
                yv[j] = cur[k + j];
            }
#pragma unroll
            for (int j = 0; j < SU; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const bool d = (k + j == i0 + r);
                    const float qp = d ? dp[r] : ((q[j][r] < 0.0f) ? 0.0f : q[j][r]);
                    const float qn = d ? dn[r] : ((q[j][r] > 0.0f) ? 0.0f : -q[j][r]);
                    ap[r] += qp * yv[j];
                    an[r] += qn * yv[j];
                    if constexpr (FUSE) aq[r] += yv[j] * q[j][r];  // Y'Qd :110, k in order
                }
        }
        for (; k < N; ++k) {
            const sf4 q = *reinterpret_cast<const sf4*>(col + (size_t)k * ldq);
            const float yk = cur[k];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool d = (k == i0 + r);
                ap[r] += (d ? dp[r] : ((q[r] < 0.0f) ? 0.0f : q[r])) * yk;
                an[r] += (d ? dn[r] : ((q[r] > 0.0f) ? 0.0f : -q[r])) * yk;
                if constexpr (FUSE) aq[r] += yk * q[r];
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + r;
            if (i < N) {
                const float f = A.Fd[i];
                const float num = an[r] + 1.0f * max_ref(0.0f, -f);
                const float den = ap[r] + 1.0f * max_ref(0.0f, f);
                nxt[i] = num / den * cur[i];
                if constexpr (FUSE) tq[i] = aq[r];
            }
        }
    }
}

template <int NT, bool VEC, int MINB = 1>
__global__ void __launch_bounds__(NT, MINB) k_solve_single(SolveArgs A0, SolveState* __restrict__ st0) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SolveArgs A = problem_at(A0, blockIdx.x);
    SolveState* st = st0 + blockIdx.x;
    if (st->status == kStatusDone || st->status == kStatusCapped) return;  // finished in an earlier launch
    const int N = A.N, M = A.M, ldq = A.ldq;
    // the fused form keeps Y_{h+1} in nxt through terminate(), so the Fd.Y
    // terms get a buffer of their own; otherwise they use nxt (free until the
    // update), and the workgroup needs less LDS (more of them per CU)
    float* ya = lds;              // ldq
    float* yb = ya + ldq;         // ldq
    float* tq = yb + ldq;         // N   (Y'Qd row, Jd)
    float* fyb = tq + ldq;        // N   (Fd.Y terms; fused form only)
    float* tM = (A.sym ? fyb + ldq : fyb);  // M   (Gp'Y + Fp)
    float* Us = tM + A.ldm;       // M   (U)
    float* tu = Us + A.ldm;       // M   (U'Qp row, Jp)
    __shared__ float s_J[2];
    const int tid = threadIdx.x;
    // converge mode of a problem whose Qd is bit-symmetric: the update to
    // Y_{h+1} runs first, speculatively, fused with terminate(Y_h)'s Y'Qd; it
    // is dropped when terminate(Y_h) stops (every value is the reference's)
    // (taken only after a feasible terminate(): an infeasible one stops at
    // checkFeas and never reads Qd, so fusing would only add work)
    const bool fuse_ok = A.mode == kModeConverge && A.sym && A.sym[blockIdx.x];
    bool was_feasible = false;

    long long h = st->h;  // printed h of the current iterate
    for (int i = tid; i < ldq; i += NT) {
        ya[i] = (i < N) ? (st->resume ? A.Y[i] : 1000.0f) : 0.0f;
        yb[i] = 0.0f;
    }
    __syncthreads();
    float* cur = ya;
    float* nxt = yb;
    int status = kStatusContinue;
    long long done_here = 0;
    for (;;) {
        const bool fuse = fuse_ok && was_feasible;
        float* fy = A.sym ? fyb : nxt;
        if (fuse) {
            if constexpr (VEC) single_update4<NT, true>(A, cur, nxt, tq);
            else single_update<NT, true>(A, cur, nxt, tq);
            __syncthreads();
        }
        if (A.mode != kModeFixed) {
            // ---- terminate(Y)  PQP_CPU.c:673-687 ----
            // computeUfromY :352-360
            if constexpr (VEC) {
                for (int j = 2 * tid; j < M; j += 2 * NT) {
                    float t[2];
                    col_dotv<2, kSU>(A.Gp + j, M, cur, N, t);
                    tM[j] = t[0] + 1.0f * A.Fp[j];
                    tM[j + 1] = t[1] + 1.0f * A.Fp[j + 1];
                }
            } else {
                for (int j = tid; j < M; j += NT) tM[j] = seq_dot<kSU>(A.Gp + j, M, cur, N) + 1.0f * A.Fp[j];
            }
            __syncthreads();
            // row access of Qp_inv / Gp through their transposes when given (lane
            // i walks column i of QinvT / GpT: coalesced), else row by row
            // (VEC with the transposes: four adjacent rows per lane, 16-byte
            // coalesced loads of the transposed copy, each row's sum in j order)
            if (VEC && A.QinvT && M >= 4 * NT) {
                for (int i0 = 4 * tid; i0 < M; i0 += 4 * NT) {
                    float t[4];
                    col_dotv<4, kSU4>(A.QinvT + i0, M, tM, M, t);
#pragma unroll
                    for (int c = 0; c < 4; ++c) Us[i0 + c] = -t[c];
                }
            } else if (VEC && A.QinvT) {  // M < 4 NT: two rows per lane keep more lanes loading
                for (int i0 = 2 * tid; i0 < M; i0 += 2 * NT) {
                    float t[2];
                    col_dotv<2, kSU>(A.QinvT + i0, M, tM, M, t);
                    Us[i0] = -t[0];
                    Us[i0 + 1] = -t[1];
                }
            } else {
                for (int i = tid; i < M; i += NT)
                    Us[i] = -(A.QinvT ? seq_dot<kSU>(A.QinvT + i, M, tM, M)
                              : VEC   ? row_dot4<4>(A.Qinv + (size_t)i * M, tM, M)
                                      : seq_dot<kSU>(A.Qinv + (size_t)i * M, 1, tM, M));
            }
            __syncthreads();
            // checkFeas :632-641
            int bad = 0;
            int infeasible = 0;
            if (VEC && A.GpT && A.feas_split && N > NT) {
                // first NT rows (one per lane), then the rest only if none of them
                // is over its bound: terminate() returns 0 on ANY row over its
                // bound (:677), so a violation among the first rows decides the
                // iterate and the other rows' sums change nothing observable
                // (checkFeas's products are used for nothing else)
                {
                    const float s0 = seq_dot<kSU>(A.GpT + tid, N, Us, M);
                    const float kp = A.Kp[tid];
                    if (s0 > kp + max_ref((float)(kTol * kp), (float)kTol)) bad = 1;
                }
                infeasible = __syncthreads_or(bad);
                if (!infeasible) {
                    for (int i0 = NT + 4 * tid; i0 < N; i0 += 4 * NT) {
                        float t[4];
                        col_dotv<4, kSU4>(A.GpT + i0, N, Us, M, t);
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const float kp = A.Kp[i0 + c];
                            if (t[c] > kp + max_ref((float)(kTol * kp), (float)kTol)) bad = 1;
                        }
                    }
                }
            } else if (VEC && A.GpT) {
                for (int i0 = 4 * tid; i0 < N; i0 += 4 * NT) {
                    float t[4];
                    col_dotv<4, kSU4>(A.GpT + i0, N, Us, M, t);
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float kp = A.Kp[i0 + c];
                        if (t[c] > kp + max_ref((float)(kTol * kp), (float)kTol)) bad = 1;
                    }
                }
            } else {
                for (int i = tid; i < N; i += NT) {
                    const float s = A.GpT ? seq_dot<kSU>(A.GpT + i, N, Us, M)
                                    : VEC   ? row_dot4<4>(A.Gp + (size_t)i * M, Us, M)
                                            : seq_dot<kSU>(A.Gp + (size_t)i * M, 1, Us, M);
                    const float kp = A.Kp[i];
                    if (s > kp + max_ref((float)(kTol * kp), (float)kTol)) bad = 1;
                }
            }
            infeasible = __syncthreads_or(bad);
            was_feasible = !infeasible;
            int stop = 0;
            if (!infeasible) {
                // computeCost(Y, Qd, Fd, Md) and computeCost(U, Qp, Fp, Mp) :648-666
                if constexpr (VEC) {
                    if (!fuse)
                        for (int j = 4 * tid; j < N; j += 4 * NT) {
                            float t[4];
                            col_dotv<4, kSU4>(A.Qd + j, N, cur, N, t);
#pragma unroll
                            for (int c = 0; c < 4; ++c) tq[j + c] = t[c];
                        }
                    for (int j = 2 * tid; j < M; j += 2 * NT) {
                        float t[2];
                        col_dotv<2, kSU>(A.Qp + j, M, Us, M, t);
                        tu[j] = t[0];
                        tu[j + 1] = t[1];
                    }
                } else {
                    if (!fuse)
                        for (int j = tid; j < N; j += NT) tq[j] = seq_dot<kSU>(A.Qd + j, N, cur, N);
                    for (int j = tid; j < M; j += NT) tu[j] = seq_dot<kSU>(A.Qp + j, M, Us, M);
                }
                __syncthreads();
                // the dot products' terms formed in parallel into LDS (the
                // row buffers in place; Fd.Y into fy and Fp.U into tM), then
                // summed in k order by one lane each -- one lane reading Fd
                // from global memory term by term was the slowest part of an
                // iteration
                for (int j = tid; j < N; j += NT) {
                    tq[j] = tq[j] * cur[j];
                    fy[j] = A.Fd[j] * cur[j];
                }
                for (int j = tid; j < M; j += NT) {
                    tu[j] = tu[j] * Us[j];
                    tM[j] = A.Fp[j] * Us[j];
                }
                __syncthreads();
                const int jt = (NT >= 128) ? 64 : 1;  // second scalar chain on another wave
                if (tid == 0 || tid == jt) {
                    const bool dual = (tid == 0);
                    const float* qv = dual ? tq : tu;
                    const float* lv = dual ? fy : tM;
                    const int n = dual ? N : M;
                    // (Z'Q).Z :652-655 and F'Z :656-657, each in k order; the two
                    // chains interleaved (read 16 bytes at a time where N, M are
                    // multiples of 4 and the vectors 16-byte aligned)
                    float quad = 0.0f, lin = 0.0f;
                    int k = 0;
                    if constexpr (VEC)
                        for (; k + 4 <= n; k += 4) {
                            const sf4 a = *reinterpret_cast<const sf4*>(qv + k), b = *reinterpret_cast<const sf4*>(lv + k);
                            quad += a.x;
                            lin += b.x;
                            quad += a.y;
                            lin += b.y;
                            quad += a.z;
                            lin += b.z;
                            quad += a.w;
                            lin += b.w;
                        }
                    for (; k < n; ++k) {
                        quad += qv[k];
                        lin += lv[k];
                    }
                    float J = 0.0f;
                    J = (float)((double)J + 0.5 * (double)quad);
                    J += lin;
                    J += (dual ? A.Md[0] : A.Mp[0]) / 2;
                    s_J[dual ? 1 : 0] = J;
                }
                __syncthreads();
                const float Jp = s_J[0], Jd = s_J[1];
                stop = 1;
                if (Jp > -Jd) stop = 0;
                if ((double)(Jp + Jd) > kTol) stop = 0;
                if ((double)(Jp + Jd) / fabs((double)Jd) > kTol) stop = 0;
                if (tid == 0) {
                    st->Jp = Jp;
                    st->Jd = Jd;
                    st->have_costs = 1;
                }
            }
            if (A.mode == kModeTerminate) {
                if (tid == 0) st->last_stop = stop;
                status = kStatusDone;
                break;
            }
            if (stop) {
                status = kStatusDone;
                break;
            }
            if (A.max_updates > 0 && h - 1 >= A.max_updates) {
                status = kStatusCapped;
                break;
            }
        } else {
            if (h >= A.num_iter) {  // while(h < NUM_ITER)
                status = kStatusDone;
                break;
            }
        }
        if (done_here >= A.chunk) {
            status = kStatusContinue;
            break;
        }
        // ---- updateY2  PQP_CPU.c:603-618 (one lane per row) ----
        if (!fuse) {
            if constexpr (VEC) single_update4<NT, false>(A, cur, nxt, nullptr);
            else single_update<NT, false>(A, cur, nxt, nullptr);
        }
        __syncthreads();
        float* t = cur;
        cur = nxt;
        nxt = t;
        ++h;
        ++done_here;
    }
    for (int i = tid; i < N; i += NT) A.Y[i] = cur[i];
    if (A.mode != kModeFixed)
        for (int i = tid; i < M; i += NT) A.U[i] = Us[i];
    if (tid == 0) {
        st->h = h;
        st->status = status;
        st->resume = 1;
        if (status == kStatusContinue && A.pending) atomicAdd(A.pending, 1);
    }
}

// </solve-single>

// <solve-pipe> (bench.py hashes the text up to </solve-pipe>: k_solve_pipe PMC records are keyed by it)
// ---------------------------------------------------------------------------
// k_solve_pipe: converge mode of solveQuadraticDual (PQP_CPU.c:694-750), one
// workgroup per problem from global memory, like k_solve_single, but with Gp
// read ONCE per iteration instead of twice.  terminate(Y_h) needs Gp'Y_h
// (computeUfromY :355) and Gp U_h (checkFeas :636); the update to Y_{h+1}
// needs only Y_h (updateY2 :603-618), so it runs first, speculatively, and
// one pass over Gp then gives checkFeas(h)'s rows AND Gp'Y_{h+1}, i.e. the
// next iterate's computeUfromY:
//   phase X  Y_{h+1} = updateY2(Y_h) (+ Y_h'Qd fused when Qd is bit-symmetric
//            and the previous iterate was feasible), U_h = -Qp_inv tM_h
//   phase Y  Gp in 128 x 96 tiles, each staged once through LDS: lane r of
//            waves 0 and 2 sums row r's terms Gp[i][j] U_h[j] (j in order,
//            the partial carried across the tiles of a row block), lane c of
//            waves 1 and 3 column c's terms Gp[i][j] Y_{h+1}[i] (i in order,
//            the partial carried in LDS across row blocks); the next tile's
//            loads are in flight meanwhile (variants: 64 x 64 tiles on waves
//            0 and 1, two or four tiles ahead)
//   then     checkFeas(h) from the row sums; computeCost on a feasible iterate
//            as k_solve_single does; Y_{h+1}, tM_{h+1} dropped when h stops.
// Every sum has the reference's operands and order, so every value is the
// reference's.  Per iteration Qd + Qp_inv + Gp (+ Qp when feasible) are read
// once each: 4N^2 + 4M^2 + 4NM (+ 4M^2) bytes, against k_solve_single's two
// passes over Gp.  Needs the wide-load conditions and Qp_inv' (QinvT).
// ---------------------------------------------------------------------------
constexpr int kPipeTR = 64, kPipeTC = 64, kPipeTS = kPipeTC + 1;  // tile rows, columns, LDS row stride
// BIG: one 128 x 96 tile at a time (single LDS slot, the next tile's loads in
// registers): rows summed on waves 0 and 2, columns on waves 1 and 3, so every
// wave runs a chain and a step holds 3x the terms of a 64 x 64 tile for 2x the
// chain length
constexpr int kPipeBR = 128, kPipeBC = 96, kPipeBS = kPipeBC + 1, kPipeBQ = kPipeBR * kPipeBC / 4 / 256;
__host__ __device__ inline size_t pipe_tile_floats(bool big = false) {
    return big ? (size_t)kPipeBR * kPipeBS : (size_t)2 * kPipeTR * kPipeTS;
}

template <int NT, int PD, int SU, int MINB, bool BIG = false>
__global__ void __launch_bounds__(NT, MINB) k_solve_pipe(SolveArgs A0, SolveState* __restrict__ st0) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SolveArgs A = problem_at(A0, blockIdx.x);
    SolveState* st = st0 + blockIdx.x;
    if (st->status == kStatusDone || st->status == kStatusCapped) return;  // finished in an earlier launch
    const int N = A.N, M = A.M, ldq = A.ldq, ldm = A.ldm;
    float* ya = lds;            // ldq   Y_h / Y_{h+1}
    float* yb = ya + ldq;       // ldq
    float* tq = yb + ldq;       // ldq   Y_h'Qd (Jd)
    float* tMa = tq + ldq;      // ldm   tM_h = Gp'Y_h + Fp / tM_{h+1}
    float* tMb = tMa + ldm;     // ldm
    float* Us = tMb + ldm;      // ldm   U_h
    float* tile = Us + ldm;     // 2 x TR x TS (phase Y), then fy, tu, fu (costs)
    float* fy = tile;           // ldq   Fd.Y terms
    float* tu = fy + ldq;       // ldm   U'Qp row, then its terms
    float* fu = tu + ldm;       // ldm   Fp.U terms
    __shared__ float s_J[2];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const bool fuse_ok = A.sym && A.sym[blockIdx.x];
    // a launch's first iterate fuses Y'Qd as if the previous one was feasible:
    // resumed converge solves (chunks of a long solve) then need no separate
    // pass over Qd for Jd, and an infeasible first iterate costs only the
    // fused sum's VALU work
    bool was_feasible = true;
    constexpr int TR = BIG ? kPipeBR : kPipeTR, TC = BIG ? kPipeBC : kPipeTC;
    const int nI = (N + TR - 1) / TR, nJ = (M + TC - 1) / TC, nT = nI * nJ;

    long long h = st->h;
    for (int i = tid; i < ldq; i += NT) {
        ya[i] = (i < N) ? (st->resume ? A.Y[i] : 1000.0f) : 0.0f;
        yb[i] = 0.0f;
    }
    __syncthreads();
    float* cur = ya;
    float* nxt = yb;
    // tM_h for the launch's first iterate (computeUfromY :355-356)
    for (int j = 2 * tid; j < M; j += 2 * NT) {
        float t[2];
        col_dotv<2, kSU>(A.Gp + j, M, cur, N, t);
        tMa[j] = t[0] + 1.0f * A.Fp[j];
        tMa[j + 1] = t[1] + 1.0f * A.Fp[j + 1];
    }
    __syncthreads();
    float* tMc = tMa;  // tM of the current iterate
    float* tMn = tMb;  // tM of the next
    int status = kStatusContinue;
    long long done_here = 0;
    // timing trace (pqp_tune_trace "mid"): thread 0's phase totals in shader
    // cycles -- X (update, U), Y (the pass over Gp), the costs and decision
    const bool tr = A0.trace && (int)blockIdx.x < A0.trace_n;  // uniform: the totals stay in SGPRs
    unsigned long long t0 = 0, acc_ph[3] = {0, 0, 0}, n_it = 0;
    // tile t = (I, J), I = t / nJ: lane l loads rows (l >> 4) + 16 s, s < 4,
    // columns 4 (l & 15) .. +3 (16 lanes per 256-byte row segment)
    auto load_tile = [&](int t, sf4 (&r)[4]) {
        const int I = t / nJ, J = t - I * nJ;
        const int col = J * kPipeTC + 4 * (tid & 15);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int row = I * kPipeTR + (tid >> 4) + 16 * s;
            r[s] = (row < N && col < M)
                       ? __builtin_nontemporal_load(reinterpret_cast<const sf4*>(A.Gp + (size_t)row * M + col))
                       : sf4{0.0f, 0.0f, 0.0f, 0.0f};
        }
    };
    for (;;) {
        // this iterate breaks before its update whatever terminate() says:
        // no speculative update or next tM
        const bool last = done_here >= A.chunk || (A.max_updates > 0 && h - 1 >= A.max_updates);
        const bool fuse = fuse_ok && was_feasible && !last;
        if (tr) t0 = __builtin_amdgcn_s_memtime();
        // ---- phase X ----
        if (!last) {
            if (fuse) single_update4<NT, true, SU>(A, cur, nxt, tq);
            else single_update4<NT, false, SU>(A, cur, nxt, nullptr);
        }
        for (int i0 = 2 * tid; i0 < M; i0 += 2 * NT) {  // computeUfromY :357-359
            float t[2];
            col_dotv<2, kSU>(A.QinvT + i0, M, tMc, M, t);
            Us[i0] = -t[0];
            Us[i0 + 1] = -t[1];
        }
        // ---- phase Y: one pass over Gp ----
        int bad = 0;
        if constexpr (BIG) {
            // tile t = (I, J): lane l loads chunk e = l + 256 s of the tile's
            // 128 rows x 24 16-byte chunks (a row's 384 bytes by 24 lanes)
            auto load_big = [&](int t, sf4 (&r)[kPipeBQ]) {
                const int I = t / nJ, J = t - I * nJ;
#pragma unroll
                for (int s = 0; s < kPipeBQ; ++s) {
                    const int e = tid + 256 * s, rr = e / 24, c4 = e - rr * 24;
                    const int row = I * kPipeBR + rr, col = J * kPipeBC + 4 * c4;
                    r[s] = (row < N && col < M)
                               ? __builtin_nontemporal_load(reinterpret_cast<const sf4*>(A.Gp + (size_t)row * M + col))
                               : sf4{0.0f, 0.0f, 0.0f, 0.0f};
                }
            };
            sf4 rb[kPipeBQ];
            load_big(0, rb);
            __syncthreads();  // Y_{h+1}, U_h complete; the tile area is free
            if (tr) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                acc_ph[0] += t - t0;
                t0 = t;
            }
            float racc = 0.0f;  // waves 0 and 2: row sum of the current row block
            for (int t = 0; t < nT; ++t) {
#pragma unroll
                for (int s = 0; s < kPipeBQ; ++s) {
                    const int e = tid + 256 * s, rr = e / 24, c4 = e - rr * 24;
                    float* d = tile + rr * kPipeBS + 4 * c4;
                    d[0] = rb[s].x;
                    d[1] = rb[s].y;
                    d[2] = rb[s].z;
                    d[3] = rb[s].w;
                }
                if (t + 1 < nT) load_big(t + 1, rb);
                __syncthreads();  // tile t staged
                const int I = t / nJ, J = t - I * nJ;
                const int nr = min(kPipeBR, N - I * kPipeBR), nc = min(kPipeBC, M - J * kPipeBC);
                if ((wave & 1) == 0) {
                    // checkFeas :636: gu[i] = sum_j Gp[i][j] U[j], j in order
                    const int rl = (wave >> 1) * 64 + lane;
                    if (J == 0) racc = 0.0f;
                    if (rl < nr) {
                        const float* tr = tile + rl * kPipeBS;
                        const float* u = Us + J * kPipeBC;
                        float s = racc;
                        int c = 0;
                        for (; c + 8 <= nc; c += 8) {
                            float g[8];
#pragma unroll
                            for (int e = 0; e < 8; ++e) g[e] = tr[c + e];
                            const sf4 u0 = *reinterpret_cast<const sf4*>(u + c), u1 = *reinterpret_cast<const sf4*>(u + c + 4);
#pragma unroll
                            for (int e = 0; e < 8; ++e) s += g[e] * (e < 4 ? u0[e] : u1[e - 4]);
                        }
                        for (; c < nc; ++c) s += tr[c] * u[c];
                        racc = s;
                        if (J == nJ - 1) {  // compare :338-341
                            const float kp = A.Kp[I * kPipeBR + rl];
                            if (s > kp + max_ref((float)(kTol * kp), (float)kTol)) bad = 1;
                        }
                    }
                } else if (!last) {
                    // Gp'Y_{h+1} :355: tmp[j] = sum_i Gp[i][j] Y[i], i in order
                    const int cl = (wave >> 1) * 64 + lane;
                    if (cl < nc) {
                        const int col = J * kPipeBC + cl;
                        const float* y = nxt + I * kPipeBR;
                        float s = (I == 0) ? 0.0f : tMn[col];
                        int r = 0;
                        for (; r + 8 <= nr; r += 8) {
                            float g[8];
#pragma unroll
                            for (int e = 0; e < 8; ++e) g[e] = tile[(r + e) * kPipeBS + cl];
                            const sf4 y0 = *reinterpret_cast<const sf4*>(y + r), y1 = *reinterpret_cast<const sf4*>(y + r + 4);
#pragma unroll
                            for (int e = 0; e < 8; ++e) s += g[e] * (e < 4 ? y0[e] : y1[e - 4]);
                        }
                        for (; r < nr; ++r) s += tile[r * kPipeBS + cl] * y[r];
                        tMn[col] = (I == nI - 1) ? s + 1.0f * A.Fp[col] : s;  // matrixAdd :356
                    }
                }
                __syncthreads();  // the slot is free for tile t + 1
            }
        } else {
        sf4 rq[PD][4];  // the next PD tiles' loads in flight
#pragma unroll
        for (int d = 0; d < PD; ++d)
            if (d < nT) load_tile(d, rq[d]);
        __syncthreads();  // Y_{h+1}, U_h complete; the tile area is free
        if (tr) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            acc_ph[0] += t - t0;
            t0 = t;
        }
        float racc = 0.0f;  // wave 0: row sum of the current row block
        for (int t = 0; t < nT; ++t) {
            float* tl = tile + (t & 1) * (kPipeTR * kPipeTS);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                float* d = tl + ((tid >> 4) + 16 * s) * kPipeTS + 4 * (tid & 15);
                d[0] = rq[0][s].x;
                d[1] = rq[0][s].y;
                d[2] = rq[0][s].z;
                d[3] = rq[0][s].w;
            }
#pragma unroll
            for (int d = 0; d + 1 < PD; ++d)
#pragma unroll
                for (int s = 0; s < 4; ++s) rq[d][s] = rq[d + 1][s];
            if (t + PD < nT) load_tile(t + PD, rq[PD - 1]);
            __syncthreads();  // tile t staged (tile t - 2's readers are past the previous barrier)
            const int I = t / nJ, J = t - I * nJ;
            const int nr = min(kPipeTR, N - I * kPipeTR), nc = min(kPipeTC, M - J * kPipeTC);
            if (wave == 0) {
                // checkFeas :636: gu[i] = sum_j Gp[i][j] U[j], j in order
                if (J == 0) racc = 0.0f;
                if (lane < nr) {
                    const float* tr = tl + lane * kPipeTS;
                    const float* u = Us + J * kPipeTC;
                    float s = racc;
                    int c = 0;
                    for (; c + 8 <= nc; c += 8) {
                        float g[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) g[e] = tr[c + e];
                        const sf4 u0 = *reinterpret_cast<const sf4*>(u + c), u1 = *reinterpret_cast<const sf4*>(u + c + 4);
#pragma unroll
                        for (int e = 0; e < 8; ++e) s += g[e] * (e < 4 ? u0[e] : u1[e - 4]);
                    }
                    for (; c < nc; ++c) s += tr[c] * u[c];
                    racc = s;
                    if (J == nJ - 1) {  // compare :338-341
                        const float kp = A.Kp[I * kPipeTR + lane];
                        if (s > kp + max_ref((float)(kTol * kp), (float)kTol)) bad = 1;
                    }
                }
            } else if (wave == 1 && !last) {
                // Gp'Y_{h+1} :355: tmp[j] = sum_i Gp[i][j] Y[i], i in order
                if (lane < nc) {
                    const int col = J * kPipeTC + lane;
                    const float* y = nxt + I * kPipeTR;
                    float s = (I == 0) ? 0.0f : tMn[col];
                    int r = 0;
                    for (; r + 8 <= nr; r += 8) {
                        float g[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) g[e] = tl[(r + e) * kPipeTS + lane];
                        const sf4 y0 = *reinterpret_cast<const sf4*>(y + r), y1 = *reinterpret_cast<const sf4*>(y + r + 4);
#pragma unroll
                        for (int e = 0; e < 8; ++e) s += g[e] * (e < 4 ? y0[e] : y1[e - 4]);
                    }
                    for (; r < nr; ++r) s += tl[r * kPipeTS + lane] * y[r];
                    tMn[col] = (I == nI - 1) ? s + 1.0f * A.Fp[col] : s;  // matrixAdd :356
                }
            }
        }
        }
        const int infeasible = __syncthreads_or(bad);
        was_feasible = !infeasible;
        if (tr) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            acc_ph[1] += t - t0;
            t0 = t;
            ++n_it;
        }
        int stop = 0;
        if (!infeasible) {
            // computeCost(Y, Qd, Fd, Md) and computeCost(U, Qp, Fp, Mp) :648-666
            if (!fuse)
                for (int j = 4 * tid; j < N; j += 4 * NT) {
                    float t[4];
                    col_dotv<4, kSU4>(A.Qd + j, N, cur, N, t);
#pragma unroll
                    for (int c = 0; c < 4; ++c) tq[j + c] = t[c];
                }
            for (int j = 2 * tid; j < M; j += 2 * NT) {
                float t[2];
                col_dotv<2, kSU>(A.Qp + j, M, Us, M, t);
                tu[j] = t[0];
                tu[j + 1] = t[1];
            }
            __syncthreads();
            for (int j = tid; j < N; j += NT) {
                tq[j] = tq[j] * cur[j];
                fy[j] = A.Fd[j] * cur[j];
            }
            for (int j = tid; j < M; j += NT) {
                tu[j] = tu[j] * Us[j];
                fu[j] = A.Fp[j] * Us[j];
            }
            __syncthreads();
            if (tid == 0 || tid == 64) {
                const bool dual = (tid == 0);
                const float* qv = dual ? tq : tu;
                const float* lv = dual ? fy : fu;
                const int n = dual ? N : M;  // multiples of 4 here, the vectors 16-byte aligned
                // (Z'Q).Z :652-655 and F'Z :656-657, each in k order; the two
                // chains interleaved and read 16 bytes at a time (one after the
                // other, term by term, they took most of the cost phase)
                float quad = 0.0f, lin = 0.0f;
                for (int k = 0; k < n; k += 4) {
                    const sf4 a = *reinterpret_cast<const sf4*>(qv + k), b = *reinterpret_cast<const sf4*>(lv + k);
                    quad += a.x;
                    lin += b.x;
                    quad += a.y;
                    lin += b.y;
                    quad += a.z;
                    lin += b.z;
                    quad += a.w;
                    lin += b.w;
                }
                float J = 0.0f;
                J = (float)((double)J + 0.5 * (double)quad);
                J += lin;
                J += (dual ? A.Md[0] : A.Mp[0]) / 2;
                s_J[dual ? 1 : 0] = J;
            }
            __syncthreads();
            const float Jp = s_J[0], Jd = s_J[1];
            stop = 1;
            if (Jp > -Jd) stop = 0;
            if ((double)(Jp + Jd) > kTol) stop = 0;
            if ((double)(Jp + Jd) / fabs((double)Jd) > kTol) stop = 0;
            if (tid == 0) {
                st->Jp = Jp;
                st->Jd = Jd;
                st->have_costs = 1;
            }
        }
        if (tr) acc_ph[2] += __builtin_amdgcn_s_memtime() - t0;
        if (stop) {
            status = kStatusDone;
            break;
        }
        if (A.max_updates > 0 && h - 1 >= A.max_updates) {
            status = kStatusCapped;
            break;
        }
        if (done_here >= A.chunk) {
            status = kStatusContinue;
            break;
        }
        float* t = cur;
        cur = nxt;
        nxt = t;
        t = tMc;
        tMc = tMn;
        tMn = t;
        ++h;
        ++done_here;
        __syncthreads();  // the cost phase's reads of the tile area before the next phase Y's writes
    }
    for (int i = tid; i < N; i += NT) A.Y[i] = cur[i];
    for (int i = tid; i < M; i += NT) A.U[i] = Us[i];
    if (tr && tid == 0) {  // totals over the launches of a solve
        unsigned long long* T = A0.trace + 16 * (size_t)blockIdx.x;
        for (int p = 0; p < 3; ++p) T[p] += acc_ph[p];
        T[4] += n_it;
    }
    if (tid == 0) {
        st->h = h;
        st->status = status;
        st->resume = 1;
        if (status == kStatusContinue && A.pending) atomicAdd(A.pending, 1);
    }
}
// </solve-pipe>

// ---------------------------------------------------------------------------
// k_solve_small: solveQuadraticDual for problems that fit in LDS (the bundled
// MPC problem: N = 28, M = 7).  One 256-thread workgroup, everything staged in
// LDS once, and the four waves take fixed ROLES so that the independent pieces
// of an iteration run concurrently on the CU's four SIMDs:
//   phase A  wave 0: updateY2 -- 2 lanes per row (even lane: num with the
//                    stored Qdn_theta, odd lane: den with Qdp_theta), literal
//                    reference arithmetic, then num/den*y
//            wave 1: tM = Gp'Y + Fp                 (computeUfromY, :355-356)
//            wave 2: tq = Y'Qd and s = tq.Y          (computeCost(Y,Qd..), :652-653)
//            wave 3: lin = Fd'Y                     (:657)
//   phase B  wave 1: U = -Qp_inv tM, checkFeas, Jp, the three gap tests
// terminate(Y_h) and the update from Y_h both read only Y_h, so the update is
// computed speculatively and dropped when terminate() stops -- the arithmetic
// of every value is exactly the reference's.
// ---------------------------------------------------------------------------
struct SmallLayout {
    int S, Qd, Gp, Qi, Qp, Kp, Fd, Fdp, Fdn, th, Fp, ya, yb, tq, tM, U, tu, nd, total;
};
__host__ __device__ inline int align4(int n) { return (n + 3) & ~3; }
__host__ __device__ inline SmallLayout small_layout(int N, int M) {
    SmallLayout L;
    int o = 0;
    L.S = o;   o += align4(2 * N * N);
    L.Qd = o;  o += align4(N * N);
    L.Gp = o;  o += align4(N * M);
    L.Qi = o;  o += align4(M * M);
    L.Qp = o;  o += align4(M * M);
    L.Kp = o;  o += align4(N);
    L.Fd = o;  o += align4(N);
    L.Fdp = o; o += align4(N);
    L.Fdn = o; o += align4(N);
    L.th = o;  o += align4(N);
    L.Fp = o;  o += align4(M);
    L.ya = o;  o += align4(N);
    L.yb = o;  o += align4(N);
    L.tq = o;  o += align4(N);
    L.tM = o;  o += align4(M);
    L.U = o;   o += align4(M);
    L.tu = o;  o += align4(M);
    L.nd = o;  o += align4(2 * N);
    L.total = o + 8;  // + scalars
    return L;
}

__global__ void __launch_bounds__(256) k_solve_small(SolveArgs A0, SolveState* __restrict__ st0) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SolveArgs A = problem_at(A0, blockIdx.x);
    SolveState* st = st0 + blockIdx.x;
    if (st->status == kStatusDone || st->status == kStatusCapped) return;
    const int N = A.N, M = A.M;
    const SmallLayout L = small_layout(N, M);
    float* S = lds + L.S;      // [k][i][2]: (k*N + i)*2 + side; side 0 = Qdn_theta, 1 = Qdp_theta
    float* Qd = lds + L.Qd;    // row-major
    float* Gp = lds + L.Gp;    // row-major N x M
    float* Qi = lds + L.Qi;    // Qp_inv row-major
    float* Qp = lds + L.Qp;
    float* Kp = lds + L.Kp;
    float* Fd = lds + L.Fd;
    float* Fdp = lds + L.Fdp;
    float* Fdn = lds + L.Fdn;
    float* th = lds + L.th;
    float* Fp = lds + L.Fp;
    float* tq = lds + L.tq;
    float* tM = lds + L.tM;
    float* Us = lds + L.U;
    float* tu = lds + L.tu;
    float* nd = lds + L.nd;
    float* sc = lds + L.total - 8;  // [0] s_dual [1] lin_dual [2] stop [3] Jp [4] Jd
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const bool conv = (A.mode != kModeFixed);

    // ---- stage the problem (once per launch) ----
    for (int e = tid; e < N * N; e += 256) Qd[e] = A.Qd[e];
    for (int i = tid; i < N; i += 256) {
        Fd[i] = A.Fd[i];
        Fdp[i] = max_ref(0.0f, A.Fd[i]);   // matrixPos(Fdp, Fd) :703
        Fdn[i] = max_ref(0.0f, -A.Fd[i]);  // matrixNeg(Fdn, Fd) :704
    }
    if (conv) {
        for (int e = tid; e < N * M; e += 256) Gp[e] = A.Gp[e];
        for (int e = tid; e < M * M; e += 256) {
            Qi[e] = A.Qinv[e];
            Qp[e] = A.Qp[e];
        }
        for (int i = tid; i < N; i += 256) Kp[i] = A.Kp[i];
        for (int j = tid; j < M; j += 256) Fp[j] = A.Fp[j];
    }
    __syncthreads();
    // computeTheta (:503-519): theta_i = max(sum_k max(0,-Qd[i][k])*1, 5)
    for (int i = tid; i < N; i += 256) {
        float s = 0.0f;
        for (int k = 0; k < N; ++k) s += max_ref(0.0f, -Qd[i * N + k]) * 1.0f;
        th[i] = max_ref(s, 5.0f);
    }
    __syncthreads();
    // computeQdn_theta / computeQdp_theta (:524-537), stored interleaved
    for (int e = tid; e < N * N; e += 256) {
        const int i = e / N, k = e % N;
        const float q = Qd[e];
        const float t = (i == k) ? th[i] : 0.0f;
        S[(k * N + i) * 2 + 0] = max_ref(0.0f, -q) + 1.0f * t;
        S[(k * N + i) * 2 + 1] = max_ref(0.0f, q) + 1.0f * t;
    }
    float* cur = lds + L.ya;
    float* nxt = lds + L.yb;
    for (int i = tid; i < N; i += 256) cur[i] = st->resume ? A.Y[i] : 1000.0f;  // initMat(Y,1000) :710
    const float Md = conv ? A.Md[0] : 0.0f, Mp = conv ? A.Mp[0] : 0.0f;
    __syncthreads();

    long long h = st->h;
    long long done_here = 0;
    int status = kStatusContinue;
    for (;;) {
        const bool need_term = conv;
        const bool may_update = (A.mode != kModeTerminate);
        // ---------------- phase A ----------------
        if (wave == 0) {
            if (may_update) {
                for (int p = lane; p < 2 * N; p += 64) nd[p] = seq_dot(S + p, 2 * N, cur, N);  // :608-609
                __builtin_amdgcn_wave_barrier();
                for (int i = lane; i < N; i += 64) {
                    const float num = nd[2 * i] + 1.0f * Fdn[i];     // :611
                    const float den = nd[2 * i + 1] + 1.0f * Fdp[i]; // :612
                    nxt[i] = num / den * cur[i];                     // :594
                }
            }
        } else if (need_term && wave == 1) {
            for (int j = lane; j < M; j += 64) tM[j] = seq_dot(Gp + j, M, cur, N) + 1.0f * Fp[j];
        } else if (need_term && wave == 2) {
            for (int j = lane; j < N; j += 64) tq[j] = seq_dot(Qd + j, N, cur, N);
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) sc[0] = seq_dot(tq, 1, cur, N);
        } else if (need_term && wave == 3) {
            if (lane == 0) sc[1] = seq_dot(Fd, 1, cur, N);
        }
        __syncthreads();
        // ---------------- phase B: terminate() decision (wave 1) ----------------
        if (need_term && wave == 1) {
            for (int i = lane; i < M; i += 64) Us[i] = -seq_dot(Qi + i * M, 1, tM, M);  // :357-358
            __builtin_amdgcn_wave_barrier();
            int bad = 0;  // checkFeas :632-641
            for (int i = lane; i < N; i += 64) {
                const float s = seq_dot(Gp + i * M, 1, Us, M);
                const float kp = Kp[i];
                if (s > kp + max_ref((float)(kTol * kp), (float)kTol)) bad = 1;
            }
            const bool infeasible = __any(bad);
            int stop = 0;
            if (!infeasible) {
                for (int j = lane; j < M; j += 64) tu[j] = seq_dot(Qp + j, M, Us, M);  // U'Qp
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) {
                    const float quad = seq_dot(tu, 1, Us, M);
                    const float lin = seq_dot(Fp, 1, Us, M);
                    float Jp = 0.0f;
                    Jp = (float)((double)Jp + 0.5 * (double)quad);
                    Jp += lin;
                    Jp += Mp / 2;
                    float Jd = 0.0f;
                    Jd = (float)((double)Jd + 0.5 * (double)sc[0]);
                    Jd += sc[1];
                    Jd += Md / 2;
                    stop = gap_stop(Jp, Jd) ? 1 : 0;  // :683-685
                    sc[3] = Jp;
                    sc[4] = Jd;
                    st->Jp = Jp;
                    st->Jd = Jd;
                    st->have_costs = 1;
                }
            }
            if (lane == 0) sc[2] = (float)stop;
        }
        __syncthreads();
        if (need_term) {
            const bool stop = sc[2] != 0.0f;
            if (A.mode == kModeTerminate) {
                if (tid == 0) st->last_stop = stop ? 1 : 0;
                status = kStatusDone;
                break;
            }
            if (stop) {
                status = kStatusDone;
                break;
            }
            if (A.max_updates > 0 && h - 1 >= A.max_updates) {
                status = kStatusCapped;
                break;
            }
        } else if (h >= A.num_iter) {  // while(h < NUM_ITER)
            status = kStatusDone;
            break;
        }
        if (done_here >= A.chunk) {
            status = kStatusContinue;
            break;
        }
        // accept the update computed in phase A
        float* t = cur;
        cur = nxt;
        nxt = t;
        ++h;
        ++done_here;
        // no barrier needed: the next phase A reads `cur` (written before the
        // last __syncthreads) and writes `nxt`, which nobody reads until after
        // the next __syncthreads
    }
    for (int i = tid; i < N; i += 256) A.Y[i] = cur[i];
    if (conv)
        for (int i = tid; i < M; i += 256) A.U[i] = Us[i];
    if (tid == 0) {
        st->h = h;
        st->status = status;
        st->resume = 1;
        if (status == kStatusContinue && A.pending) atomicAdd(A.pending, 1);
    }
}

// ---------------------------------------------------------------------------
// k_solve_tiny<NMAX>: N, M <= NMAX (the bundled problem, N = 28, M = 7).
// Same roles as k_solve_small, but every lane keeps its slice of the
// (constant) matrices in VGPRs for the whole solve, cross-lane values move by
// v_readlane, and one barrier per iteration suffices (per-iteration scalars are
// double-buffered by parity; every wave evaluates the stop decision from the
// same LDS words, so control flow stays uniform).  Registers and LDS beyond N/M
// are zero: an extra term adds exactly +0 to an accumulator that is never -0,
// so the fully unrolled NMAX-step sums are bit-identical to the N-step ones.
// Launched with 64 threads (wave 0 only) in fixed mode, 256 otherwise.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float rdl(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

template <int NMAX, int MMAX>
__global__ void __launch_bounds__(256) k_solve_tiny(SolveArgs A0, SolveState* __restrict__ st0) {
    const SolveArgs A = problem_at(A0, blockIdx.x);
    SolveState* st = st0 + blockIdx.x;
    if (st->status == kStatusDone || st->status == kStatusCapped) return;
    __shared__ __attribute__((aligned(16))) float ybuf[2][NMAX];
    __shared__ float sc[2][8];  // [parity]: 0 s_dual, 1 lin_dual, 2 infeasible, 3 quad_p, 4 lin_p, 5 stop
    const int N = A.N, M = A.M;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const bool conv = (A.mode != kModeFixed);

    // ---- one-time setup: each role loads its slice into registers ----
    float mat[NMAX];  // wave 0: split row; wave 1: Gp column; wave 2: Qd column; wave 3: unused
    float mat2[MMAX], mat3[MMAX], mat4[MMAX];  // wave 1: Gp row, Qp_inv row, Qp column
    float vA = 0.0f, vB = 0.0f;  // per-lane scalars of the role
#pragma unroll
    for (int k = 0; k < NMAX; ++k) mat[k] = 0.0f;
#pragma unroll
    for (int k = 0; k < MMAX; ++k) mat2[k] = mat3[k] = mat4[k] = 0.0f;
    if (wave == 0) {
        const int i = lane >> 1, side = lane & 1;
        if (i < N) {
            float th = 0.0f;  // computeTheta (:503-519)
            for (int k = 0; k < N; ++k) th += max_ref(0.0f, -A.Qd[i * N + k]) * 1.0f;
            th = max_ref(th, 5.0f);
#pragma unroll
            for (int k = 0; k < NMAX; ++k) {
                if (k < N) {
                    const float q = A.Qd[i * N + k];
                    const float t = (i == k) ? th : 0.0f;
                    // side 0: Qdn_theta (numerator), side 1: Qdp_theta  (:524-537)
                    mat[k] = (side ? max_ref(0.0f, q) : max_ref(0.0f, -q)) + 1.0f * t;
                }
            }
            const float f = A.Fd[i];
            vA = side ? max_ref(0.0f, f) : max_ref(0.0f, -f);  // Fdp / Fdn  (:703-704)
        }
    } else if (conv && wave == 1) {
#pragma unroll
        for (int k = 0; k < NMAX; ++k)
            if (lane < M && k < N) mat[k] = A.Gp[k * M + lane];      // Gp column  (Gp'Y)
#pragma unroll
        for (int k = 0; k < MMAX; ++k) {
            if (lane < N && k < M) mat2[k] = A.Gp[lane * M + k];     // Gp row     (Gp U)
            if (lane < M && k < M) mat3[k] = A.Qinv[lane * M + k];   // Qp_inv row (Qp_inv t)
            if (lane < M && k < M) mat4[k] = A.Qp[k * M + lane];     // Qp column  (U'Qp)
        }
        vA = (lane < M) ? A.Fp[lane] : 0.0f;
        vB = (lane < N) ? A.Kp[lane] : 0.0f;
    } else if (conv && wave == 2) {
#pragma unroll
        for (int k = 0; k < NMAX; ++k)
            if (lane < N && k < N) mat[k] = A.Qd[k * N + lane];      // Qd column  (Y'Qd)
    } else if (conv && wave == 3) {
        vA = (lane < N) ? A.Fd[lane] : 0.0f;
    }
    const float Md = conv ? A.Md[0] : 0.0f, Mp = conv ? A.Mp[0] : 0.0f;
    for (int k = tid; k < NMAX; k += blockDim.x) {
        ybuf[0][k] = (k < N) ? (st->resume ? A.Y[k] : 1000.0f) : 0.0f;  // initMat(Y, 1000) :710
        ybuf[1][k] = 0.0f;
    }
    __syncthreads();

    long long h = st->h;
    long long done_here = 0;
    int status = kStatusContinue;
    int cb = 0;  // ybuf index of the current iterate
    for (int par = 0;; par ^= 1) {
        const float* cur = ybuf[cb];
        float* nxt = ybuf[cb ^ 1];
        float yv[NMAX];
#pragma unroll
        for (int k = 0; k < NMAX; k += 4) {
            const float4 t = *reinterpret_cast<const float4*>(cur + k);
            yv[k] = t.x;
            yv[k + 1] = t.y;
            yv[k + 2] = t.z;
            yv[k + 3] = t.w;
        }
        if (wave == 0) {
            if (A.mode != kModeTerminate) {  // updateY2 (:603-618)
                float acc = 0.0f;
#pragma unroll
                for (int k = 0; k < NMAX; ++k) acc += mat[k] * yv[k];  // :608-609
                // both shuffles run with the full wave active (a lane-divergent
                // __shfl would read an inactive partner lane)
                const float other = __shfl_xor(acc, 1);
                const float fdp = __shfl_xor(vA, 1);
                const int i = lane >> 1;
                if (!(lane & 1) && i < N) {
                    const float fdn = vA;
                    const float num = acc + 1.0f * fdn;    // :611
                    const float den = other + 1.0f * fdp;  // :612
                    nxt[i] = num / den * cur[i];           // :594
                }
            }
        } else if (conv && wave == 1) {
            // computeUfromY (:352-360): t = Gp'Y + Fp ; U = -(Qp_inv t)
            float t = 0.0f;
#pragma unroll
            for (int k = 0; k < NMAX; ++k) t += mat[k] * yv[k];
            t = t + 1.0f * vA;
            if (lane >= M) t = 0.0f;
            float u = 0.0f;
#pragma unroll
            for (int j = 0; j < MMAX; ++j) u += mat3[j] * rdl(t, j);
            u = (lane < M) ? -u : 0.0f;
            // checkFeas (:632-641)
            float g = 0.0f;
#pragma unroll
            for (int j = 0; j < MMAX; ++j) g += mat2[j] * rdl(u, j);
            const int bad = (lane < N) && (g > vB + max_ref((float)(kTol * vB), (float)kTol));
            const bool infeasible = __any(bad);
            // computeCost(U, Qp, Fp, Mp) (:648-666): row = U'Qp ; quad = row.U ; lin = Fp'U
            float row = 0.0f;
#pragma unroll
            for (int k = 0; k < MMAX; ++k) row += rdl(u, k) * mat4[k];
            if (lane >= M) row = 0.0f;
            float quad = 0.0f, lin = 0.0f;
#pragma unroll
            for (int j = 0; j < MMAX; ++j) {
                const float uj = rdl(u, j);
                quad += rdl(row, j) * uj;
                lin += rdl(vA, j) * uj;
            }
            if (lane == 0) {
                sc[par][2] = infeasible ? 1.0f : 0.0f;
                sc[par][3] = quad;
                sc[par][4] = lin;
            }
            if (lane < M) A.U[lane] = u;  // computeUfromY writes U on every terminate()
        } else if (conv && wave == 2) {
            // computeCost(Y, Qd, Fd, Md): row = Y'Qd ; s = row.Y
            float row = 0.0f;
#pragma unroll
            for (int k = 0; k < NMAX; ++k) row += yv[k] * mat[k];
            float s2 = 0.0f;
#pragma unroll
            for (int j = 0; j < NMAX; ++j) s2 += rdl(row, j) * yv[j];
            if (lane == 0) sc[par][0] = s2;
        } else if (conv && wave == 3) {
            float lin = 0.0f;
#pragma unroll
            for (int k = 0; k < NMAX; ++k) lin += rdl(vA, k) * yv[k];
            if (lane == 0) sc[par][1] = lin;
        }
        __syncthreads();
        if (conv) {
            // the costs and gap tests (:648-687) on one wave only; the others
            // wait for its verdict at a second barrier instead of repeating
            // the double-precision tests four times
            if (wave == 1) {
                int stop1 = 0;
                if (sc[par][2] == 0.0f) {
                    float Jp = 0.0f;
                    Jp = (float)((double)Jp + 0.5 * (double)sc[par][3]);
                    Jp += sc[par][4];
                    Jp += Mp / 2;
                    float Jd = 0.0f;
                    Jd = (float)((double)Jd + 0.5 * (double)sc[par][0]);
                    Jd += sc[par][1];
                    Jd += Md / 2;
                    stop1 = gap_stop(Jp, Jd) ? 1 : 0;  // :683-685
                    if (lane == 0) {
                        st->Jp = Jp;
                        st->Jd = Jd;
                        st->have_costs = 1;
                    }
                }
                if (lane == 0) sc[par][5] = stop1 ? 1.0f : 0.0f;
            }
            __syncthreads();
            const int stop = sc[par][5] != 0.0f;
            if (A.mode == kModeTerminate) {
                if (tid == 0) st->last_stop = stop;
                status = kStatusDone;
                break;
            }
            if (stop) {
                status = kStatusDone;
                break;
            }
            if (A.max_updates > 0 && h - 1 >= A.max_updates) {
                status = kStatusCapped;
                break;
            }
        } else if (h >= A.num_iter) {
            status = kStatusDone;
            break;
        }
        if (done_here >= A.chunk) {
            status = kStatusContinue;
            break;
        }
        cb ^= 1;  // accept the update
        ++h;
        ++done_here;
    }
    for (int i = tid; i < N; i += blockDim.x) A.Y[i] = ybuf[cb][i];
    if (tid == 0) {
        st->h = h;
        st->status = status;
        st->resume = 1;
        if (status == kStatusContinue && A.pending) atomicAdd(A.pending, 1);
    }
}

// ---------------------------------------------------------------------------
// k_fixed_tiny<NMAX>: the fixed-iteration mode (while(h < NUM_ITER), no
// terminate) of one N <= NMAX problem on ONE wave: lane 2i + side holds row
// i's split row (Qdn_theta / Qdp_theta incl. Theta) in VGPRs, y lives in LDS.
// Per update: the products (packed multiplies, off the add chain), the
// sequential adds, the num/den exchange by a DPP lane swap (not an LDS
// permute), the division.  The iterate's own y_i is read at the top of the
// update so its latency hides under the chain.  One wave: a ds_write followed
// by the next update's ds_reads needs no workgroup barrier.  RL: the iterate
// never leaves the registers -- y_k on lane 2k, broadcast by v_readlane.
// ---------------------------------------------------------------------------
template <int NMAX, bool RL>
__global__ void __launch_bounds__(64) k_fixed_tiny(SolveArgs A0, SolveState* __restrict__ st0) {
    const SolveArgs A = problem_at(A0, blockIdx.x);
    SolveState* st = st0 + blockIdx.x;
    if (st->status == kStatusDone || st->status == kStatusCapped) return;
    __shared__ __attribute__((aligned(16))) float ybuf[2][NMAX];
    const int N = A.N;
    const int lane = threadIdx.x, i = lane >> 1, side = lane & 1;
    const bool row = i < N;
    float mat[NMAX];
#pragma unroll
    for (int k = 0; k < NMAX; ++k) mat[k] = 0.0f;
    float fd_own = 0.0f;
    if (row) {
        float th = 0.0f;  // computeTheta (:503-519)
        for (int k = 0; k < N; ++k) th += max_ref(0.0f, -A.Qd[i * N + k]) * 1.0f;
        th = max_ref(th, 5.0f);
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
            if (k < N) {
                const float q = A.Qd[i * N + k];
                const float t = (i == k) ? th : 0.0f;
                mat[k] = (side ? max_ref(0.0f, q) : max_ref(0.0f, -q)) + 1.0f * t;  // :524-537
            }
        }
        const float f = A.Fd[i];
        fd_own = side ? max_ref(0.0f, f) : max_ref(0.0f, -f);  // Fdp / Fdn (:703-704)
    }
    for (int k = lane; k < NMAX; k += 64) {
        ybuf[0][k] = (k < N) ? (st->resume ? A.Y[k] : 1000.0f) : 0.0f;  // initMat(Y, 1000) :710
        ybuf[1][k] = 0.0f;
    }
    __syncthreads();
    const int ic = row ? i : 0;
    long long h = st->h;
    long long done_here = 0;
    int cb = 0;
    int status = kStatusContinue;
    if constexpr (RL) {
        // the iterate stays in registers: y_k on lane 2k, broadcast to every
        // lane by v_readlane (wave-uniform, SGPRs) -- no LDS round trip and no
        // barrier between updates
        float yk = (!side && row) ? ybuf[0][i] : 0.0f;
        typedef float f2v __attribute__((ext_vector_type(2)));
        for (;;) {
            if (h >= A.num_iter) {  // while(h < NUM_ITER)
                status = kStatusDone;
                break;
            }
            if (done_here >= A.chunk) break;
            // this row's y_i (lane 2i) on its den lane 2i+1: DPP quad_perm
            // [0,0,2,2] within the quad, no LDS round trip (a ds_bpermute here
            // left its latency after the division, on the loop's critical path)
            const float yi = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(yk), 0xA0, 0xF, 0xF, true));
            float p[NMAX];
#pragma unroll
            for (int k = 0; k < NMAX; k += 2) {
                const float y0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(yk), 2 * k));
                const float y1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(yk), 2 * k + 2));
                const f2v pr = f2v{mat[k], mat[k + 1]} * f2v{y0, y1};
                p[k] = pr.x;
                p[k + 1] = pr.y;
            }
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < NMAX; ++k) acc += p[k];  // :608-609, k in order
            const float v = acc + 1.0f * fd_own;        // even lane: num (:611), odd lane: den (:612)
            const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
            const float yn = v / den * yi;              // :594
            yk = (!side && row) ? yn : 0.0f;            // lanes past 2N hold +0 (the padding y_k)
            ++h;
            ++done_here;
        }
        if (!side && row) ybuf[0][i] = yk;
        cb = 0;
        __syncthreads();
    }
    for (;;) {
        if constexpr (RL) break;
        if (h >= A.num_iter) {  // while(h < NUM_ITER)
            status = kStatusDone;
            break;
        }
        if (done_here >= A.chunk) break;
        const float* cur = ybuf[cb];
        float* nxt = ybuf[cb ^ 1];
        const float yi = cur[ic];
        typedef float f4v __attribute__((ext_vector_type(4)));
        typedef float f2v __attribute__((ext_vector_type(2)));
        float p[NMAX];
#pragma unroll
        for (int k = 0; k < NMAX; k += 4) {
            const f4v y = *reinterpret_cast<const f4v*>(cur + k);
            const f2v lo = f2v{mat[k], mat[k + 1]} * f2v{y.x, y.y};
            const f2v hi = f2v{mat[k + 2], mat[k + 3]} * f2v{y.z, y.w};
            p[k] = lo.x;
            p[k + 1] = lo.y;
            p[k + 2] = hi.x;
            p[k + 3] = hi.y;
        }
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < NMAX; ++k) acc += p[k];  // :608-609, k in order
        const float v = acc + 1.0f * fd_own;        // even lane: num (:611), odd lane: den (:612)
        // lane ^ 1 by DPP quad_perm(1,0,3,2); the whole wave is active here
        const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
        if (!side && row) nxt[i] = v / den * yi;    // :594
        __syncthreads();
        cb ^= 1;
        ++h;
        ++done_here;
    }
    for (int k = lane; k < N; k += 64) A.Y[k] = ybuf[cb][k];
    if (lane == 0) {
        st->h = h;
        st->status = status;
        st->resume = 1;
        if (status == kStatusContinue && A.pending) atomicAdd(A.pending, 1);
    }
}

// ---------------------------------------------------------------------------
// k_solve_wave<NMAX, MMAX>: converge mode (terminate() before every update,
// PQP_CPU.c:694-750) of one N <= NMAX, M <= MMAX problem on ONE wave, for
// throughput over many problems (one problem per 64-thread workgroup, several
// problems per SIMD).  The same arithmetic as k_solve_tiny, packed two sums per
// lane so the terminate() mat-vecs ride along with the update's:
//   pass over k (one v_pk_mul + one v_pk_add per k):
//     .x  lanes 2i+side < 2N : the split row i (Qdn_theta / Qdp_theta)   -> num / den
//     .y  lanes j < N        : Qd column j                                -> (Y'Qd)_j   (:652)
//         lanes N + j < N + M: Gp column j                                -> (Gp'Y)_j   (:354)
//   U = -(Qp_inv t) on lanes < M, then one pass over j < M:
//     .x  lanes i < N : Gp row i -> (Gp U)_i (checkFeas :632-641)
//     .y  lanes k < M : Qp column k -> (U'Qp)_k (computeCost :652)
//   and the four scalar dot products in two packed pairs:
//     (U'Qp . U, Fp . U) and (Y'Qd . Y, Fd . Y)  (:655-657)
// Every sum keeps the reference's order from +0.0f with rounded products (no
// FMA; a packed op rounds each half exactly like its scalar form), and the
// padding terms (beyond N / M) add exactly +0 to sums that are never -0.
// Vectors cross lanes through LDS (one wave: program order suffices).
// ---------------------------------------------------------------------------
template <int NMAX, int MMAX, bool PIPE>
__global__ void __launch_bounds__(64) k_solve_wave(SolveArgs A0, SolveState* __restrict__ st0) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    typedef float f4v __attribute__((ext_vector_type(4)));
    static_assert(NMAX % 4 == 0 && MMAX % 4 == 0 && NMAX <= 32 && MMAX <= 32, "one wave");
    const SolveArgs A = problem_at(A0, blockIdx.x);
    SolveState* st = st0 + blockIdx.x;
    if (st->status == kStatusDone || st->status == kStatusCapped) return;
    __shared__ __attribute__((aligned(16))) float ybuf[2][NMAX];
    __shared__ float junk[64];  // per-lane sink: stores are unconditional (no branch splits the iteration)
    __shared__ __attribute__((aligned(16))) float rowb[NMAX];  // Y'Qd
    __shared__ __attribute__((aligned(16))) float tb[MMAX];    // t = Gp'Y + Fp
    __shared__ __attribute__((aligned(16))) float ub[MMAX];    // U
    __shared__ __attribute__((aligned(16))) float rpb[MMAX];   // U'Qp
    const int N = A.N, M = A.M;
    const int lane = threadIdx.x, i = lane >> 1, side = lane & 1;

    f2v mat[NMAX];
    f2v gq[MMAX];
    float qinv[MMAX];
#pragma unroll
    for (int k = 0; k < NMAX; ++k) mat[k] = f2v{0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < MMAX; ++j) {
        gq[j] = f2v{0.0f, 0.0f};
        qinv[j] = 0.0f;
    }
    // setup: branch-free (clamped addresses, selects) and a few loads in flight
    // at a time, so its register peak stays below the loop's
    const bool rowl = i < N;
    const int ir = rowl ? i : 0;
    float th = 0.0f;  // computeTheta (:503-519)
    for (int k = 0; k < N; ++k) th += max_ref(0.0f, -A.Qd[ir * N + k]) * 1.0f;
    th = max_ref(th, 5.0f);
    const bool colq = lane < N, colg = lane >= N && lane < N + M;
    const int jq = colq ? lane : 0, jg = colg ? lane - N : 0;
    // Fd . Y rides in the pass too: on the free .x lane 2N, or (N = 32) the
    // free .y lane N + M (N = M = 32 is left to k_solve_tiny)
    const int lf = (2 * N < 64) ? 2 * N : N + M;
    const bool fx = (2 * N < 64) && lane == lf, fy = (2 * N >= 64) && lane == lf;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {
        if (k % 4 == 0) __builtin_amdgcn_sched_barrier(0);
        const int kc = (k < N) ? k : 0;
        const float q = A.Qd[ir * N + kc];
        const float t = (ir == k) ? th : 0.0f;
        const float sp = (side ? max_ref(0.0f, q) : max_ref(0.0f, -q)) + 1.0f * t;  // :524-537
        const float fk = A.Fd[kc];               // Fd (Fd . Y)
        mat[k].x = (k < N) ? (rowl ? sp : (fx ? fk : 0.0f)) : 0.0f;
        const float qc = A.Qd[kc * N + jq];      // Qd column (Y'Qd)
        const float gc = A.Gp[kc * M + jg];      // Gp column (Gp'Y)
        mat[k].y = (k < N) ? (colq ? qc : (colg ? gc : (fy ? fk : 0.0f))) : 0.0f;
    }
    const int jm = lane < M ? lane : 0, ig = lane < N ? lane : 0;
#pragma unroll
    for (int j = 0; j < MMAX; ++j) {
        if (j % 4 == 0) __builtin_amdgcn_sched_barrier(0);
        const int jc = (j < M) ? j : 0;
        const float gr = A.Gp[ig * M + jc];      // Gp row (Gp U): row i = lane
        const float qp = A.Qp[jc * M + jm];      // Qp column (U'Qp)
        const float qi = A.Qinv[jm * M + jc];    // Qp_inv row (Qp_inv t)
        const float fj = A.Fp[jc];               // Fp (Fp . U) on the free .x lane N
        gq[j].x = (j < M) ? ((lane < N) ? gr : (lane == N ? fj : 0.0f)) : 0.0f;
        gq[j].y = (j < M && lane < M) ? qp : 0.0f;
        qinv[j] = (j < M && lane < M) ? qi : 0.0f;
    }
    __builtin_amdgcn_sched_barrier(0);
    float fd_own = 0.0f, fp_own = 0.0f, kp = 0.0f;
    {
        const float f = A.Fd[ir];
        fd_own = rowl ? (side ? max_ref(0.0f, f) : max_ref(0.0f, -f)) : 0.0f;  // Fdp / Fdn (:703-704)
        const float fp = A.Fp[jg];
        fp_own = colg ? fp : 0.0f;
    }
    if (lane < N) kp = A.Kp[lane];
    const float Md = A.Md[0], Mp = A.Mp[0];
    for (int k = lane; k < NMAX; k += 64) {
        ybuf[0][k] = (k < N) ? (st->resume ? A.Y[k] : 1000.0f) : 0.0f;  // initMat(Y, 1000) :710
        ybuf[1][k] = 0.0f;
        rowb[k] = 0.0f;
    }
    for (int j = lane; j < MMAX; j += 64) tb[j] = ub[j] = rpb[j] = 0.0f;
    __syncthreads();

    const int ic = (i < N) ? i : 0;
    long long h = st->h;
    long long done_here = 0;
    int status = kStatusContinue;
    int cb = 0;
    float u_last = 0.0f, Jp_last = 0.0f, Jd_last = 0.0f;
    bool have = false;
    // the fused pass over k: one v_pk_mul + v_pk_add per k
    auto pass = [&](const float* yb) {
        f2v a = f2v{0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < NMAX; k += 4) {
            const f4v y = *reinterpret_cast<const f4v*>(yb + k);
            a += mat[k] * f2v{y.x, y.x};  // :608-609 / :354 / :652, k in order
            a += mat[k + 1] * f2v{y.y, y.y};
            a += mat[k + 2] * f2v{y.z, y.z};
            a += mat[k + 3] * f2v{y.w, y.w};
        }
        return a;
    };
    const bool wr_y = !side && i < N, wr_row = lane < N, wr_t = lane >= N && lane < N + M, wr_m = lane < MMAX;
    // PIPE: every store unconditional (lanes that do not own the word write
    // their own junk word), so no branch splits the iteration; plain: masked
    // stores (fewer registers)
    auto put = [&](bool own, float* dst, float v) {
        if constexpr (PIPE) {
            *(own ? dst : junk + lane) = v;
        } else {
            if (own) *dst = v;
        }
    };
    f2v acc = f2v{0.0f, 0.0f};
    if constexpr (PIPE) acc = pass(ybuf[cb]);
    for (;;) {
        // PIPE (software-pipelined): the pass over the NEXT iterate (speculative:
        // used only if this terminate() says go on) runs beside this iterate's
        // terminate() chains; nothing branches between them.  Shorter
        // iterations, more registers (fewer problems per SIMD).
        const float* cur = ybuf[cb];
        float* nxt = ybuf[cb ^ 1];
        float yi = cur[ic];
        asm volatile("" : "+v"(yi));  // read early: its latency hides under the pass
        if constexpr (!PIPE) acc = pass(cur);
        // ---- updateY2's epilogue ----
        {
            const float v = acc.x + 1.0f * fd_own;  // even lane: num (:611), odd lane: den (:612)
            const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
            put(wr_y, nxt + i, v / den * yi);  // :594
        }
        f2v acc_next = f2v{0.0f, 0.0f};
        if constexpr (PIPE) acc_next = pass(nxt);
        // ---- terminate(): computeUfromY (:352-360) ----
        put(wr_row, rowb + lane, acc.y);
        put(wr_t, tb + (lane - N), acc.y + 1.0f * fp_own);  // tmp = Gp'Y ; tmp += Fp
        const float lin_d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fx ? acc.x : acc.y), lf));  // Fd . Y
        // Y'Qd . Y (computeCost, Jd) first: its chain is independent of U's
        float s2 = 0.0f;
#pragma unroll
        for (int k = 0; k < NMAX; k += 4) {
            const f4v r = *reinterpret_cast<const f4v*>(rowb + k);
            const f4v y = *reinterpret_cast<const f4v*>(cur + k);
            const f2v lo = f2v{r.x, r.y} * f2v{y.x, y.y};
            const f2v hi = f2v{r.z, r.w} * f2v{y.z, y.w};
            s2 += lo.x;
            s2 += lo.y;
            s2 += hi.x;
            s2 += hi.y;
        }
        float ua = 0.0f;
#pragma unroll
        for (int j = 0; j < MMAX; j += 4) {
            const f4v t = *reinterpret_cast<const f4v*>(tb + j);
            ua += qinv[j] * t.x;
            ua += qinv[j + 1] * t.y;
            ua += qinv[j + 2] * t.z;
            ua += qinv[j + 3] * t.w;
        }
        const float u = (lane < M) ? -ua : 0.0f;  // U = -U
        put(wr_m, ub + lane, u);
        // ---- checkFeas (Gp U vs Kp) and U'Qp in one pass over j ----
        f2v g = f2v{0.0f, 0.0f};
        float uv[MMAX];
#pragma unroll
        for (int j = 0; j < MMAX; j += 4) {
            const f4v t = *reinterpret_cast<const f4v*>(ub + j);
            uv[j] = t.x;
            uv[j + 1] = t.y;
            uv[j + 2] = t.z;
            uv[j + 3] = t.w;
        }
#pragma unroll
        for (int j = 0; j < MMAX; ++j) g += gq[j] * f2v{uv[j], uv[j]};
        const int bad = (lane < N) && (g.x > kp + max_ref((float)(kTol * kp), (float)kTol));
        const bool infeasible = __any(bad);
        put(wr_m, rpb + lane, g.y);
        const float lin_p = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g.x), N));  // Fp . U
        // ---- computeCost (:648-666): U'Qp . U and Y'Qd . Y, sequential ----
        float quad = 0.0f;
#pragma unroll
        for (int j = 0; j < MMAX; j += 4) {
            const f4v r = *reinterpret_cast<const f4v*>(rpb + j);
            quad += r.x * uv[j];
            quad += r.y * uv[j + 1];
            quad += r.z * uv[j + 2];
            quad += r.w * uv[j + 3];
        }
        u_last = u;
        // ---- the gap tests (:673-687), wave-uniform ----
        int stop = 0;
        if (!infeasible) {
            float Jp = 0.0f;
            Jp = (float)((double)Jp + 0.5 * (double)quad);
            Jp += lin_p;
            Jp += Mp / 2;
            float Jd = 0.0f;
            Jd = (float)((double)Jd + 0.5 * (double)s2);
            Jd += lin_d;
            Jd += Md / 2;
            stop = gap_stop(Jp, Jd);  // :683-685
            Jp_last = Jp;
            Jd_last = Jd;
            have = true;
        }
        if (stop) {
            status = kStatusDone;
            break;
        }
        if (A.max_updates > 0 && h - 1 >= A.max_updates) {
            status = kStatusCapped;
            break;
        }
        if (done_here >= A.chunk) {
            status = kStatusContinue;
            break;
        }
        cb ^= 1;  // accept the update
        if constexpr (PIPE) acc = acc_next;
        ++h;
        ++done_here;
    }
    for (int k = lane; k < N; k += 64) A.Y[k] = ybuf[cb][k];
    if (lane < M) A.U[lane] = u_last;  // computeUfromY wrote U on every terminate(): the last one stands
    if (lane == 0) {
        if (have) {
            st->Jp = Jp_last;
            st->Jd = Jd_last;
            st->have_costs = 1;
        }
        st->h = h;
        st->status = status;
        st->resume = 1;
        if (status == kStatusContinue && A.pending) atomicAdd(A.pending, 1);
    }
}

// (a register cap of 4 waves per SIMD was measured 30 % slower: it spills
// inside the loop).  Up to a few thousand problems every one gets its own SIMD
// slot at once, so the pipelined form's shorter iterations win; beyond that
// the plain form's smaller register file (3 vs 2 problems per SIMD at the
// bundled size) wins on throughput.
template <int NMAX, bool PIPE>
static void launch_wave_mp(int B, const SolveArgs& a, SolveState* st, hipStream_t s) {
    if (a.M <= 8)
        hipLaunchKernelGGL((k_solve_wave<NMAX, 8, PIPE>), dim3(B), dim3(64), 0, s, a, st);
    else if (a.M <= 16)
        hipLaunchKernelGGL((k_solve_wave<NMAX, 16, PIPE>), dim3(B), dim3(64), 0, s, a, st);
    else
        hipLaunchKernelGGL((k_solve_wave<NMAX, 32, PIPE>), dim3(B), dim3(64), 0, s, a, st);
}
template <int NMAX>
static void launch_wave_m(int B, const SolveArgs& a, SolveState* st, hipStream_t s) {
    if (B <= g_tune.wave_pipe_max_b) launch_wave_mp<NMAX, true>(B, a, st, s);
    else launch_wave_mp<NMAX, false>(B, a, st, s);
}

template <int NMAX>
static void launch_tiny_m(int B, const SolveArgs& a, SolveState* st, int threads, hipStream_t s) {
    if (a.M <= 8)
        hipLaunchKernelGGL((k_solve_tiny<NMAX, 8>), dim3(B), dim3(threads), 0, s, a, st);
    else if (a.M <= 16)
        hipLaunchKernelGGL((k_solve_tiny<NMAX, 16>), dim3(B), dim3(threads), 0, s, a, st);
    else
        hipLaunchKernelGGL((k_solve_tiny<NMAX, 32>), dim3(B), dim3(threads), 0, s, a, st);
}

template <bool RL>
static void launch_fixed_tiny(int B, const SolveArgs& a, SolveState* st, hipStream_t s) {
    if (a.N <= 8) hipLaunchKernelGGL((k_fixed_tiny<8, RL>), dim3(B), dim3(64), 0, s, a, st);
    else if (a.N <= 16) hipLaunchKernelGGL((k_fixed_tiny<16, RL>), dim3(B), dim3(64), 0, s, a, st);
    else if (a.N <= 24) hipLaunchKernelGGL((k_fixed_tiny<24, RL>), dim3(B), dim3(64), 0, s, a, st);
    else if (a.N <= 28) hipLaunchKernelGGL((k_fixed_tiny<28, RL>), dim3(B), dim3(64), 0, s, a, st);
    else hipLaunchKernelGGL((k_fixed_tiny<32, RL>), dim3(B), dim3(64), 0, s, a, st);
}

static hipError_t launch_tiny_grid(int B, const SolveArgs& a, SolveState* st, hipStream_t s) {
    // the unrolled sums run to the next instantiated width >= N (>= M): the
    // sequential chain is the critical path, so keep the padding small
    if (a.mode == kModeFixed) {
        if (B <= g_tune.fixed_rl_max_b) launch_fixed_tiny<true>(B, a, st, s);
        else launch_fixed_tiny<false>(B, a, st, s);
        return hipGetLastError();
    }
    if (a.mode == kModeConverge && B >= g_tune.wave_min_b && a.N + a.M < 64) {  // many problems: one wave each
        if (a.N <= 8) launch_wave_m<8>(B, a, st, s);
        else if (a.N <= 16) launch_wave_m<16>(B, a, st, s);
        else if (a.N <= 24) launch_wave_m<24>(B, a, st, s);
        else if (a.N <= 28) launch_wave_m<28>(B, a, st, s);
        else launch_wave_m<32>(B, a, st, s);
        return hipGetLastError();
    }
    const int threads = (a.mode == kModeFixed) ? 64 : 256;
    if (a.N <= 8) launch_tiny_m<8>(B, a, st, threads, s);
    else if (a.N <= 16) launch_tiny_m<16>(B, a, st, threads, s);
    else if (a.N <= 24) launch_tiny_m<24>(B, a, st, threads, s);
    else if (a.N <= 28) launch_tiny_m<28>(B, a, st, threads, s);
    else launch_tiny_m<32>(B, a, st, threads, s);
    return hipGetLastError();
}
hipError_t launch_solve_tiny(const SolveArgs& a, SolveState* st, hipStream_t s) { return launch_tiny_grid(1, a, st, s); }

// ---------------------------------------------------------------------------
// k_solve_mid: solveQuadraticDual (PQP_CPU.c:694-750) for mid-size problems
// -- the MPC plant over a few horizon steps, N ~ 33..165 -- one workgroup
// per problem with Qd, Gp, Qp_inv and Qp each held in LDS ONCE (no split
// copies: the update forms its split entries from Qd on the fly), so a
// problem is read from HBM once per launch and every iteration runs out of
// LDS.  Layout: Qd rows 16-byte aligned with a stride of 4 (mod 8) dwords
// (ldn = round8(N) + 4): a lane-per-row walk reads 16 bytes per lane
// conflict-free and a lane-per-column walk reads consecutive dwords; Gp,
// Qp_inv, Qp with an ODD stride (4-byte reads, conflict-free both ways).
// Every dimension is padded to a multiple of 8 with zeros, so each walk is
// whole blocks of 8 terms: a padded term adds +0 (or -0) to a sum that starts
// at +0.0f and therefore is never -0, which leaves it unchanged.  Shared
// vectors are 16-byte aligned and read as 16-byte broadcasts.  The blocks of
// a walk are software-pipelined two deep (loads of block b+1 issued before
// block b's arithmetic): with one or two workgroups per CU there are too few
// waves to hide LDS latency otherwise.
//
// One iteration (terminate(Y_h), then the update from Y_h, computed
// speculatively and dropped when terminate() stops -- every value is the
// reference's):
//   phase A  update rows i < N (one lane each; Y'Qd's column i and its
//            product with y_i fused in once an iterate was feasible and Qd is
//            bit-symmetric), tM = Gp'Y + Fp (one lane per column) and Fd.Y
//            (one more lane), and -- Qd not symmetric, previous iterate
//            feasible -- the Y'Qd columns, on separate waves
//   phase B  U = -Qp_inv tM (computeUfromY :352-360); a spare wave sums the
//            (Y'Qd).Y terms when phase A formed them
//   phase C  checkFeas, any row over its bound -> infeasible (:632-641)
//   phase D  (feasible) the (U'Qp).U and Fp.U terms (and the (Y'Qd).Y terms
//            when phase A did not form them)
//   phase E  (feasible) lanes of wave 0 sum what is left in k order; Jp, Jd
//            and the three gap tests (:648-687)
// Chunked and resumable like k_solve_small (state in SolveState).
// ---------------------------------------------------------------------------
__host__ __device__ inline int round8(int n) { return (n + 7) & ~7; }
struct MidLayout {
    int nk, mk;    // N, M rounded up to 8
    int ldn, ldm;  // row strides of Qd (nk + 4) and of Qp (mk + 1)
    int ldg, ldi;  // row strides of Gp' (nk + 4; rows 0..mk-1 the columns of Gp, row mk Fd) and Qp_inv (mk + 4)
    int ya, yb, tq, dP, dN, Fdp, Fdn, Fd, Kp, tM, Us, tu, fu, Fp, sc, Qd, Gp, Qi, Qp, total;
};
__host__ __device__ inline MidLayout mid_layout(int N, int M, bool conv) {
    MidLayout L;
    L.nk = round8(N);
    L.mk = round8(M);
    L.ldn = L.nk + 4;
    L.ldm = L.mk + 1;
    L.ldg = L.nk + 4;
    L.ldi = L.mk + 4;
    int o = 0;
    L.ya = o;  o += L.nk;
    L.yb = o;  o += L.nk;
    L.tq = o;  o += L.nk;
    L.dP = o;  o += L.nk;
    L.dN = o;  o += L.nk;
    L.Fdp = o; o += L.nk;
    L.Fdn = o; o += L.nk;
    L.Fd = o;  o += L.nk;
    L.sc = o;  o += 8;
    if (conv) {
        L.Kp = o;  o += L.nk;
        L.tM = o;  o += L.mk;
        L.Us = o;  o += L.mk;
        L.tu = o;  o += L.mk;
        L.fu = o;  o += L.mk;
        L.Fp = o;  o += L.mk;
    } else {
        L.Kp = L.tM = L.Us = L.tu = L.fu = L.Fp = 0;
    }
    L.Qd = o;  o += L.nk * L.ldn;
    if (conv) {
        L.Gp = o;  o += (L.mk + 1) * L.ldg;
        L.Qi = o;  o += L.mk * L.ldi;
        L.Qp = o;  o += L.mk * L.ldm;
    } else {
        L.Gp = L.Qi = L.Qp = 0;
    }
    L.total = o;
    return L;
}
// threads of the k_solve_mid workgroup: enough waves for phase A at once
__host__ __device__ inline int mid_threads(int N, int M, bool conv) {
    const int w = (N + 63) / 64 + (conv ? (M + 64) / 64 : 0);
    return w <= 2 ? 128 : (w <= 4 ? 256 : 512);
}

// 8 terms of a strided walk: a[(k + j) * as] (per-lane a and as) and the
// broadcast b[k + j]
struct MidBlk {
    float a[8];
    sf4 b0, b1;
};
__device__ __forceinline__ void mid_load(MidBlk& B, const float* a, int as, const float* b, int k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) B.a[j] = a[(k + j) * as];
    B.b0 = *reinterpret_cast<const sf4*>(b + k);
    B.b1 = *reinterpret_cast<const sf4*>(b + k + 4);
}
// PK: the products two at a time (v_pk_mul_f32, each half rounded as the
// scalar multiply), then the adds in k order -- a quarter fewer instructions
// (the 80-VGPR mid2 build keeps the scalar form: the packed one spilled there)
template <bool PK = false>
__device__ __forceinline__ void mid_acc(float& s, const MidBlk& B) {
    if constexpr (PK) {
        const sf2 p0 = sf2{B.a[0], B.a[1]} * sf2{B.b0.x, B.b0.y}, p1 = sf2{B.a[2], B.a[3]} * sf2{B.b0.z, B.b0.w};
        const sf2 p2 = sf2{B.a[4], B.a[5]} * sf2{B.b1.x, B.b1.y}, p3 = sf2{B.a[6], B.a[7]} * sf2{B.b1.z, B.b1.w};
        s += p0.x; s += p0.y; s += p1.x; s += p1.y;
        s += p2.x; s += p2.y; s += p3.x; s += p3.y;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) s += B.a[j] * (j < 4 ? B.b0[j] : B.b1[j - 4]);
    }
}
// s = sum_k a[k * as] * b[k], k = 0..n8-1 (n8 a multiple of 8) in the
// reference's order, product rounded before each add
template <bool PK = false>
__device__ __forceinline__ float mid_dot(const float* a, int as, const float* b, int n8) {
    float s = 0.0f;
    MidBlk c, x;
    mid_load(c, a, as, b, 0);
    int k = 0;
    for (; k + 16 < n8; k += 16) {
        mid_load(x, a, as, b, k + 8);
        mid_acc<PK>(s, c);
        mid_load(c, a, as, b, k + 16);
        mid_acc<PK>(s, x);
    }
    if (k + 8 < n8) {
        mid_load(x, a, as, b, k + 8);
        mid_acc<PK>(s, c);
        mid_acc<PK>(s, x);
    } else {
        mid_acc<PK>(s, c);
    }
    return s;
}
// s = sum_k a[k] * b[k] over a 16-byte-aligned LDS row a (per lane, 16-byte
// loads) and the broadcast b, k = 0..n8-1 in order
struct RowDotBlk {
    sf4 a0, a1, b0, b1;
};
__device__ __forceinline__ void rowdot_load(RowDotBlk& B, const float* a, const float* b, int k) {
    B.a0 = *reinterpret_cast<const sf4*>(a + k);
    B.a1 = *reinterpret_cast<const sf4*>(a + k + 4);
    B.b0 = *reinterpret_cast<const sf4*>(b + k);
    B.b1 = *reinterpret_cast<const sf4*>(b + k + 4);
}
template <bool PK = false>
__device__ __forceinline__ void rowdot_acc(float& s, const RowDotBlk& B) {
    if constexpr (PK) {
        const sf2 p0 = sf2{B.a0.x, B.a0.y} * sf2{B.b0.x, B.b0.y}, p1 = sf2{B.a0.z, B.a0.w} * sf2{B.b0.z, B.b0.w};
        const sf2 p2 = sf2{B.a1.x, B.a1.y} * sf2{B.b1.x, B.b1.y}, p3 = sf2{B.a1.z, B.a1.w} * sf2{B.b1.z, B.b1.w};
        s += p0.x; s += p0.y; s += p1.x; s += p1.y;
        s += p2.x; s += p2.y; s += p3.x; s += p3.y;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) s += (j < 4 ? B.a0[j] : B.a1[j - 4]) * (j < 4 ? B.b0[j] : B.b1[j - 4]);
    }
}
template <bool PK = false>
__device__ __forceinline__ float mid_dot_row(const float* a, const float* b, int n8) {
    float s = 0.0f;
    RowDotBlk c, x;
    rowdot_load(c, a, b, 0);
    int k = 0;
    for (; k + 16 < n8; k += 16) {
        rowdot_load(x, a, b, k + 8);
        rowdot_acc<PK>(s, c);
        rowdot_load(c, a, b, k + 16);
        rowdot_acc<PK>(s, x);
    }
    if (k + 8 < n8) {
        rowdot_load(x, a, b, k + 8);
        rowdot_acc<PK>(s, c);
        rowdot_acc<PK>(s, x);
    } else {
        rowdot_acc<PK>(s, c);
    }
    return s;
}

// s = sum_k v[k], k = 0..n8-1 in order (v 16-byte aligned, per lane)
__device__ __forceinline__ void mid_add8(float& s, sf4 a, sf4 b) {
    s += a.x; s += a.y; s += a.z; s += a.w;
    s += b.x; s += b.y; s += b.z; s += b.w;
}
__device__ __forceinline__ float mid_sum(const float* v, int n8) {
    float s = 0.0f;
    sf4 c0 = *reinterpret_cast<const sf4*>(v), c1 = *reinterpret_cast<const sf4*>(v + 4), x0, x1;
    int k = 0;
    for (; k + 16 < n8; k += 16) {
        x0 = *reinterpret_cast<const sf4*>(v + k + 8);
        x1 = *reinterpret_cast<const sf4*>(v + k + 12);
        mid_add8(s, c0, c1);
        c0 = *reinterpret_cast<const sf4*>(v + k + 16);
        c1 = *reinterpret_cast<const sf4*>(v + k + 20);
        mid_add8(s, x0, x1);
    }
    if (k + 8 < n8) {
        x0 = *reinterpret_cast<const sf4*>(v + k + 8);
        x1 = *reinterpret_cast<const sf4*>(v + k + 12);
        mid_add8(s, c0, c1);
        mid_add8(s, x0, x1);
    } else {
        mid_add8(s, c0, c1);
    }
    return s;
}

// A walk over nb blocks with the loads of D - 1 blocks in flight ahead of the
// block being summed (round 6, k_solve_mid2): at 8 waves per CU an LDS read
// returns later than one block's few instructions take, which left every
// block of the one-block-ahead forms above waiting.  buf[u] holds block
// jb + u; a load past the end re-reads the last block (harmless, no branch).
// Blocks are summed in order, so every sum keeps its k order.
template <int D, class Blk, class Load, class Acc>
__device__ __forceinline__ void ring_walk(int nb, Load load, Acc acc) {
    Blk buf[D];
#pragma unroll
    for (int u = 0; u < D - 1; ++u) load(buf[u], u < nb ? u : nb - 1);
    int jb = 0;
    for (; jb + D <= nb; jb += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const int nxt = jb + u + D - 1;
            load(buf[(u + D - 1) % D], nxt < nb ? nxt : nb - 1);
            acc(buf[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < D - 1; ++u)
        if (jb + u < nb) acc(buf[u]);
}
// mid_dot_row / mid_sum / mid_dot through ring_walk (n8 a multiple of 8, >= 8)
template <int D, bool PK = false>
__device__ __forceinline__ float mid_dot_row_ring(const float* a, const float* b, int n8) {
    float s = 0.0f;
    ring_walk<D, RowDotBlk>(
        n8 >> 3, [&](RowDotBlk& B, int j) { rowdot_load(B, a, b, 8 * j); },
        [&](const RowDotBlk& B) { rowdot_acc<PK>(s, B); });
    return s;
}
struct SumBlk {
    sf4 c0, c1;
};
template <int D>
__device__ __forceinline__ float mid_sum_ring(const float* v, int n8) {
    float s = 0.0f;
    ring_walk<D, SumBlk>(
        n8 >> 3,
        [&](SumBlk& B, int j) {
            B.c0 = *reinterpret_cast<const sf4*>(v + 8 * j);
            B.c1 = *reinterpret_cast<const sf4*>(v + 8 * j + 4);
        },
        [&](const SumBlk& B) { mid_add8(s, B.c0, B.c1); });
    return s;
}
template <int D, bool PK = false>
__device__ __forceinline__ float mid_dot_ring(const float* a, int as, const float* b, int n8) {
    float s = 0.0f;
    ring_walk<D, MidBlk>(
        n8 >> 3, [&](MidBlk& B, int j) { mid_load(B, a, as, b, 8 * j); },
        [&](const MidBlk& B) { mid_acc<PK>(s, B); });
    return s;
}

// The split entries of one off-diagonal Qd value q in max form, qp =
// (q<0?0:q) and qn = (q>0?0:-q) (bit-identical to the reference's
// max(0,+-q)+0.0f products).  FAST (the problem's Qd holds no NaN,
// checked when it is staged): one v_max_f32 each.  v_max_f32 differs from the
// selects only on a NaN and in the sign of a zero result, and a signed zero
// does not change a sum that starts at +0.0f and only ever adds products of
// non-negative values (never -0).  Inline asm: the compiler's own fmaxf
// quiets each operand first (one more instruction per value).
template <bool FAST>
__device__ __forceinline__ void split_q(float q, float& qp, float& qn) {
    if constexpr (FAST) {
        asm("v_max_f32 %0, %1, 0" : "=v"(qp) : "v"(q));
        asm("v_max_f32_e64 %0, -%1, 0" : "=v"(qn) : "v"(q));
    } else {
        qp = (q < 0.0f) ? 0.0f : q;
        qn = (q > 0.0f) ? 0.0f : -q;
    }
}

// 8 terms of an update row: Qd[i][k..k+7] (16-byte loads of the row) and the
// broadcast y_k..y_k+7
struct RowBlk {
    sf4 q0, q1, y0, y1;
};
__device__ __forceinline__ void row_load(RowBlk& B, const float* q, const float* y, int k) {
    B.q0 = *reinterpret_cast<const sf4*>(q + k);
    B.q1 = *reinterpret_cast<const sf4*>(q + k + 4);
    B.y0 = *reinterpret_cast<const sf4*>(y + k);
    B.y1 = *reinterpret_cast<const sf4*>(y + k + 4);
}
// (ap, an) ride as one packed pair: one v_pk_mul_f32 and one v_pk_add_f32 per
// k (each half of a packed op rounds as the scalar op).  DIAG: the block
// holds the diagonal k = i of some lanes' rows, where the literal
// max(0,+-q_ii)+Theta_i (dp, dn) replaces the split entries.  FUSE adds aq +=
// y_k Qd[i][k] (Y'Qd's column i when Qd is bit-symmetric, computeCost :652,
// :110).
template <bool DIAG, bool FUSE, bool FAST>
__device__ __forceinline__ void row_block(const RowBlk& B, int k, int i, float dp, float dn, sf2& acc, float& aq) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float q = j < 4 ? B.q0[j] : B.q1[j - 4];
        const float yk = j < 4 ? B.y0[j] : B.y1[j - 4];
        float qp, qn;
        split_q<FAST>(q, qp, qn);
        if constexpr (DIAG) {
            const bool d = (k + j == i);
            qp = d ? dp : qp;
            qn = d ? dn : qn;
        }
        acc += sf2{qp, qn} * sf2{yk, yk};
        if constexpr (FUSE) aq += yk * q;
    }
}
template <bool FUSE, bool FAST>
__device__ __forceinline__ void row_step(const RowBlk& B, int k, int w0, int i, float dp, float dn, sf2& acc,
                                         float& aq) {
    if (k >= w0 && k < w0 + 64) row_block<true, FUSE, FAST>(B, k, i, dp, dn, acc, aq);
    else row_block<false, FUSE, FAST>(B, k, i, dp, dn, acc, aq);
}

// update row i (updateY2, PQP_CPU.c:603-618) into nxt[i], k = 0..nk-1 in
// order, the diagonal test only in the blocks of the 64 columns that hold the
// diagonal of this wave's rows; FUSE: tq[i] = (Y'Qd)_i * y_i as well
template <bool FUSE, bool FAST>
__device__ __forceinline__ void mid_update(const float* Qd, int ldn, int nk, const float* cur, float* nxt, float* tq,
                                           const float* dP, const float* dN, const float* Fdn, const float* Fdp,
                                           int i) {
    const float* q = Qd + i * ldn;
    const float dp = dP[i], dn = dN[i];
    const int w0 = __builtin_amdgcn_readfirstlane(i & ~63);  // rows of a wave share it
    sf2 acc = {0.0f, 0.0f};
    float aq = 0.0f;
    RowBlk c, x;
    row_load(c, q, cur, 0);
    int k = 0;
    for (; k + 16 < nk; k += 16) {
        row_load(x, q, cur, k + 8);
        row_step<FUSE, FAST>(c, k, w0, i, dp, dn, acc, aq);
        row_load(c, q, cur, k + 16);
        row_step<FUSE, FAST>(x, k + 8, w0, i, dp, dn, acc, aq);
    }
    if (k + 8 < nk) {
        row_load(x, q, cur, k + 8);
        row_step<FUSE, FAST>(c, k, w0, i, dp, dn, acc, aq);
        row_step<FUSE, FAST>(x, k + 8, w0, i, dp, dn, acc, aq);
    } else {
        row_step<FUSE, FAST>(c, k, w0, i, dp, dn, acc, aq);
    }
    const float y = cur[i];
    if constexpr (FUSE) tq[i] = aq * y;   // (Y'Qd)_i * Y_i, computeCost :652-655
    const float num = acc.y + 1.0f * Fdn[i];  // :611
    const float den = acc.x + 1.0f * Fdp[i];  // :612
    nxt[i] = num / den * y;                   // :594
}

template <int NT>
__global__ void __launch_bounds__(NT) k_solve_mid(SolveArgs A0, SolveState* __restrict__ st0) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SolveArgs A = problem_at(A0, blockIdx.x);
    SolveState* st = st0 + blockIdx.x;
    if (st->status == kStatusDone || st->status == kStatusCapped) return;
    const int N = A.N, M = A.M;
    const bool conv = (A.mode != kModeFixed);
    const MidLayout L = mid_layout(N, M, conv);
    const int ldn = L.ldn, ldm = L.ldm, ldg = L.ldg, ldi = L.ldi, nk = L.nk, mk = L.mk;
    float* Qd = lds + L.Qd;
    float* Gp = lds + L.Gp;
    float* Qi = lds + L.Qi;
    float* Qp = lds + L.Qp;
    float* tq = lds + L.tq;
    float* tM = lds + L.tM;
    float* Us = lds + L.Us;
    float* tu = lds + L.tu;
    float* fu = lds + L.fu;
    float* Fp = lds + L.Fp;
    float* dP = lds + L.dP;
    float* dN = lds + L.dN;
    float* Fdp = lds + L.Fdp;
    float* Fdn = lds + L.Fdn;
    float* Fd = lds + L.Fd;
    float* Kp = lds + L.Kp;
    float* sc = lds + L.sc;  // [0] (Y'Qd).Y  [1] Fd.Y  [2] stop
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

    // ---- stage the problem (once per launch; padding zero) ----
    for (int e = tid; e < L.total; e += NT) lds[e] = 0.0f;
    __syncthreads();
    for (int e = tid; e < N * N; e += NT) {
        const int i = e / N, k = e - i * N;
        Qd[i * ldn + k] = A.Qd[e];
    }
    for (int i = tid; i < N; i += NT) {
        const float f = A.Fd[i];
        Fd[i] = f;
        Fdp[i] = max_ref(0.0f, f);   // matrixPos(Fdp, Fd) :703
        Fdn[i] = max_ref(0.0f, -f);  // matrixNeg(Fdn, Fd) :704
    }
    if (conv) {
        for (int e = tid; e < N * M; e += NT) {  // Gp' (Gp'Y walks rows of it with 16-byte loads)
            const int i = e / M, j = e - i * M;
            Gp[j * ldg + i] = A.Gp[e];
        }
        for (int i = tid; i < N; i += NT) Gp[mk * ldg + i] = A.Fd[i];  // Fd.Y rides as row mk
        for (int e = tid; e < M * M; e += NT) {
            const int i = e / M, j = e - i * M;
            Qi[i * ldi + j] = A.Qinv[e];
            Qp[i * ldm + j] = A.Qp[e];
        }
        for (int i = tid; i < N; i += NT) Kp[i] = A.Kp[i];
        for (int j = tid; j < M; j += NT) Fp[j] = A.Fp[j];
    }
    float* cur = lds + L.ya;
    float* nxt = lds + L.yb;
    for (int i = tid; i < N; i += NT) cur[i] = st->resume ? A.Y[i] : 1000.0f;  // initMat(Y,1000) :710
    __syncthreads();
    // computeTheta (:503-519) and the diagonal literals of computeQdp_theta /
    // computeQdn_theta (:524-537); Qd bit-symmetric?  any NaN in it?
    int asym = 0, nan = 0;
    for (int i = tid; i < N; i += NT) {
        const float* row = Qd + i * ldn;
        float s = 0.0f;
        for (int k = 0; k < N; ++k) {
            s += max_ref(0.0f, -row[k]) * 1.0f;
            if (k > i && __float_as_uint(row[k]) != __float_as_uint(Qd[k * ldn + i])) asym = 1;
            if (row[k] != row[k]) nan = 1;
        }
        const float th = max_ref(s, 5.0f), qii = row[i];
        dP[i] = max_ref(0.0f, qii) + 1.0f * th;
        dN[i] = max_ref(0.0f, -qii) + 1.0f * th;
    }
    const bool sym = !__syncthreads_or(asym);
    const bool fast = !__syncthreads_or(nan);
    const float Md = conv ? A.Md[0] : 0.0f, Mp = conv ? A.Mp[0] : 0.0f;

    const bool may_update = (A.mode != kModeTerminate);
    const int nR = may_update ? (N + 63) & ~63 : 0;  // update-row items (whole waves)
    const int nT = conv ? (M + 64) & ~63 : 0;        // tM items, and Fd.Y on item M
    const int nU = (M + 63) & ~63;                   // U (and later (U'Qp).U) items
    // M < 64: the tM wave goes straight on to U = -Qp_inv tM in phase A (it
    // finishes long before the update rows), so phase B and its barrier vanish
    const bool uInA = conv && M < 64 && nR + 64 <= NT;
    const int nRC = (N + 63) & ~63;                  // checkFeas row items
    const bool quadC = nRC < NT;                     // a wave free for the (Y'Qd).Y sum in phase C
    float Jp_last = 0.0f, Jd_last = 0.0f;            // costs of the last feasible terminate() (wave 0)
    bool costs = false;
    long long h = st->h;
    long long done_here = 0;
    int status = kStatusContinue;
    bool was_feasible = false;
    // timing trace (pqp_tune_trace "mid"): wave 0's phase totals, each wave's
    // phase-A busy time, in shader cycles
    const bool tr = A0.trace && (int)blockIdx.x < A0.trace_n;
    unsigned long long t_top = 0, t_ph = 0, acc_busyA = 0, acc_ph[4] = {0, 0, 0, 0}, n_it = 0;
    for (;;) {
        if (tr) t_top = t_ph = __builtin_amdgcn_s_memtime();
        const bool fuse = conv && was_feasible && sym;   // (Y'Qd).Y terms inside the update rows
        const bool spec = conv && was_feasible && !sym;  // ... in columns beside them
        const bool have_tq = fuse || spec;
        // ---------------- phase A ----------------
        const int nA = nR + nT + (spec ? nR : 0);
        for (int it = tid; it < nA; it += NT) {
            if (it < nR) {
                const int i = it;
                if (i < N) {
                    if (fast) {
                        if (fuse) mid_update<true, true>(Qd, ldn, nk, cur, nxt, tq, dP, dN, Fdn, Fdp, i);
                        else mid_update<false, true>(Qd, ldn, nk, cur, nxt, tq, dP, dN, Fdn, Fdp, i);
                    } else {
                        if (fuse) mid_update<true, false>(Qd, ldn, nk, cur, nxt, tq, dP, dN, Fdn, Fdp, i);
                        else mid_update<false, false>(Qd, ldn, nk, cur, nxt, tq, dP, dN, Fdn, Fdp, i);
                    }
                }
            } else if (it < nR + nT) {
                const int j = it - nR;
                if (j <= M) {  // tM_j = Gp'Y + Fp (:355-356); item M: Fd.Y (:656-657)
                    const float s = mid_dot_row(Gp + (j < M ? j : mk) * ldg, cur, nk);
                    if (j < M) tM[j] = s + 1.0f * Fp[j];
                    else sc[1] = s;
                }
            } else {
                const int j = it - nR - nT;
                if (j < N)  // Y'Qd, column access :110
                    tq[j] = mid_dot(Qd + j, ldn, cur, nk) * cur[j];
            }
        }
        if (uInA && tid >= nR && tid < nR + 64) {
            // the tM wave: its own tM stores are visible to its own later LDS
            // reads (a wave's LDS accesses complete in order)
            __builtin_amdgcn_wave_barrier();
            const int i = tid - nR;
            if (i < M) Us[i] = -mid_dot_row(Qi + i * ldi, tM, mk);  // :357-358
        }
        if (tr) acc_busyA += __builtin_amdgcn_s_memtime() - t_top;
        __syncthreads();
        if (tr) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            acc_ph[0] += t - t_ph;
            t_ph = t;
            ++n_it;
        }
        if (conv) {
            // ---------------- phase B: U = -Qp_inv tM (M >= 64) ----------------
            if (!uInA) {
                for (int i = tid; i < M; i += NT) Us[i] = -mid_dot_row(Qi + i * ldi, tM, mk);  // :357-358
                __syncthreads();
            }
            if (tr) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                acc_ph[1] += t - t_ph;
                t_ph = t;
            }
            // ------- phase C: checkFeas; (Y'Qd).Y on a free wave -------
            int bad = 0;
            if (tid < nRC) {
                for (int i = tid; i < N; i += NT) {
                    const float s = mid_dot(Gp + i, ldg, Us, mk);  // row i of Gp: column i of Gp'
                    const float kp = Kp[i];
                    if (s > kp + max_ref((float)(kTol * kp), (float)kTol)) bad = 1;
                }
            } else if (have_tq && tid == nRC) {
                sc[0] = mid_sum(tq, nk);
            }
            const bool infeasible = __syncthreads_or(bad);
            if (tr) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                acc_ph[2] += t - t_ph;
                t_ph = t;
            }
            int stop = 0;
            if (!infeasible) {
                // ------------ phase D: the dot products' terms ------------
                const int nN = have_tq ? 0 : (N + 63) & ~63;
                for (int it = tid; it < nU + nN; it += NT) {
                    if (it < nU) {
                        const int j = it;
                        if (j < M) {
                            tu[j] = mid_dot(Qp + j, ldm, Us, mk) * Us[j];  // (U'Qp).U
                            fu[j] = Fp[j] * Us[j];                         // Fp'U
                        }
                    } else {
                        const int j = it - nU;
                        if (j < N)  // (Y'Qd).Y
                            tq[j] = mid_dot(Qd + j, ldn, cur, nk) * cur[j];
                    }
                }
                __syncthreads();
                // ------------ phase E: the sums left, the costs, the tests ------------
                if (wave == 0) {
                    float s = 0.0f;
                    if (lane < 3 && (lane > 0 || !(have_tq && quadC)))  // one instruction stream
                        s = mid_sum(lane == 0 ? tq : (lane == 1 ? tu : fu), lane == 0 ? nk : mk);
                    const float quad_d = (have_tq && quadC) ? sc[0] : rdl(s, 0);
                    const float lin_d = sc[1], quad_p = rdl(s, 1), lin_p = rdl(s, 2);
                    float Jd = 0.0f;
                    Jd = (float)((double)Jd + 0.5 * (double)quad_d);
                    Jd += lin_d;
                    Jd += Md / 2;
                    float Jp = 0.0f;
                    Jp = (float)((double)Jp + 0.5 * (double)quad_p);
                    Jp += lin_p;
                    Jp += Mp / 2;
                    const int sp = gap_stop(Jp, Jd) ? 1 : 0;  // :683-685
                    if (lane == 0) sc[2] = (float)sp;
                    // to SolveState once, at the end: a global store here would
                    // hold the barrier below for its round trip every iterate
                    Jp_last = Jp;
                    Jd_last = Jd;
                    costs = true;
                }
                __syncthreads();
                stop = sc[2] != 0.0f;
                if (tr) acc_ph[3] += __builtin_amdgcn_s_memtime() - t_ph;
            }
            was_feasible = !infeasible;
            if (A.mode == kModeTerminate) {
                if (tid == 0) st->last_stop = stop;
                status = kStatusDone;
                break;
            }
            if (stop) {
                status = kStatusDone;
                break;
            }
            if (A.max_updates > 0 && h - 1 >= A.max_updates) {
                status = kStatusCapped;
                break;
            }
        } else if (h >= A.num_iter) {  // while(h < NUM_ITER)
            status = kStatusDone;
            break;
        }
        if (done_here >= A.chunk) {
            status = kStatusContinue;
            break;
        }
        // accept the update computed in phase A.  The next phase A reads cur
        // (written before the last barrier) and writes nxt and tq (read by
        // nobody until after the next barrier: tq's last readers, in phases B
        // and E, are behind one).
        float* t = cur;
        cur = nxt;
        nxt = t;
        ++h;
        ++done_here;
    }
    for (int i = tid; i < N; i += NT) A.Y[i] = cur[i];
    if (conv)
        for (int i = tid; i < M; i += NT) A.U[i] = Us[i];
    if (tr && lane == 0) {  // totals over the launches of a solve
        unsigned long long* T = A0.trace + 16 * (size_t)blockIdx.x;
        if (wave < 8) T[8 + wave] += acc_busyA;
        if (wave == 0) {
            for (int p = 0; p < 4; ++p) T[p] += acc_ph[p];
            T[4] += n_it;
        }
    }
    if (tid == 0) {
        if (costs) {
            st->Jp = Jp_last;
            st->Jd = Jd_last;
            st->have_costs = 1;
        }
        st->h = h;
        st->status = status;
        st->resume = 1;
        if (status == kStatusContinue && A.pending) atomicAdd(A.pending, 1);
    }
}

// <solve-mid2> (bench.py hashes the text up to </solve-mid2>: the VALU counter records in profiles/pmc_valu.json are keyed by it)
// ---------------------------------------------------------------------------
// k_solve_mid2: path 3 with terminate() pipelined beside the update (round 4).
// updateY2 needs only Y_h (PQP_CPU.c:603-618), so phase s of the loop runs,
// on disjoint waves of one workgroup per problem, everything that needs only
// what earlier phases produced:
//   UW (waves 0 .. nUW-1, nUW = ceil(N / 32)): Y_{s+1} = updateY2(Y_s).  Lanes
//       2r + side hold one side of row 32w + r: side 1 sums den's terms
//       max(0,q)*y (:609), side 0 sums min(q,0)*y = -(max(0,-q)*y) (exact:
//       negation is exact and rounding is sign-symmetric), so num = 0 - sum
//       (:608; the 0 - turns the all-zero sum's -0 back into the reference's
//       +0).  One v_med3_f32(q, 0, +-inf) per k gives either side's split
//       entry: three instructions per k instead of the one-lane-per-row form's
//       two v_max_f32 and a packed multiply and add.  The literal
//       (max(0,+-q_ii) + Theta_i) * y on the diagonal (:524-537).  The lanes of
//       a pair meet once per row: num / den * y (:594).  Where Qd holds a NaN,
//       or Y_s a NaN or inf (whose sign the negated form could flip), the
//       phase takes the selects of the reference's max instead.
//   T  (wave nUW): tM = Gp'Y_s + Fp (computeUfromY :355-356) on lanes j < M,
//       Fd.Y_s (computeCost :656) on lane M, then U_s = -Qp_inv tM (:357-358).
//   C  (the other waves): terminate(Y_{s-1}) -- checkFeas's rows Gp U_{s-1}
//       (:632-641, one lane per row), the (U'Qp).U and Fp.U terms and the
//       three cost sums (:648-666) on the last C wave -- and, on the row
//       waves, (Y_s'Qd)_j Y_s,j (:652-655, Qd column j) for the next phase.
// After the phase barrier every thread reads the C waves' flags and sums and
// takes terminate(s-1)'s decision (:673-687) itself.  Y_s and Y_{s+1} are
// dropped when it stops (or a launch ends); each launch starts its pipeline
// from the saved Y_h.  Every sum keeps the reference's operands and order:
// the same bits as k_solve_mid.  N <= 160, M < 64 (nUW + 1 + 2 <= 8 waves);
// other mid sizes, and terminate() alone, stay on k_solve_mid.
// Band (round 5): the update rows and the Y'Qd rows of a wave sum only the k
// from the first to the last nonzero entry of the wave's rows and columns
// (found once, when Qd is staged; the diagonal always inside).  While every
// y_k is finite, a zero entry's term is +-0, and a sum that starts at +0.0f
// (and so is never -0) is unchanged by adding +-0: the skipped terms change
// no bit.  A phase whose Y_s holds a NaN or inf sums every k.  A dense Qd
// has the whole range as its band; an MPC problem's stage structure (the
// horizon leg: 28-row blocks) leaves a wave of 32 or 64 rows 28-84 of the k.
// ---------------------------------------------------------------------------
// Round 6 (profiles/r06/mid2_ring_qpt_r06t.txt, bits identical): the T, C and
// cost waves' row dots and sums keep their loads three blocks deep and the
// strided checkFeas dots two (ring_walk), and Qp is staged transposed so the
// cost wave's U'Qp terms read 16-byte rows instead of strided words: H = 4 /
// 5 28.2 / 57.4 -> 25.2 / 51.2 ms, the dense n_dual 140 companion 84.7 -> 77.7
#ifndef PQP_M2_TSUM  // k_solve_mid2: the T wave's spare lane 63 takes the cost wave's longest sum
#define PQP_M2_TSUM 1
#endif
#ifndef PQP_M2_QPT  // k_solve_mid2: Qp kept transposed (the cost wave's U'Qp terms read rows)
#define PQP_M2_QPT 1
#endif
#ifndef PQP_M2_RING  // k_solve_mid2's row dots and sums: loads this many blocks deep (0: one ahead)
#define PQP_M2_RING 3
#endif
#ifndef PQP_M2_RINGD  // ... and the strided dots (checkFeas rows)
#define PQP_M2_RINGD 2
#endif
#ifndef PQP_M2_RING_LEAN  // the same in the 80-VGPR builds (H = 2 / 3: 11.0 / 25.8 -> 10.0 / 23.8 ms at 2)
#define PQP_M2_RING_LEAN 2
#endif
#ifndef PQP_M2_RINGD_LEAN
#define PQP_M2_RINGD_LEAN 2
#endif
template <bool PK, int D>
__device__ __forceinline__ float m2_dot_row(const float* a, const float* b, int n8) {
    if constexpr (D >= 2) return mid_dot_row_ring<D, PK>(a, b, n8);
    else return mid_dot_row<PK>(a, b, n8);
}
template <bool PK, int D>
__device__ __forceinline__ float m2_dot(const float* a, int as, const float* b, int n8) {
    if constexpr (D >= 2) return mid_dot_ring<D, PK>(a, as, b, n8);
    else return mid_dot<PK>(a, as, b, n8);
}
template <int D>
__device__ __forceinline__ float m2_sum(const float* v, int n8) {
    if constexpr (D >= 2) return mid_sum_ring<D + 1>(v, n8);
    else return mid_sum(v, n8);
}
struct Mid2Layout {
    int nk, mk, ldn, ldm, ldg, ldi;
    int y, tq, dP, dN, Fdp, Fdn, Kp, tM, Us, tu, fu, Fp, fdy, flag, band, sums, ones, Qd, Gp, Qi, Qp, total;
};
__host__ __device__ inline Mid2Layout mid2_layout(int N, int M, bool conv) {
    Mid2Layout L;
    L.nk = round8(N);
    L.mk = round8(M);
    L.ldn = L.nk + 4;
    L.ldm = PQP_M2_QPT ? L.mk + 4 : L.mk + 1;  // QPT: Qp' rows, 16-byte aligned
    L.ldg = L.nk + 4;
    L.ldi = L.mk + 4;
    int o = 0;
    L.y = o;    o += 3 * L.nk;      // Y_{s-1}, Y_s, Y_{s+1}: ring by s mod 3
    L.tq = o;   o += 2 * L.nk;      // (Y_s'Qd)_j Y_s,j: ring by s & 1
    L.dP = L.tq;                    // the diagonal literals: read into registers before the first
    L.dN = L.tq + L.nk;             // phase, then their space is the tq ring's
    L.Fdp = o;  o += L.nk;
    L.Fdn = o;  o += L.nk;
    L.flag = o; o += 16;            // [0..11] checkFeas flags per C row wave; [12 + s&1] Y non-finite
    L.band = o; o += 16;            // nonzero k-bands (mid2_band): 64-row groups [0..2] lo, [3..5] hi; 32-row [6..10], [11..15]
    if (conv) {
        L.Kp = o;   o += L.nk;
        L.tM = o;   o += L.mk;
        L.Us = o;   o += 2 * L.mk;  // U_s: ring by s & 1
        L.tu = o;   o += L.mk;
        L.fu = o;   o += L.mk;
        L.Fp = o;   o += L.mk;
        L.fdy = o;  o += 4;         // Fd.Y_s: ring by s & 1
        L.sums = o; o += 4;         // (Y'Qd).Y, (U'Qp).U, Fp.U of iterate s-1
        L.ones = o; o += PQP_M2_TSUM ? L.nk : 0;  // 1.0f: T's lane 63 sums (Y'Qd)_j Y_j as a dot
    } else {
        L.Kp = L.tM = L.Us = L.tu = L.fu = L.Fp = L.fdy = L.sums = L.ones = 0;
    }
    L.Qd = o;  o += L.nk * L.ldn;
    if (conv) {
        L.Gp = o;  o += (L.mk + 1) * L.ldg;  // Gp' with Fd as row mk
        L.Qi = o;  o += L.mk * L.ldi;
        L.Qp = o;  o += L.mk * L.ldm;
    } else {
        L.Gp = L.Qi = L.Qp = 0;
    }
    L.total = o;
    return L;
}
// waves of each role: UW (PAIR: 32 rows per wave, lane sides; else 64 rows,
// one lane per row), T (one), C (ceil(N/64) row waves and the cost wave)
__host__ __device__ inline int mid2_uw(int N, bool pair) { return pair ? (N + 31) / 32 : (N + 63) / 64; }
// C row waves: `crows` checkFeas rows (and Y'Qd terms) per wave, 64 or 32
__host__ __device__ inline int mid2_cr(int N, int crows) { return (N + crows - 1) / crows; }
__host__ __device__ inline int mid2_waves(int N, bool conv, bool pair, int crows) {
    return mid2_uw(N, pair) + (conv ? 1 + mid2_cr(N, crows) + 1 : 0);
}
// mid2 takes (N, M) in converge or fixed mode when T fits one wave and the
// workgroup 16
__host__ __device__ inline bool mid2_fits(int N, int M, bool conv, bool pair, int crows) {
    return (!conv || M < 64) && mid2_waves(N, conv, pair, crows) <= 16;
}

// 8 terms of one side of update row i (k .. k+7).  FAST: the v_med3_f32
// split (no NaN in Qd, Y finite); else the reference's selects on +y.  DIAG:
// the block holds the diagonal of some rows of this wave.
template <bool FAST, bool DIAG>
__device__ __forceinline__ void mid2_block(float& acc, sf4 q0, sf4 q1, sf4 y0, sf4 y1, int k, int w0, int side,
                                           float lim, float dv) {
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float qk = j < 4 ? q0[j] : q1[j - 4];
        if constexpr (FAST) {
            asm("v_med3_f32 %0, %1, 0, %2" : "=v"(t[j]) : "v"(qk), "v"(lim));
        } else {
            t[j] = side ? ((qk < 0.0f) ? 0.0f : qk) : ((qk > 0.0f) ? 0.0f : -qk);
        }
        if constexpr (DIAG) {
            // k + j is the diagonal of row w0 + r, r = k + j - w0 (uniform): its
            // two lanes 2r, 2r + 1 take the literal, by a mask made on the
            // scalar unit -- one v_cndmask per k instead of a compare and a select
            const unsigned long long m = 3ull << (2 * (k + j - w0));
            asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(t[j]) : "v"(t[j]), "v"(dv), "s"(m));
        }
    }
    // products two at a time (v_pk_mul_f32, each half rounded as the scalar
    // multiply), then the adds in k order
    const sf2 p0 = sf2{t[0], t[1]} * sf2{y0.x, y0.y};
    const sf2 p1 = sf2{t[2], t[3]} * sf2{y0.z, y0.w};
    const sf2 p2 = sf2{t[4], t[5]} * sf2{y1.x, y1.y};
    const sf2 p3 = sf2{t[6], t[7]} * sf2{y1.z, y1.w};
    acc += p0.x; acc += p0.y; acc += p1.x; acc += p1.y;
    acc += p2.x; acc += p2.y; acc += p3.x; acc += p3.y;
}
// one side of update row i, k = klo..khi-1 in order (the row group's band,
// mid2_band), the next block's LDS reads in flight while a block is summed
template <bool FAST>
__device__ __forceinline__ float mid2_side(const float* q, const float* y, int klo, int khi, int i, int side,
                                           float lim, float dv, int w0) {
    float acc = 0.0f;
    sf4 q0 = *reinterpret_cast<const sf4*>(q + klo), q1 = *reinterpret_cast<const sf4*>(q + klo + 4);
    sf4 y0 = *reinterpret_cast<const sf4*>(y + klo), y1 = *reinterpret_cast<const sf4*>(y + klo + 4);
    for (int k = klo; k < khi; k += 8) {
        const int kn = (k + 8 < khi) ? k + 8 : k;  // next block (the last one re-read at the end)
        const sf4 nq0 = *reinterpret_cast<const sf4*>(q + kn), nq1 = *reinterpret_cast<const sf4*>(q + kn + 4);
        const sf4 ny0 = *reinterpret_cast<const sf4*>(y + kn), ny1 = *reinterpret_cast<const sf4*>(y + kn + 4);
        if (k >= w0 && k < w0 + 32) mid2_block<FAST, true>(acc, q0, q1, y0, y1, k, w0, side, lim, dv);
        else mid2_block<FAST, false>(acc, q0, q1, y0, y1, k, w0, side, lim, dv);
        q0 = nq0; q1 = nq1; y0 = ny0; y1 = ny1;
    }
    return acc;
}

// 8 terms of update row w0 + lane, both sides packed (k_solve_mid's
// row_block).  DIAG: the block lies in the 64 columns of the wave's diagonal;
// column k + j is the diagonal of lane k + j - w0 only, which takes the literal
// by a mask made on the scalar unit (two v_cndmask per k, no compare)
// product first in the one-lane-per-row update (round 6, H = 5 51.5 -> 49.9 ms,
// dense n_dual 140 78.1 -> 73.8, profiles/r06/mid2_pf_r06v.txt); FAST then also
// needs Qd finite and Y finite and >= 0 (the staged and per-phase flags)
#ifndef PQP_M2_PF
#define PQP_M2_PF 1
#endif
// (the one-lane-per-row build's last, 12-row update wave at n_dual 140 as lane
// sides: slower, H = 5 50.3 -> 50.9 ms, dense 73.8 -> 79.9; profiles/r06/
// mid2_tail_lean_r06w.txt)
template <bool DIAG, bool FAST, bool PF = false>
__device__ __forceinline__ void mid2_rblock(const RowBlk& B, int k, int w0, float dp, float dn, sf2& acc) {
    if constexpr (PF) {
        // product first (round 6): p = q y_k, then max(0, p) and max(0, -p) --
        // the same values as max(0, +-q) y_k while Qd is finite and every y_k
        // finite and >= 0 (PF: the staged Qd flag and the phase's Y flag; a
        // zero's sign never matters in these sums): one multiply per k instead
        // of two.  The diagonal's literal products (dp, dn = dP_i y_i, dN_i y_i,
        // formed by the caller) replace the split terms by the scalar mask.
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
            const sf2 q2 = j < 4 ? sf2{B.q0[j], B.q0[j + 1]} : sf2{B.q1[j - 4], B.q1[j - 3]};
            const sf2 y2 = j < 4 ? sf2{B.y0[j], B.y0[j + 1]} : sf2{B.y1[j - 4], B.y1[j - 3]};
            const sf2 p = q2 * y2;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float tp, tn;
                asm("v_max_f32 %0, %1, 0" : "=v"(tp) : "v"(p[h]));
                asm("v_max_f32_e64 %0, -%1, 0" : "=v"(tn) : "v"(p[h]));
                if constexpr (DIAG) {
                    const unsigned long long m = 1ull << (k + j + h - w0);
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(tp) : "v"(tp), "v"(dp), "s"(m));
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(tn) : "v"(tn), "v"(dn), "s"(m));
                }
                acc += sf2{tp, tn};
            }
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float q = j < 4 ? B.q0[j] : B.q1[j - 4];
        const float yk = j < 4 ? B.y0[j] : B.y1[j - 4];
        float qp, qn;
        split_q<FAST>(q, qp, qn);
        if constexpr (DIAG) {
            const unsigned long long m = 1ull << (k + j - w0);
            asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(qp) : "v"(qp), "v"(dp), "s"(m));
            asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(qn) : "v"(qn), "v"(dn), "s"(m));
        }
        acc += sf2{qp, qn} * sf2{yk, yk};
    }
}
// SMASK: the scalar-mask diagonal (the 128-VGPR build; the 80-VGPR build
// keeps k_solve_mid's per-lane compare: the masks' SGPRs made it spill more,
// H = 2 / 3 +2 / +4 %, profiles/r05/band)
template <bool FAST, bool SMASK, bool PF = false>
__device__ __forceinline__ void mid2_rstep(const RowBlk& B, int k, int w0, int i, float dp, float dn, sf2& acc) {
    if constexpr (SMASK) {
        if (k >= w0 && k < w0 + 64) mid2_rblock<true, FAST, PF>(B, k, w0, dp, dn, acc);
        else mid2_rblock<false, FAST, PF>(B, k, w0, dp, dn, acc);
    } else {
        float aq = 0.0f;
        row_step<false, FAST>(B, k, w0, i, dp, dn, acc, aq);
    }
}
// one update row on one lane, both sides packed (k_solve_mid's form):
// Y_next[i] = num / den * y_i (PQP_CPU.c:603-618), k = klo..khi-1
template <bool FAST, bool SMASK, bool PF = false>
__device__ __forceinline__ float mid2_row(const float* q, const float* y, int klo, int khi, int i, float dp,
                                          float dn, float fdn, float fdp, int w0) {
    static_assert(!PF || (FAST && SMASK), "the product-first form is a form of the scalar-mask max form");
    if constexpr (PF) {  // mid2_rblock's product-first form takes the diagonal's products
        const float yi = y[i];
        dp = dp * yi;
        dn = dn * yi;
    }
    sf2 acc = {0.0f, 0.0f};
    RowBlk c, x;
    row_load(c, q, y, klo);
    int k = klo;
    for (; k + 16 < khi; k += 16) {
        row_load(x, q, y, k + 8);
        mid2_rstep<FAST, SMASK, PF>(c, k, w0, i, dp, dn, acc);
        row_load(c, q, y, k + 16);
        mid2_rstep<FAST, SMASK, PF>(x, k + 8, w0, i, dp, dn, acc);
    }
    if (k + 8 < khi) {
        row_load(x, q, y, k + 8);
        mid2_rstep<FAST, SMASK, PF>(c, k, w0, i, dp, dn, acc);
        mid2_rstep<FAST, SMASK, PF>(x, k + 8, w0, i, dp, dn, acc);
    } else {
        mid2_rstep<FAST, SMASK, PF>(c, k, w0, i, dp, dn, acc);
    }
    const float num = acc.y + 1.0f * fdn;  // :611
    const float den = acc.x + 1.0f * fdp;  // :612
    return num / den * y[i];               // :594
}

#ifndef PQP_M2_DEC1  // k_solve_mid2, converge mode, lane-side build of up to 16 waves: one wave takes each decision
#define PQP_M2_DEC1 1
#endif
#ifndef PQP_M2PK_T  // k_solve_mid2 (1024 build): packed products in T's dots, checkFeas, the Y'Qd terms, U'Qp
#define PQP_M2PK_T 1
#endif
#ifndef PQP_M2PK_F
#define PQP_M2PK_F 0  // (packed: the 1024 build spilled)
#endif
#ifndef PQP_M2PK_C
#define PQP_M2PK_C 0  // (packed: the 1024 build spilled)
#endif
#ifndef PQP_M2PK_Q
#define PQP_M2PK_Q 1
#endif
// BAND: the band sums (the lean one-lane-per-row build also comes without
// them, for N <= 64: one row group, whose band is all k on any MPC problem,
// and the band's registers cost that build 7 %, profiles/r05/band)
template <int MAXT, bool PAIR, int MINW = 1, bool BAND = true>
__global__ void __launch_bounds__(MAXT, MINW) k_solve_mid2(SolveArgs A0, SolveState* __restrict__ st0) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SolveArgs A = problem_at(A0, blockIdx.x);
    SolveState* st = st0 + blockIdx.x;
    if (st->status == kStatusDone || st->status == kStatusCapped) return;
    const int N = A.N, M = A.M;
    const bool conv = (A.mode == kModeConverge);
    const Mid2Layout L = mid2_layout(N, M, conv);
    const int ldn = L.ldn, ldm = L.ldm, ldg = L.ldg, ldi = L.ldi, nk = L.nk, mk = L.mk;
    float* Qd = lds + L.Qd;
    float* Gp = lds + L.Gp;
    float* Qi = lds + L.Qi;
    float* Qp = lds + L.Qp;
    float* Yr = lds + L.y;
    float* tq = lds + L.tq;
    float* dP = lds + L.dP;
    float* dN = lds + L.dN;
    float* Fdp = lds + L.Fdp;
    float* Fdn = lds + L.Fdn;
    float* Kp = lds + L.Kp;
    float* tM = lds + L.tM;
    float* Us = lds + L.Us;
    float* tu = lds + L.tu;
    float* fu = lds + L.fu;
    float* Fp = lds + L.Fp;
    float* fdy = lds + L.fdy;
    float* sums = lds + L.sums;
    int* flag = reinterpret_cast<int*>(lds + L.flag);  // [0..11] checkFeas per C row wave, [12 + p] Y non-finite
    int* band = reinterpret_cast<int*>(lds + L.band);
    const int NT = blockDim.x;  // 64 * mid2_waves(N, conv, PAIR, crows)
    const int tid = threadIdx.x, lane = tid & 63;
    const int nUW = mid2_uw(N, PAIR), wT = nUW, wC0 = nUW + 1;
#ifndef PQP_M2_PERM
#define PQP_M2_PERM 1
#endif
    // Roles over the hardware waves: the SIMDs take waves w and w + 4.  With
    // three update waves, T, three C row waves and the cost wave (the
    // one-lane-per-row build, 128 < N <= 160: one workgroup per CU), the C row
    // waves -- whose chains set the phase -- share a SIMD with the short third
    // update wave and with T, instead of with the first two update waves:
    // hardware waves 0..7 take roles C0, C1, UW0, UW1, UW2, T, C2, cost
    // (H = 5: 59.8 -> 57.0 ms).  The lane-side build with four update waves
    // (96 < N <= 128, two workgroups per CU): C0, C1, cost, T, UW3, UW0, UW1,
    // UW2 -- the C row waves beside the short fourth update wave and the first
    // (H = 4: 31.7 -> 28.1 ms).  The lean build with two update waves was
    // slower so (C0, C1 alone on a SIMD: H = 3 26.3 -> 27.7 ms) and keeps
    // its order (profiles/r05/band/perm_*.txt).
    int wave = tid >> 6;
    if constexpr (PQP_M2_PERM && !PAIR && MINW == 1)
        if (NT == 512 && nUW == 3) wave = wave < 2 ? wave + 4 : (wave < 6 ? wave - 2 : wave);
#ifndef PQP_M2_PERM4
#define PQP_M2_PERM4 1
#endif
    if constexpr (PQP_M2_PERM4 && PAIR && MINW == 1)
        if (NT == 512 && nUW == 4) {
            wave = wave < 3 ? wave + 5 : (wave == 3 ? 4 : (wave == 4 ? 3 : wave - 5));
        }
    // C waves that take checkFeas rows and the Y'Qd terms (crows each); wave
    // wC0 + nCR the costs
    const int crows = (NT / 64 - nUW - 2 >= (N + 31) / 32) ? 32 : 64;
    const int nCR = mid2_cr(N, crows);
    const int wDec = wC0 + nCR;  // converge mode: the cost wave also takes each decision
    // T's lane 63 sums (Y'Qd).Y (below): H = 5 51.9 -> 50.3 ms, dense n_dual 140
    // 75.4 -> 74.1; the lane-side build (two problems per CU) measured 25.75 ->
    // 25.93 at H = 4 and keeps the cost wave's sum (profiles/r06/mid2_tsum_r06x.txt)
    const bool tsum = PQP_M2_TSUM && !PAIR && M < 63;
    constexpr bool PK = MINW == 1;  // packed dot products (the 80-VGPR build spilled with them)
    constexpr int RD = MINW == 1 ? PQP_M2_RING : PQP_M2_RING_LEAN;     // load depth of the row dots / sums
    constexpr int RDD = MINW == 1 ? PQP_M2_RINGD : PQP_M2_RINGD_LEAN;  // ... of the strided dots
    // one decision per phase (on the cost wave) where the phase is bound by
    // VALU issue -- the lane-side build, two problems per CU at n_dual 112:
    // 38.9 -> 37.7 ms; elsewhere the single decider's latency between the
    // phase's two barriers cost more than the instructions it saved (H = 2 /
    // 3 / 5: +9 / +3.5 / +2.4 %, profiles/r05/mid2_dec_pk_ab.txt)
    constexpr bool DEC1 = PQP_M2_DEC1 && PAIR && MINW == 1;

    // ---- stage the problem (once per launch; padding zero) ----
    for (int e = tid; e < L.total; e += NT) lds[e] = 0.0f;
    __syncthreads();
    for (int e = tid; e < N * N; e += NT) {
        const int i = e / N, k = e - i * N;
        Qd[i * ldn + k] = A.Qd[e];
    }
    for (int i = tid; i < N; i += NT) {
        const float f = A.Fd[i];
        Fdp[i] = max_ref(0.0f, f);   // matrixPos(Fdp, Fd) :703
        Fdn[i] = max_ref(0.0f, -f);  // matrixNeg(Fdn, Fd) :704
    }
    if (conv) {
        for (int e = tid; e < N * M; e += NT) {
            const int i = e / M, j = e - i * M;
            Gp[j * ldg + i] = A.Gp[e];
        }
        for (int i = tid; i < N; i += NT) Gp[mk * ldg + i] = A.Fd[i];  // Fd.Y rides as row mk
        for (int e = tid; e < M * M; e += NT) {
            const int i = e / M, j = e - i * M;
            Qi[i * ldi + j] = A.Qinv[e];
            if (PQP_M2_QPT) Qp[j * ldm + i] = A.Qp[e];
            else Qp[i * ldm + j] = A.Qp[e];
        }
        for (int i = tid; i < N; i += NT) Kp[i] = A.Kp[i];
        for (int j = tid; j < M; j += NT) Fp[j] = A.Fp[j];
        if (PQP_M2_TSUM)
            for (int k = tid; k < nk; k += NT) lds[L.ones + k] = 1.0f;
    }
    long long h0 = st->h;
    int ynf = 0;
    for (int i = tid; i < N; i += NT) {
        const float y = st->resume ? A.Y[i] : 1000.0f;  // initMat(Y,1000) :710
        Yr[(int)(h0 % 3) * nk + i] = y;
        if (!(PQP_M2_PF ? (y >= 0.0f && y <= 3.402823466e38f) : fabsf(y) <= 3.402823466e38f)) ynf = 1;
    }
    __syncthreads();
    // computeTheta (:503-519), the diagonal literals (:524-537); any NaN in
    // Qd?  Qd bit-symmetric (then Y'Qd's column j is row j's dot, read 16 bytes
    // at a time)?
    // The band of each row group (mid2_band): the k from the first to the
    // last nonzero (or NaN) of its rows and columns, the diagonal included,
    // rounded out to blocks of 8; lo kept as nk - lo so that both ends are
    // maxima over the zeroed words.
    int nan = 0, asym = 0, qinf = 0;
    const bool dense = (A.tiny_flags & kMid2Dense) != 0;
    for (int i = tid; i < N; i += NT) {
        const float* row = Qd + i * ldn;
        float s = 0.0f;
        int lo = i, hi = i;
        for (int k = 0; k < N; ++k) {
            s += max_ref(0.0f, -row[k]) * 1.0f;
            if (row[k] != row[k]) nan = 1;
            if (fabsf(row[k]) == __builtin_inff()) qinf = 1;
            if (k > i && __float_as_uint(row[k]) != __float_as_uint(Qd[k * ldn + i])) asym = 1;
            if (row[k] != 0.0f || Qd[k * ldn + i] != 0.0f) {
                lo = k < lo ? k : lo;
                hi = k > hi ? k : hi;
            }
        }
        if (dense) {
            lo = 0;
            hi = nk - 1;
        }
        const int lo8 = lo & ~7, hi8 = (hi + 8) & ~7;
        atomicMax(&band[i >> 6], nk - lo8);
        atomicMax(&band[3 + (i >> 6)], hi8);
        atomicMax(&band[6 + (i >> 5)], nk - lo8);
        atomicMax(&band[11 + (i >> 5)], hi8);
        const float th = max_ref(s, 5.0f), qii = row[i];
        dP[i] = max_ref(0.0f, qii) + 1.0f * th;
        dN[i] = max_ref(0.0f, -qii) + 1.0f * th;
    }
    const bool sym = !__syncthreads_or(asym);
    const bool fast = !__syncthreads_or(nan);
    const bool qfinite = fast && !__syncthreads_or(qinf);  // the product-first update form's Qd condition
    bool y_nonfinite = __syncthreads_or(ynf);
    const float Md = conv ? A.Md[0] : 0.0f, Mp = conv ? A.Mp[0] : 0.0f;

    // per-lane constants of the update role.  PAIR: lane 2r + side holds one
    // side of row 32 w + r (side 0 sums the negated num terms, so its diagonal
    // literal is -dN); else lane l holds row 64 w + l, both sides packed.
    const int side = lane & 1;
    const int urow = PAIR ? 32 * wave + (lane >> 1) : 64 * wave + lane;
    const bool uw = wave < nUW && urow < N;
    const float lim = side ? __builtin_inff() : -__builtin_inff();
    const float dpr = uw ? dP[urow] : 0.0f, dnr = uw ? dN[urow] : 0.0f;
    const float dv = side ? dpr : -dnr;
    const float fdv = uw ? (side ? Fdp[urow] : Fdn[urow]) : 0.0f;
    const float fdp = uw ? Fdp[urow] : 0.0f, fdn = uw ? Fdn[urow] : 0.0f;
    // uniform: the diagonal masks are scalar
    const int w0 = __builtin_amdgcn_readfirstlane(PAIR ? 32 * wave : 64 * wave);
    __syncthreads();  // dP / dN read: the tq ring may be written from here on
    const bool tr = A0.trace && (int)blockIdx.x < A0.trace_n;
    unsigned long long busy = 0, t_phase = 0, n_ph = 0, t0 = 0;
    unsigned long long seg_a = 0;  // trace: the first part of the T / C / cost roles

    float Jp_last = 0.0f, Jd_last = 0.0f;
    bool costs = false;
    int status = kStatusContinue;
    long long t_out = h0;
    // After phase s's barrier, on every thread: terminate(s-1)'s decision
    // (converge mode) or the fixed-mode loop test.  Returns true to leave the
    // loop (status and t_out set).  Every wave runs its role in a loop of its
    // own (so each role's registers are allocated apart), each iteration with
    // the same two barriers and this same uniform decision.
    auto decide = [&](long long s) -> bool {
        if (conv) {
            if (s == h0) return false;  // nothing pending in the launch's first phase
            const long long t = s - 1;
            int infeasible = 0;
            for (int c = 0; c < nCR; ++c) infeasible |= flag[c];
            int stop = 0;
            if (!infeasible) {
                float Jd = 0.0f;
                Jd = (float)((double)Jd + 0.5 * (double)sums[0]);
                Jd += fdy[t & 1];
                Jd += Md / 2;
                float Jp = 0.0f;
                Jp = (float)((double)Jp + 0.5 * (double)sums[1]);
                Jp += sums[2];
                Jp += Mp / 2;
                stop = gap_stop(Jp, Jd) ? 1 : 0;  // :683-685
                Jp_last = Jp;
                Jd_last = Jd;
                costs = true;
            }
            t_out = t;
            if (stop) { status = kStatusDone; return true; }
            if (A.max_updates > 0 && t - 1 >= A.max_updates) { status = kStatusCapped; return true; }
            if (t - h0 >= A.chunk) { status = kStatusContinue; return true; }
            return false;
        }
        t_out = s;
        if (s >= A.num_iter) { status = kStatusDone; return true; }  // while(h < NUM_ITER)
        if (s - h0 >= A.chunk) { status = kStatusContinue; return true; }
        return false;
    };
    // The phase's end: its barrier, then (converge mode, DEC1) the cost wave alone
    // takes terminate(s-1)'s decision and posts it in LDS (flag[14] leave,
    // flag[15] t_out - h0), and a second barrier; every wave reads it (one
    // decision per phase instead of one per wave: its double-precision gap
    // tests were ~7 % of the kernel's VALU instructions).  Between the two
    // barriers every wave also reads Y_{s+1}'s non-finite flag; the next
    // phase writes the flags only after the second barrier.
    auto phase_end = [&](long long s) -> bool {
        if (tr) busy += __builtin_amdgcn_s_memtime() - t0;
        __syncthreads();
        if (tr && wave == 0) {
            t_phase += __builtin_amdgcn_s_memtime() - t0;
            ++n_ph;
        }
        bool leave;
        if (conv && DEC1) {
            if (wave == wDec) {
                const bool d = decide(s);
                if (lane == 0) {
                    flag[14] = d ? 1 : 0;
                    flag[15] = (int)(t_out - h0);
                }
            }
            y_nonfinite = flag[12 + (int)((s + 1) & 1)] != 0;  // Y_{s+1}, the next phase's Y_s
            __syncthreads();
            leave = flag[14] != 0;
            if (leave) t_out = h0 + flag[15];
        } else {
            leave = decide(s);
            y_nonfinite = flag[12 + (int)((s + 1) & 1)] != 0;
            __syncthreads();
        }
        return leave;
    };

    if (wave < nUW) {
        // ---------------- UW: Y_{s+1} = updateY2(Y_s) ----------------
        const float* q = Qd + (uw ? urow : 0) * ldn;
        // the wave's band (its rows' nonzero k), valid while Y_s is finite
        // (read from LDS once: per phase it cost 4-8 %, profiles/r05/band)
        const int bg = PAIR ? 6 + wave : wave;
        const int blo = BAND ? __builtin_amdgcn_readfirstlane(nk - band[bg]) : 0;
        const int bhi = BAND ? __builtin_amdgcn_readfirstlane(band[bg + (PAIR ? 5 : 3)]) : nk;
        for (long long s = h0;; ++s) {
            const float* ycur = Yr + (int)(s % 3) * nk;
            float* ynext = Yr + (int)((s + 1) % 3) * nk;
            // Y_{s+1}'s non-finite flag goes to slot (s+1)&1; slot s&1 was last
            // read before the previous phase's second barrier
            if (wave == 0 && lane == 0) flag[12 + (int)(s & 1)] = 0;
            if (tr) t0 = __builtin_amdgcn_s_memtime();
            // a zero entry's term is +-0 while y_k is finite, and the sum (from
            // +0.0f, never -0) is unchanged by it: the terms outside the band
            // are skipped exactly; a non-finite Y_s (0 * inf = NaN) takes every k
            const int klo = (BAND && !y_nonfinite) ? blo : 0, khi = (BAND && !y_nonfinite) ? bhi : nk;
            if (uw) {
                if constexpr (PAIR) {
                    float acc = (fast && !y_nonfinite) ? mid2_side<true>(q, ycur, klo, khi, urow, side, lim, dv, w0)
                                                       : mid2_side<false>(q, ycur, klo, khi, urow, side, lim, side ? dv : -dv, w0);
                    if (fast && !y_nonfinite && !side) acc = 0.0f - acc;  // num's terms were summed negated
                    const float v = acc + 1.0f * fdv;                     // num += Fdn :611; den += Fdp :612
                    const float other = __shfl_xor(v, 1);
                    if (side) {
                        const float y = ycur[urow];
                        const float yn = other / v * y;  // updY :594
                        ynext[urow] = yn;
                        if (!(PQP_M2_PF ? (yn >= 0.0f && yn <= 3.402823466e38f) : fabsf(yn) <= 3.402823466e38f))
                            flag[12 + (int)((s + 1) & 1)] = 1;
                    }
                } else {
                    // k_solve_mid's row (max form, or the selects where Qd holds a NaN)
                    float yn;
                    if (PQP_M2_PF && MINW == 1 && qfinite && !y_nonfinite)
                        yn = mid2_row<true, MINW == 1, PQP_M2_PF && MINW == 1>(q, ycur, klo, khi, urow, dpr, dnr, fdn, fdp, w0);
                    else if (fast)
                        yn = mid2_row<true, MINW == 1>(q, ycur, klo, khi, urow, dpr, dnr, fdn, fdp, w0);
                    else
                        yn = mid2_row<false, MINW == 1>(q, ycur, klo, khi, urow, dpr, dnr, fdn, fdp, w0);
                    ynext[urow] = yn;
                    if (!(PQP_M2_PF ? (yn >= 0.0f && yn <= 3.402823466e38f) : fabsf(yn) <= 3.402823466e38f))
                            flag[12 + (int)((s + 1) & 1)] = 1;
                }
            }
            if (phase_end(s)) break;  // (its second barrier: the flags are read before the next phase writes)
        }
    } else if (conv && wave == wT) {
        // ------------- T: tM = Gp'Y_s + Fp, Fd.Y_s, U_s = -Qp_inv tM -------------
        const float* grow = Gp + (lane < M ? lane : mk) * ldg;
        const float* qirow = Qi + (lane < M ? lane : 0) * ldi;
        const float fpl = lane < M ? Fp[lane] : 0.0f;
        // lane 63, spare when M < 63, sums the previous iterate's (Y'Qd)_j Y_j
        // (:652-655) as the dot with a vector of ones, in j order (x * 1.0f is
        // x): the cost wave's 1 + n_dual-long single-lane chain rides in T's
        // own instructions (round 6)
        const bool l63 = tsum && lane == 63;
        for (long long s = h0;; ++s) {
            const float* ycur = Yr + (int)(s % 3) * nk;
            if (tr) t0 = __builtin_amdgcn_s_memtime();
            if (lane <= M || l63) {
                const float d = m2_dot_row<PK && PQP_M2PK_T, RD>(l63 ? tq + ((s - 1) & 1) * nk : grow,
                                                                 l63 ? lds + L.ones : ycur, nk);
                if (lane < M) tM[lane] = d + 1.0f * fpl;  // :355-356
                else if (lane == M) fdy[s & 1] = d;       // Fd.Y :656
                else sums[0] = d;                         // (Y'Qd).Y of iterate s-1
            }
            __builtin_amdgcn_wave_barrier();
            if (tr) seg_a += __builtin_amdgcn_s_memtime() - t0;
            if (lane < M) Us[(s & 1) * mk + lane] = -m2_dot_row<PK && PQP_M2PK_T, RD>(qirow, tM, mk);  // :357-358
            if (phase_end(s)) break;
        }
    } else if (conv) {
        // ---------------- C: terminate(Y_{s-1}); Y_s'Qd ----------------
        const int cw = wave - wC0;
        // the Y'Qd rows' band (the crows-row group of this wave)
        const int cg = cw < nCR ? (crows == 64 ? cw : 6 + cw) : 0;
        const int clo = BAND ? __builtin_amdgcn_readfirstlane(nk - band[cg]) : 0;
        const int chi = BAND ? __builtin_amdgcn_readfirstlane(band[cg + (crows == 64 ? 3 : 5)]) : nk;
        for (long long s = h0;; ++s) {
            const float* ycur = Yr + (int)(s % 3) * nk;
            const bool pend = s > h0;
            const float* Uo = Us + ((s - 1) & 1) * mk;
            if (tr) t0 = __builtin_amdgcn_s_memtime();
            if (cw < nCR) {
                const int l = cw * crows + lane;  // rows [cw * crows, +crows): lanes < crows
                const int lend = lane < crows ? N : 0;
                int bad = 0;
                if (pend)
                    for (int i = l; i < lend; i += crows * nCR) {
                        const float g = m2_dot<PK && PQP_M2PK_F, RDD>(Gp + i, ldg, Uo, mk);  // row i of Gp . U  :636
                        const float kp = Kp[i];
                        if (g > kp + max_ref((float)(kTol * kp), (float)kTol)) bad = 1;  // compare :338
                    }
                // the vote over every lane's rows, taken with the whole wave
                // active (inside `lane == 0` it would see lane 0's rows only)
                const bool any_bad = __any(bad);
                if (pend && lane == 0) flag[cw] = any_bad ? 1 : 0;
                if (tr) seg_a += __builtin_amdgcn_s_memtime() - t0;
                float* tqs = tq + (s & 1) * nk;  // for terminate(s), next phase
                // (Y'Qd)_j Y_j :652-655 over the band while Y_s is finite (as
                // the update's sums); column j = row j when Qd is symmetric
                const bool cb = BAND && !y_nonfinite;
                const int klo = cb ? clo : 0, kn = (cb ? chi : nk) - klo;
                for (int j = l; j < lend; j += crows * nCR)
                    tqs[j] = (sym ? m2_dot_row<PK && PQP_M2PK_C, RD>(Qd + j * ldn + klo, ycur + klo, kn)
                                  : m2_dot<PK && PQP_M2PK_C, RDD>(Qd + klo * ldn + j, ldn, ycur + klo, kn)) * ycur[j];
            } else if (pend && cw == nCR) {
                if (lane < M) {
                    tu[lane] = (PQP_M2_QPT ? m2_dot_row<PK && PQP_M2PK_Q, RD>(Qp + lane * ldm, Uo, mk)
                                           : m2_dot<PK && PQP_M2PK_Q, RDD>(Qp + lane, ldm, Uo, mk)) *
                               Uo[lane];  // (U'Qp).U terms :652-655 (column lane of Qp)
                    fu[lane] = Fp[lane] * Uo[lane];                         // Fp'U :656-657
                }
                __builtin_amdgcn_wave_barrier();
                if (tr) seg_a += __builtin_amdgcn_s_memtime() - t0;
                if (lane < 3 && !(tsum && lane == 0)) {
                    const float* v = lane == 0 ? tq + ((s - 1) & 1) * nk : (lane == 1 ? tu : fu);
                    const float r = m2_sum<RD>(v, lane == 0 ? nk : mk);
                    sums[lane] = r;
                }
            }
            if (phase_end(s)) break;
        }
    } else {
        // fixed mode: the waves beside the update keep the barrier count
        for (long long s = h0;; ++s) {
            if (tr) t0 = __builtin_amdgcn_s_memtime();
            if (phase_end(s)) break;
        }
    }
    // the result: Y and U of iterate t_out (converge) or Y_s (fixed)
    const float* yo = Yr + (int)(t_out % 3) * nk;
    for (int i = tid; i < N; i += NT) A.Y[i] = yo[i];
    if (conv)
        for (int i = tid; i < M; i += NT) A.U[i] = Us[(t_out & 1) * mk + i];
    if (tr && lane == 0) {
        unsigned long long* T = A0.trace + 16 * (size_t)blockIdx.x;
        if (wave < 8) T[8 + wave] += busy;
        if (wave == 0) {
            T[0] += t_phase;
            T[4] += n_ph;
        }
        // the first part of T (Gp'Y), of the first C wave (checkFeas) and of
        // the cost wave (the U'Qp terms); each role's rest is its busy - this
        if (conv && wave == wT) T[1] += seg_a;
        if (conv && wave == wC0) T[2] += seg_a;
        if (conv && wave == wC0 + nCR) T[3] += seg_a;
    }
    // the state: written by the wave that took the decisions
    if ((conv && DEC1) ? (wave == wDec && lane == 0) : tid == 0) {
        if (costs) {
            st->Jp = Jp_last;
            st->Jd = Jd_last;
            st->have_costs = 1;
        }
        st->h = t_out;
        st->status = status;
        st->resume = 1;
        if (status == kStatusContinue && A.pending) atomicAdd(A.pending, 1);
    }
}
// </solve-mid2>

size_t solve_mid_lds_bytes(int N, int M, bool conv) {
    return sizeof(float) * (size_t)mid_layout(N, M, conv).total;
}
constexpr size_t kMidLdsBudget = 150 * 1024;

static hipError_t launch_mid_grid(int B, const SolveArgs& a0, SolveState* st, hipStream_t s) {
    SolveArgs a = a0;
    if (g_tune.mid2_dense) a.tiny_flags |= kMid2Dense;
    const bool conv2 = a.mode == kModeConverge;
    // the update rows as lane sides where that measured faster: the horizon
    // sweep (profiles/r04/mid2_arms.jsonl) at n_dual 112 (H = 4) 40.4 vs 43.4
    // ms, and slower at 56, 84 and 140 (more waves per workgroup, fewer
    // workgroups per CU); mid2_pair 1 / 2 force either form
    const bool pair = g_tune.mid2_pair == 1 || (g_tune.mid2_pair == 0 && a.N >= 96 && a.N <= 128);
    // 32 rows per C wave measured slower at every H (more waves per workgroup);
    // so did 32-row C waves running checkFeas and the Y'Qd terms side by side on
    // the two halves of their lanes (round 6: H = 5 58.2 -> 68.0 ms, the dense
    // n_dual 140 companion 84.9 -> 92.2, H = 2 11.2 -> 19.1;
    // profiles/r06/mid2_csplit_dropped_r06g.jsonl)
    const int crows = 64;
    if (a.mode != kModeTerminate && !g_tune.mid_v1 && a.N >= g_tune.mid2_min_n &&
        mid2_fits(a.N, a.M, conv2, pair, crows)) {
        const size_t lds = sizeof(float) * (size_t)mid2_layout(a.N, a.M, conv2).total;
        if (lds <= kMidLdsBudget) {
            const int nt = 64 * mid2_waves(a.N, conv2, pair, crows);
            // workgroups of <= 6 waves: the build held to 80 VGPRs (6 waves per
            // SIMD), so as many problems share a CU as LDS allows (n_dual 56: 6
            // instead of 4, 84: 4 instead of 2)
            const bool lean = nt <= 384;  // (the 128-VGPR build here: H = 2 / 3 13.1 / 37.2 vs 11.2 / 30.2 ms, profiles/r04)
            if (lean && pair) hipLaunchKernelGGL((k_solve_mid2<384, true, 6>), dim3(B), dim3(nt), lds, s, a, st);
            else if (lean && a.N > 64) hipLaunchKernelGGL((k_solve_mid2<384, false, 6>), dim3(B), dim3(nt), lds, s, a, st);
            else if (lean) hipLaunchKernelGGL((k_solve_mid2<384, false, 6, false>), dim3(B), dim3(nt), lds, s, a, st);
            else if (pair) hipLaunchKernelGGL((k_solve_mid2<1024, true>), dim3(B), dim3(nt), lds, s, a, st);
            else hipLaunchKernelGGL((k_solve_mid2<1024, false>), dim3(B), dim3(nt), lds, s, a, st);
            g_last_batch_kernel = 3;
            return hipGetLastError();
        }
    }
    g_last_batch_kernel = 2;
    const bool conv = a.mode != kModeFixed;
    const size_t lds = solve_mid_lds_bytes(a.N, a.M, conv);
    const int nt = mid_threads(a.N, a.M, conv);
    if (nt == 128) hipLaunchKernelGGL((k_solve_mid<128>), dim3(B), dim3(128), lds, s, a, st);
    else if (nt == 256) hipLaunchKernelGGL((k_solve_mid<256>), dim3(B), dim3(256), lds, s, a, st);
    else hipLaunchKernelGGL((k_solve_mid<512>), dim3(B), dim3(512), lds, s, a, st);
    return hipGetLastError();
}

size_t solve_small_lds_bytes(int N, int M) { return sizeof(float) * (size_t)small_layout(N, M).total; }

static hipError_t launch_small_grid(int B, const SolveArgs& a, SolveState* st, hipStream_t s) {
    hipLaunchKernelGGL(k_solve_small, dim3(B), dim3(256), solve_small_lds_bytes(a.N, a.M), s, a, st);
    return hipGetLastError();
}
hipError_t launch_solve_small(const SolveArgs& a, SolveState* st, hipStream_t s) { return launch_small_grid(1, a, st, s); }

// ---------------------------------------------------------------------------
// Host-side launchers (declared in pqp_launch.h)
// ---------------------------------------------------------------------------

template <int U, bool NTL>
static void launch_iterate_t(int B, const float* QdT, long long qstride, int ldq, int N, const float* theta,
                             const float* Fd, int ldv, const float* Y0, float* Y, int updates, hipStream_t s) {
    const size_t lds = (size_t)2 * ldq * sizeof(float);
    if (N <= 256)
        hipLaunchKernelGGL((k_batch_iterate<64, U, NTL>), dim3(B), dim3(64), lds, s, QdT, qstride, ldq, N, theta, Fd,
                           ldv, Y0, Y, updates);
    else
        hipLaunchKernelGGL((k_batch_iterate<256, U, NTL>), dim3(B), dim3(256), lds, s, QdT, qstride, ldq, N, theta,
                           Fd, ldv, Y0, Y, updates);
}

static hipError_t launch_batch_iterate_one(int B, const float* QdT, long long qstride, int ldq, int N,
                                          const float* theta, const float* Fd, int ldv, const float* Y0, float* Y,
                                          int updates, hipStream_t s);

// Long runs are split into launches of at most kIterPerLaunch updates (each
// continuing from the previous one's Y), so no single launch runs unbounded.
constexpr int kIterPerLaunch = 256;
hipError_t launch_batch_iterate(int B, const float* QdT, long long qstride, int ldq, int N, const float* theta,
                                const float* Fd, int ldv, const float* Y0, float* Y, int updates, hipStream_t s) {
    int done = 0;
    do {
        const int c = (updates - done) < kIterPerLaunch ? (updates - done) : kIterPerLaunch;
        const hipError_t e = launch_batch_iterate_one(B, QdT, qstride, ldq, N, theta, Fd, ldv, done ? Y : Y0, Y, c, s);
        if (e != hipSuccess) return e;
        done += c;
    } while (done < updates);
    return hipSuccess;
}

static hipError_t launch_batch_iterate_one(int B, const float* QdT, long long qstride, int ldq, int N,
                                          const float* theta, const float* Fd, int ldv, const float* Y0, float* Y,
                                          int updates, hipStream_t s) {
    // 16-deep unroll with non-temporal Qd loads: 7.03 TB/s at N = 1024,
    // B = 4096, chunk 10.  The other unroll depths (4, 8, 32), default-policy
    // loads and max-based terms were measured and removed (DESIGN.md section 4,
    // profiles/r01/ab_4096*.txt).
    // n_dual 1024 (the bench shape): k_batch_resident, k_batch_stream with the
    // first two blocks of each problem's Qd pinned to AGPRs, the next two in
    // LDS and the fifth kept in L2 across the launch's iterations (round 6:
    // 23.8 -> 22.1 ms per launch of 10 iterations, the LDS + L2 form alone
    // 22.7; profiles/r06/iterate_ab_r06f.json, scripts/probes/stream_resident.hip;
    // same bits).  iterate_kind 3: the LDS + L2 form.
    const int kind = g_tune.iterate_kind;
    if ((kind == 0 || kind == 3) && N == 1024 && ldq == 1024 && qstride >= (long long)N * ldq &&
        qstride * 4 <= 0x7fffffffLL) {
        const size_t lds = (size_t)2 * ldq * sizeof(float) + (size_t)2 * 16 * 256 * sizeof(float4);
        if (kind == 3)  // LDS + L2 only (3/64 of Qd on chip)
            hipLaunchKernelGGL((k_batch_resident<16, 2>), dim3(B), dim3(256), lds, s, QdT, qstride, ldq, theta, Fd,
                               ldv, Y0, Y, updates);
        else  // + two register blocks (5/64 of Qd on chip)
            hipLaunchKernelGGL((k_batch_resident<16, 2, 2>), dim3(B), dim3(256), lds, s, QdT, qstride, ldq, theta, Fd,
                               ldv, Y0, Y, updates);
        return hipGetLastError();
    }
    // n_dual a multiple of 1024: k_batch_stream, one workgroup per CU, 16 + 16
    // float4 loads per lane kept in flight: 7.24-7.26 TB/s against 7.02-7.04
    // for k_batch_iterate in one process (same bits).  Measured slower and
    // dropped: 8 + 8 (3 workgroups per CU, 7.07-7.09), 32 + 32 (7.10), 16 + 16
    // capped to 256 VGPRs (2 per CU, spills: 7.05), default-policy loads
    // (6.34) -- profiles/r05/iterate_ab_*.json.
    if (kind != 1 && N % 1024 == 0) {
        const size_t lds = (size_t)2 * ldq * sizeof(float);
        hipLaunchKernelGGL((k_batch_stream<16, true>), dim3(B), dim3(256), lds, s, QdT, qstride, ldq, N, theta, Fd,
                           ldv, Y0, Y, updates);
        return hipGetLastError();
    }
    launch_iterate_t<16, true>(B, QdT, qstride, ldq, N, theta, Fd, ldv, Y0, Y, updates, s);
    return hipGetLastError();
}

hipError_t launch_batch_update(int B, const float* QdT, long long qstride, int ldq, int N, const float* theta,
                               const float* Fd, int ldv, const float* Yin, float* Yout, hipStream_t s) {
    const size_t lds = (size_t)ldq * sizeof(float);
    if (N <= 256) {
        dim3 grid(cdiv(N, 4 * 64), B);
        hipLaunchKernelGGL((k_batch_update<64, 16, true>), grid, dim3(64), lds, s, QdT, qstride, ldq, N, theta, Fd,
                           ldv, Yin, Yout);
    } else {
        dim3 grid(cdiv(N, 4 * 256), B);
        hipLaunchKernelGGL((k_batch_update<256, 16, true>), grid, dim3(256), lds, s, QdT, qstride, ldq, N, theta, Fd,
                           ldv, Yin, Yout);
    }
    return hipGetLastError();
}

hipError_t launch_update_split(const float* QpT, const float* QnT, int ldq, int N, const float* Fdp,
                               const float* Fdn, const float* Y, float* Ynext, hipStream_t s) {
    hipLaunchKernelGGL(k_update_split, dim3(cdiv(N, 256)), dim3(256), 0, s, QpT, QnT, ldq, N, Fdp, Fdn, Y, Ynext);
    return hipGetLastError();
}

hipError_t launch_pack_colmajor(int B, const float* Qd, int N, long long in_stride, float* QdT, int ldq,
                                long long qstride, hipStream_t s) {
    dim3 grid(cdiv(N, 32), cdiv(ldq, 32), B);
    hipLaunchKernelGGL(k_pack_colmajor, grid, dim3(256), 0, s, Qd, N, in_stride, QdT, ldq, qstride);
    return hipGetLastError();
}

hipError_t launch_synth_rows(uint32_t seed, long long inst, int N, int M, int row0, int rows, float* Qrows, int ld,
                             float* Fd, float* Md, hipStream_t s) {
    if (rows > 0) {
        dim3 grid(cdiv(ld, SYN_T), cdiv(rows, SYN_T), 1);
        hipLaunchKernelGGL(k_synth_qd, grid, dim3(256), 0, s, seed, inst, N, M, Qrows, ld, (long long)rows * ld, row0,
                           rows);
    }
    if (Fd) hipLaunchKernelGGL(k_synth_fd, dim3(cdiv(N, 256), 1), dim3(256), 0, s, seed, inst, N, M, Fd, N, Md);
    return hipGetLastError();
}

hipError_t launch_theta(int B, const float* QdT, int ldq, long long qstride, int N, float* theta, int ldv,
                        hipStream_t s) {
    const bool wide = (ldq & 3) == 0 && (qstride & 3) == 0 && ((uintptr_t)QdT & 15) == 0;
    for (int b0 = 0; b0 < B; b0 += 65535) {  // grid y is at most 65535
        const int nb = (B - b0) < 65535 ? (B - b0) : 65535;
        const float* q = QdT + (size_t)b0 * (size_t)qstride;
        float* t = theta + (size_t)b0 * ldv;
        if (wide)
            hipLaunchKernelGGL(k_theta4, dim3(cdiv(N, 1024), nb), dim3(256), 0, s, q, ldq, qstride, N, t, ldv);
        else
            hipLaunchKernelGGL(k_theta, dim3(cdiv(N, 256), nb), dim3(256), 0, s, q, ldq, qstride, N, t, ldv);
    }
    return hipGetLastError();
}

hipError_t launch_synth(uint32_t seed, long long inst0, int B, int N, int M, float* QdT, int ldq, long long qstride,
                        float* Fd, int ldv, float* Md, hipStream_t s) {
    // B may exceed the 65535 grid-z limit: chunk it
    for (int b0 = 0; b0 < B; b0 += 65535) {
        const int nb = (B - b0) < 65535 ? (B - b0) : 65535;
        dim3 grid(cdiv(ldq, SYN_T), cdiv(N, SYN_T), nb);
        hipLaunchKernelGGL(k_synth_qd, grid, dim3(256), 0, s, seed, inst0 + b0, N, M, QdT + (size_t)b0 * qstride,
                           ldq, qstride, 0, N);
        hipLaunchKernelGGL(k_synth_fd, dim3(cdiv(N, 256), nb), dim3(256), 0, s, seed, inst0 + b0, N, M,
                           Fd + (size_t)b0 * ldv, ldv, Md ? Md + b0 : nullptr);
    }
    return hipGetLastError();
}

static bool use_tiled(int a, int c) { return !g_tune.matmul_tiled_off && a >= 32 && c >= 32; }
// the packed 128 x 128 form: large outputs whose operands load as float4
static bool use_pk(const void* out, const float* A, int tA, const float* B, int tB, int a, int b, int c, long long sA,
                   long long sB, long long sO) {
    const auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const int ka = tA ? a : b, kb = tB ? b : c;  // each operand's contiguous dimension
    return !g_tune.matmul_tiled_off && !g_tune.matmul_pk_off && a >= 64 && c >= 64 && b >= 1 && ka % 4 == 0 &&
           kb % 4 == 0 && c % 4 == 0 && al(out) && al(A) && al(B) && sA % 4 == 0 && sB % 4 == 0 && sO % 4 == 0;
}
template <int TA, int TB>
static void launch_pk(int nb, float* out, const float* A, const float* B, int a, int b, int c, long long sA,
                      long long sB, long long sO, hipStream_t s) {
    const int tx = cdiv(c, MM8), tpp = tx * cdiv(a, MM8);
    hipLaunchKernelGGL((k_matmul_pk<TA, TB>), dim3(tpp * nb), dim3(256), 0, s, out, A, B, a, b, c, sA, sB, sO, tx,
                       tpp, nb);
}

hipError_t launch_matmul_seq(float* out, const float* A, int tA, const float* B, int tB, int a, int b, int c,
                             hipStream_t s) {
    return launch_matmul_seq_b(1, out, A, tA, B, tB, a, b, c, 0, 0, 0, s);
}
hipError_t launch_matmul_seq_b(int B, float* out, const float* A, int tA, const float* Bm, int tB, int a, int b,
                               int c, long long sA, long long sB, long long sO, hipStream_t s) {
    const long long n = (long long)a * c;
    if (n == 0 || B == 0) return hipSuccess;
    for (int b0 = 0; b0 < B; b0 += 65535) {  // grid y / z limit
        const int nb = (B - b0) < 65535 ? (B - b0) : 65535;
        if (a == 1 && b >= 32 && !g_tune.matmul_tiled_off) {  // x' B (tA is moot for a one-row A)
            hipLaunchKernelGGL(k_vecmat, dim3(cdiv(c, 256), nb), dim3(256), 0, s, out + b0 * sO, A + b0 * sA,
                               Bm + b0 * sB, tB, b, c, sA, sB, sO);
            continue;
        }
        if (c == 1 && !tA && a >= 64 && b >= 32 && !g_tune.matmul_tiled_off) {
            // (the LDS-staged k_matvec_rows only where the rows are not 16-byte
            // aligned: 2.31 vs 2.04-2.12 ms per convertToDual call, profiles/r05)
            if (b % 4 == 0 && sA % 4 == 0 && aligned16(A))
                hipLaunchKernelGGL(k_matvec_lane, dim3(cdiv(a, 64), nb), dim3(64), 0, s, out + b0 * sO,
                                   A + b0 * sA, Bm + b0 * sB, a, b, sA, sB, sO);
            else
                hipLaunchKernelGGL(k_matvec_rows, dim3(cdiv(a, 256), nb), dim3(256), 0, s, out + b0 * sO,
                                   A + b0 * sA, Bm + b0 * sB, a, b, sA, sB, sO);
            continue;
        }
        const long long tiles = (long long)cdiv(c, MM8) * cdiv(a, MM8);
        if (use_pk(out, A, tA, Bm, tB, a, b, c, sA, sB, sO) && tiles * nb < (1LL << 31)) {
            float* o = out + b0 * sO;
            const float *pa = A + b0 * sA, *pb = Bm + b0 * sB;
            if (!tA && !tB) launch_pk<0, 0>(nb, o, pa, pb, a, b, c, sA, sB, sO, s);
            else if (!tA && tB) launch_pk<0, 1>(nb, o, pa, pb, a, b, c, sA, sB, sO, s);
            else if (tA && !tB) launch_pk<1, 0>(nb, o, pa, pb, a, b, c, sA, sB, sO, s);
            else launch_pk<1, 1>(nb, o, pa, pb, a, b, c, sA, sB, sO, s);
        } else if (use_tiled(a, c))
            hipLaunchKernelGGL(k_matmul_tiled, dim3(cdiv(c, MMT), cdiv(a, MMT), nb), dim3(256), 0, s, out + b0 * sO,
                               A + b0 * sA, tA, Bm + b0 * sB, tB, a, b, c, sA, sB, sO);
        else
            hipLaunchKernelGGL(k_matmul_seq, dim3(cdiv(n, 256), nb), dim3(256), 0, s, out + b0 * sO, A + b0 * sA, tA,
                               Bm + b0 * sB, tB, a, b, c, sA, sB, sO);
    }
    return hipGetLastError();
}
hipError_t launch_axpy_b(int B, float* A, const float* Bv, float sign, int n, long long sA, long long sB,
                         hipStream_t s) {
    if (n > 0 && B > 0) hipLaunchKernelGGL(k_axpy, dim3(cdiv(n, 256), B), dim3(256), 0, s, A, Bv, sign, n, sA, sB);
    return hipGetLastError();
}
hipError_t launch_negate_b(int B, float* A, int n, long long sA, hipStream_t s) {
    if (n > 0 && B > 0) hipLaunchKernelGGL(k_negate, dim3(cdiv(n, 256), B), dim3(256), 0, s, A, n, sA);
    return hipGetLastError();
}
hipError_t launch_mp_finish_b(int B, const float* t, const float* Mp6, float* Mp, long long sMp6, hipStream_t s) {
    if (B > 0) hipLaunchKernelGGL(k_mp_finish, dim3(B), dim3(1), 0, s, t, Mp6, Mp, sMp6);
    return hipGetLastError();
}
// ---------------------------------------------------------------------------
// Blocked Gauss_Jordan (PQP_CPU.c:251-326) of many matrices, one workgroup
// each, the pivots taken kGJB at a time.  Element (j,k) of the reference's
// augmented matrix sees, at pivot step i (j != i),
//     t = m_ji / m_ii;  m_jk = m_jk - m_ik * t          (:296-302, no FMA)
// with row i's values "at step i" (after steps 0..i-1) and row j's own m_ji
// read before the step touches row j.  Rows never read each other within a
// step except the pivot row, so the order in which ROWS are processed is
// free; only each element's own sequence of steps is fixed.  Per panel of
// pivots [p0, p0 + nb):
//   1. wave 0 forms the pivot rows "at their step", P_s = row p0+s with steps
//      p0 .. p0+s-1 applied (from P_0 .. P_{s-1}), into LDS;
//   2. every row j (pivot rows included, their own step skipped) is loaded
//      once, takes the nb steps in order from the LDS panel, and is stored.
// Each element thus sees exactly the reference's operations, in its order,
// on the reference's operand values: bit-identical, with one read and one
// write of the matrix per kGJB pivots instead of one per pivot.  A row lives
// in one wave: lane l holds columns 256c + 4l + e (c < C, e < 4), so the
// broadcast of m_ji is one v_readlane and no barrier is needed inside a row's
// steps.  The last panel ends with the row scaling (:307-314) and writes the
// right half straight into res (:316-322).
// ---------------------------------------------------------------------------
template <int C>
__device__ __forceinline__ void gj_load(const float* __restrict__ row, int lane, float (&v)[4 * C]) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const sf4 q = *reinterpret_cast<const sf4*>(row + 256 * c + 4 * lane);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * c + e] = q[e];
    }
}
template <int C>
__device__ __forceinline__ void gj_store(float* __restrict__ row, int lane, const float (&v)[4 * C]) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
        sf4 q;
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] = v[4 * c + e];
        *reinterpret_cast<sf4*>(row + 256 * c + 4 * lane) = q;
    }
}
// m_{row, 256*CP + 4*lo + e}, broadcast from the lane that holds it
template <int C, int CP, int E>
__device__ __forceinline__ float gj_col(const float (&v)[4 * C], int lo) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[4 * CP + E]), lo));
}
// Steps p0 + s, s in [0, ns) (ns <= NB), of the panel whose pivot rows "at
// their step" are P[s][.] (LDS, row stride W) with diagonal Pd[s]; the step of
// pivot row `skip` (this row's own index) is left out.  The panel's pivot
// columns lie in column block CP (p0 % NB == 0, NB divides 256).
template <int C, int NB, int CP>
__device__ __forceinline__ void gj_steps(float (&v)[4 * C], const float* __restrict__ P, const float* __restrict__ Pd,
                                         int W, int p0, int ns, int skip, int lane) {
    const int lo0 = (p0 & 255) >> 2;
#pragma unroll
    for (int s = 0; s < NB; ++s) {
        if (s < ns && p0 + s != skip) {
            float mji;
            switch (s & 3) {
                case 0: mji = gj_col<C, CP, 0>(v, lo0 + (s >> 2)); break;
                case 1: mji = gj_col<C, CP, 1>(v, lo0 + (s >> 2)); break;
                case 2: mji = gj_col<C, CP, 2>(v, lo0 + (s >> 2)); break;
                default: mji = gj_col<C, CP, 3>(v, lo0 + (s >> 2)); break;
            }
            const float t = mji / Pd[s];  // temp (:298)
            const float* prow = P + (size_t)s * W;
            // (a packed form -- v_pk_mul_f32 and v_pk_add_f32 of the negated
            // product -- measured 0.140 vs 0.129 s for 4096 n = 512 inverses:
            // profiles/r04/gj_timing_packed_dropped.json)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const sf4 q = *reinterpret_cast<const sf4*>(prow + 256 * c + 4 * lane);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[4 * c + e] -= q[e] * t;  // (:301)
            }
        }
    }
}
template <int C, int NB>
__device__ __forceinline__ void gj_steps_any(float (&v)[4 * C], const float* P, const float* Pd, int W, int p0, int ns,
                                             int skip, int lane) {
    switch (p0 >> 8) {  // the pivot column block: compile-time register indices
        case 0: gj_steps<C, NB, 0>(v, P, Pd, W, p0, ns, skip, lane); break;
        case 1: if constexpr (C > 1) gj_steps<C, NB, 1>(v, P, Pd, W, p0, ns, skip, lane); break;
        case 2: if constexpr (C > 2) gj_steps<C, NB, 2>(v, P, Pd, W, p0, ns, skip, lane); break;
        case 3: if constexpr (C > 3) gj_steps<C, NB, 3>(v, P, Pd, W, p0, ns, skip, lane); break;
        default: break;  // pivots lie in the left half: column blocks < C / 2 <= 3 for C <= 8
    }
}
// m_{row, col} of the row held in v (any col), broadcast to the whole wave
template <int C>
__device__ __forceinline__ float gj_any_col(const float (&v)[4 * C], int col) {
    const int idx = 4 * (col >> 8) + (col & 3);
    float x = 0.0f;
#pragma unroll
    for (int r = 0; r < 4 * C; ++r) x = (r == idx) ? v[r] : x;
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), (col & 255) >> 2));
}

// (k_gj_blocked -- one row's multipliers at a time -- and k_gj_blocked2 -- the
// multipliers lane-parallel, every column -- were the forms before
// k_gj_blocked3; measured slower and removed in round 6: docs/DESIGN_HISTORY.md
// section 4b / 4d, profiles/r05/gj_timing_*.json)

// k_gj_blocked3's row update: rows j_i = g + r + i (i < RR) take the panel's
// steps on their own columns (left [llo, n) and the diagonal, right [n, rhi):
// see the kernel's header), each pivot row's LDS read shared by the RR rows;
// SKIP: a row leaves out its own step (the panel's pivot rows).  Each element
// is m -= q * t as the reference (:301): a packed multiply, then a packed add
// of the negated product, each half rounded as the scalar operation.
template <int C, int NB, int RR, bool SKIP>
__device__ __forceinline__ void gj3_rows(float* __restrict__ aug, float* __restrict__ res, const int* perm,
                                         const float* P, int* full, const float (&t)[NB],
                                         unsigned long long badmask, bool fullp, bool last, int n, int p0, int ns,
                                         int rwin, int g, int r, int lane) {
    constexpr int W = 256 * C;
    bool on[RR][C];
    float v[RR][4 * C];
#pragma unroll
    for (int i = 0; i < RR; ++i) {
        const int j = g + r + i;
        const bool rowfull = fullp || ((badmask >> (r + i)) & 1ull);
        if (rowfull && !fullp && lane == 0) *full = 1;  // every column from the next panel on
        const int llo = j >= p0 ? 0 : p0;
        const int rhi = n + (rowfull ? n : rwin);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int a = 256 * c + 4 * lane, b0 = 256 * c;
            const bool blk = (b0 + 256 > llo && b0 < n) || (b0 <= j && j < b0 + 256) || (b0 + 256 > n && b0 < rhi);
            on[i][c] = blk && ((a + 4 > llo && a < n) || (a <= j && j < a + 4) || (a + 4 > n && a < rhi));
            sf4 q = sf4{0, 0, 0, 0};
            if (on[i][c]) q = *reinterpret_cast<const sf4*>(aug + (size_t)j * W + 256 * c + 4 * lane);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[i][4 * c + e] = q[e];
        }
    }
#pragma unroll
    for (int s = 0; s < NB; ++s) {
        if (s < ns) {
            const float* prow = P + (size_t)s * W;
            sf4 q[C];
#pragma unroll
            for (int c = 0; c < C; ++c) q[c] = *reinterpret_cast<const sf4*>(prow + 256 * c + 4 * lane);
#pragma unroll
            for (int i = 0; i < RR; ++i) {
                if (SKIP && p0 + s == g + r + i) continue;
                const float ts = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t[s]), r + i));
                const sf2 tt = sf2{ts, ts};
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    sf2 lo = sf2{v[i][4 * c], v[i][4 * c + 1]}, hi = sf2{v[i][4 * c + 2], v[i][4 * c + 3]};
                    lo = lo - sf2{q[c].x, q[c].y} * tt;  // (:301)
                    hi = hi - sf2{q[c].z, q[c].w} * tt;
                    v[i][4 * c] = lo.x;
                    v[i][4 * c + 1] = lo.y;
                    v[i][4 * c + 2] = hi.x;
                    v[i][4 * c + 3] = hi.y;
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < RR; ++i) {
        const int j = g + r + i;
        if (!last) {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if (!on[i][c]) continue;
                sf4 q;
#pragma unroll
                for (int e = 0; e < 4; ++e) q[e] = v[i][4 * c + e];
                *reinterpret_cast<sf4*>(aug + (size_t)j * W + 256 * c + 4 * lane) = q;
            }
        } else {  // temp = m_jj; the row / temp; right column n + q is res's column perm[q]
            const float d = gj_any_col<C>(v[i], j);
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = 256 * c + 4 * lane + e;
                    if (k >= n && k < 2 * n) res[(size_t)j * n + perm[k - n]] = v[i][4 * c + e] / d;
                }
        }
    }
}

// k_gj_blocked3: k_gj_blocked2's panels and per-element operations on only
// the columns that can still change an output.  Two facts of the reference's
// loops (PQP_CPU.c:291-305), both exact:
//  * The right half is kept in the bubble pass's row order (row r's 1 at
//    column n + r; each column's operations are independent of the others, so
//    a column permutation changes no value) and res is written through the
//    permutation.  Right column n + q holds +0 in every row but row q until
//    pivot q, and while every multiplier is finite, m_jq -= (+-0) * t leaves
//    +0 and 1 as they are -- so a panel of pivots [p0, p0 + NB) touches right
//    columns [n, n + p0 + NB) only.  A non-finite multiplier (an inf or NaN t
//    turns 0 * t into NaN, as in the reference) makes its row take every
//    column, and every row from the next panel on (a sticky flag); the pivot
//    rows always take every column.
//  * Left column c of row j is read again only while row j is still to be a
//    pivot (j >= p0: its column c feeds the diagonal m_cc through step j) or
//    as row j's own diagonal (the final scaling, :307-314).  So a row j < p0
//    touches left columns [p0, n) and its diagonal only.
// Per row and panel about (n + p0 + NB) - (j < p0 ? p0 : 0) of the 2n
// columns: the loads and stores are masked per lane chunk (4 columns) and
// skipped per 256-column block; the arithmetic runs on every block.
template <int C, int NB>
__global__ void __launch_bounds__(256) k_gj_blocked3(const float* __restrict__ A, float* __restrict__ aug,
                                                     float* __restrict__ res, int n) {
    constexpr int W = 256 * C;  // padded row of the augmented matrix
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* P = lds;                                                // [NB][W] pivot rows at their step
    float* Pd = lds + NB * W;                                      // [NB] their diagonals
    int* perm = reinterpret_cast<int*>(lds + NB * W + NB);         // [n] the bubble pass's row order
    int* full = perm + n;                                          // sticky: every column from now on
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    {
        const size_t b = blockIdx.x;
        A += b * n * n;
        res += b * n * n;
        aug += b * (size_t)n * W;
    }
    // the one bubble pass on column 0 (:280-289) as a row order, then [A | I]
    // with I in that order (:262-276), zero-padded to W columns
    float* col0 = P;
    for (int r = tid; r < n; r += 256) col0[r] = A[(size_t)r * n];
    __syncthreads();
    if (tid == 0) {
        for (int r = 0; r < n; ++r) perm[r] = r;
        for (int r = n - 1; r > 0; --r)
            if (col0[perm[r - 1]] < col0[perm[r]]) {
                const int t = perm[r];
                perm[r] = perm[r - 1];
                perm[r - 1] = t;
            }
        *full = 0;
    }
    __syncthreads();
    for (int r = wv; r < n; r += 4) {
        const int src = perm[r];
        float v[4 * C];
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = 256 * c + 4 * lane + e;
                v[4 * c + e] = k < n ? A[(size_t)src * n + k] : (k == n + r ? 1.0f : 0.0f);
            }
        gj_store<C>(aug + (size_t)r * W, lane, v);
    }
    __syncthreads();
    for (int p0 = 0; p0 < n; p0 += NB) {
        const int ns = n - p0 < NB ? n - p0 : NB;
        const int rwin = p0 + NB < n ? p0 + NB : n;  // right columns [n, n + rwin) can be nonzero
        if (wv == 0) {  // 1. the pivot rows at their step, every column
            // (the next pivot row's load in flight while this one takes its steps)
            float vn[4 * C];
            gj_load<C>(aug + (size_t)p0 * W, lane, vn);
            for (int s = 0; s < ns; ++s) {
                float v[4 * C];
#pragma unroll
                for (int e = 0; e < 4 * C; ++e) v[e] = vn[e];
                if (s + 1 < ns) gj_load<C>(aug + (size_t)(p0 + s + 1) * W, lane, vn);
                gj_steps_any<C, NB>(v, P, Pd, W, p0, s, -1, lane);
                gj_store<C>(P + (size_t)s * W, lane, v);
                const float d = gj_any_col<C>(v, p0 + s);
                if (lane == 0) Pd[s] = d;
            }
            // the pivot rows' right columns past the window are +-0 unless a
            // non-finite multiplier of theirs made them NaN: then every row
            // takes every column from this panel on
            bool dirty = false;
            for (int s = 0; s < ns; ++s)
                for (int k = n + rwin + lane; k < 2 * n; k += 64) dirty |= P[(size_t)s * W + k] != 0.0f;
            if (__any(dirty) && lane == 0) *full = 1;
        }
        __syncthreads();
        const bool fullp = *full != 0;
        const bool last = p0 + NB >= n;
        for (int g = 64 * wv; g < n; g += 256) {
            // 2a. row g + lane's multipliers of the panel's steps (k_gj_blocked2)
            const int jl = g + lane;
            float t[NB];
            bool tbad = false;  // a multiplier this row uses is inf or NaN
            {
                float m[NB];
#pragma unroll
                for (int q = 0; q < NB; q += 4) {
                    const sf4 x = jl < n ? *reinterpret_cast<const sf4*>(aug + (size_t)jl * W + p0 + q) : sf4{0, 0, 0, 0};
                    m[q] = x.x;
                    m[q + 1] = x.y;
                    m[q + 2] = x.z;
                    m[q + 3] = x.w;
                }
#pragma unroll
                for (int s = 0; s < NB; ++s) {
                    float x = m[s];
#pragma unroll
                    for (int s2 = 0; s2 < s; ++s2)
                        if (p0 + s2 != jl) x -= P[(size_t)s2 * W + p0 + s] * t[s2];  // (:301) on column p0 + s
                    t[s] = x / Pd[s];  // temp (:298)
                    if (s < ns && p0 + s != jl) tbad |= !__builtin_isfinite(t[s]);
                }
            }
            const unsigned long long badmask = __ballot(tbad);
            // 2b. each row of the group takes the panel's steps on its columns:
            // R rows at a time share each LDS read of a pivot row (the LDS
            // reads, one pivot row per row and step, bounded k_gj_blocked2);
            // the rows of this panel's own pivots one at a time (their own
            // step is skipped)
            constexpr int R = C <= 4 ? 4 : 2;
            const int rend = n - g < 64 ? n - g : 64;
            int r = 0;
            for (; r + R <= rend; r += R) {
                if (g + r < p0 + ns && g + r + R > p0) {
#pragma unroll
                    for (int i = 0; i < R; ++i)
                        gj3_rows<C, NB, 1, true>(aug, res, perm, P, full, t, badmask, fullp, last, n, p0, ns, rwin, g,
                                                 r + i, lane);
                } else {
                    gj3_rows<C, NB, R, false>(aug, res, perm, P, full, t, badmask, fullp, last, n, p0, ns, rwin, g, r,
                                              lane);
                }
            }
            for (; r < rend; ++r)
                gj3_rows<C, NB, 1, true>(aug, res, perm, P, full, t, badmask, fullp, last, n, p0, ns, rwin, g, r, lane);
        }
        __syncthreads();
    }
}

// padded row width and panel of the blocked kernel for an n x n matrix (0: not handled)
static int gj_blocked_c(int n) { return n >= 1 && n <= 1024 ? (2 * n + 255) / 256 : 0; }
size_t gauss_jordan_aug_floats(int n) {
    const int c = gj_blocked_c(n);
    return c ? (size_t)n * 256 * c : (size_t)2 * n * n;
}
template <int C>
static void launch_gj_blocked_c(int B, const float* A, float* aug, float* res, int n, hipStream_t s) {
    constexpr int NB = C <= 4 ? 16 : 8;
    const size_t lds = sizeof(float) * ((size_t)NB * 256 * C + NB);
    // k_gj_blocked3: 4096 n = 512 inverses in 0.097 s (k_gj_blocked 0.127, its
    // lane-parallel-multiplier form 0.114: profiles/r05/gj_timing_*.json)
    hipLaunchKernelGGL((k_gj_blocked3<C, NB>), dim3(B), dim3(256), lds + sizeof(int) * ((size_t)n + 1), s, A, aug,
                       res, n);
}
static hipError_t launch_gj_blocked(int B, const float* A, float* aug, float* res, int n, hipStream_t s) {
    switch (gj_blocked_c(n)) {
        case 1: launch_gj_blocked_c<1>(B, A, aug, res, n, s); break;
        case 2: launch_gj_blocked_c<2>(B, A, aug, res, n, s); break;
        case 3: launch_gj_blocked_c<3>(B, A, aug, res, n, s); break;
        case 4: launch_gj_blocked_c<4>(B, A, aug, res, n, s); break;
        case 5: launch_gj_blocked_c<5>(B, A, aug, res, n, s); break;
        case 6: launch_gj_blocked_c<6>(B, A, aug, res, n, s); break;
        case 7: launch_gj_blocked_c<7>(B, A, aug, res, n, s); break;
        case 8: launch_gj_blocked_c<8>(B, A, aug, res, n, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_gauss_jordan_b(int B, const float* A, float* aug, float* fac, float* res, int n, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (n >= kGaussJordanWideMin && B <= 8) {  // few large matrices: each over many workgroups
        for (int b = 0; b < B; ++b) {
            const hipError_t e = launch_gauss_jordan_wide(A + (size_t)b * n * n, aug + (size_t)b * 2 * n * n,
                                                          reinterpret_cast<int*>(fac + (size_t)b * n),
                                                          res + (size_t)b * n * n, n, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    if (!g_tune.gj_blocked_off && gj_blocked_c(n)) return launch_gj_blocked(B, A, aug, res, n, s);
    hipLaunchKernelGGL(k_gauss_jordan, dim3(B), dim3(256), 0, s, A, aug, fac, res, n);
    return hipGetLastError();
}
hipError_t launch_axpy(float* A, const float* B, float sign, int n, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_axpy, dim3(cdiv(n, 256)), dim3(256), 0, s, A, B, sign, n);
    return hipGetLastError();
}
hipError_t launch_negate(float* A, int n, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_negate, dim3(cdiv(n, 256)), dim3(256), 0, s, A, n);
    return hipGetLastError();
}
hipError_t launch_compare(const float* gu, const float* Kp, int n, int* flag, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_compare, dim3(cdiv(n, 256)), dim3(256), 0, s, gu, Kp, n, flag);
    return hipGetLastError();
}
hipError_t launch_theta_rowmajor(const float* Qd, int N, float* theta_mat, hipStream_t s) {
    if (N > 0) hipLaunchKernelGGL(k_theta_rowmajor, dim3(cdiv(N, 256)), dim3(256), 0, s, Qd, N, theta_mat);
    return hipGetLastError();
}
hipError_t launch_cost_finish(const float* quad, const float* lin, const float* Mc, float* J, hipStream_t s) {
    hipLaunchKernelGGL(k_cost_finish, dim3(1), dim3(1), 0, s, quad, lin, Mc, J);
    return hipGetLastError();
}
hipError_t launch_mp_finish(const float* t, const float* Mp6, float* Mp, hipStream_t s) {
    hipLaunchKernelGGL(k_mp_finish, dim3(1), dim3(1), 0, s, t, Mp6, Mp);
    return hipGetLastError();
}
hipError_t launch_gauss_jordan(const float* A, float* aug, float* fac, float* res, int n, hipStream_t s) {
    return launch_gauss_jordan_b(1, A, aug, fac, res, n, s);
}

size_t solve_single_lds_bytes(int ldq, int ldm, bool fused) {
    return sizeof(float) * ((size_t)(fused ? 4 : 3) * ldq + (size_t)3 * ldm);
}

thread_local int g_last_batch_kernel = 0;
size_t solve_pipe_lds_bytes(int ldq, int ldm, bool big) {
    const size_t cost = (size_t)ldq + 2 * (size_t)ldm, tile = pipe_tile_floats(big);
    return sizeof(float) * ((size_t)3 * ldq + (size_t)3 * ldm + (tile > cost ? tile : cost));
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }
// Path 2's converge-mode kernel by shape alone (given Qp_inv' and 16-byte
// aligned arrays): k_solve_pipe reads Gp once per iteration but holds two
// workgroups per CU against k_solve_single's three, so it pays only where Gp
// is a large part of the bytes (M >= N / 3; the MPC plant over 6..32 horizon
// steps, M = N / 4, measured faster on k_solve_single:
// profiles/r03/pipe/horizon_pipe_vs_single.jsonl).  `variant`: the pipe build
// (g_tune.pipe_variant read once by the caller, so the LDS size and the kernel
// launched agree).
bool pipe_route(int N, int M, int variant) {
    const auto round4 = [](int n) { return (n + 3) & ~3; };
    const bool big = variant != 3;  // the default build's 128 x 96 tile (3: two 64 x 64 tiles in flight)
    return !g_tune.single_scalar && !g_tune.pipe_off && (g_tune.pipe_force || 3 * M >= N) && N > 64 && N % 4 == 0 &&
           M % 4 == 0 && solve_pipe_lds_bytes(round4(N), round4(M), big) <= kPipeLdsMax;
}
// CU count of the current device, queried once per device (the
// occupancy choice below ran the attribute query on every launch)
static int current_device_cus() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
    if (dev < 64) {
        const int c = cache[dev].load(std::memory_order_relaxed);
        if (c > 0) return c;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 0;
    if (dev < 64) cache[dev].store(cus, std::memory_order_relaxed);
    return cus;
}
static hipError_t launch_single_grid(int B, const SolveArgs& a, SolveState* st, hipStream_t s) {
    const size_t lds = solve_single_lds_bytes(a.ldq, a.ldm, a.sym != nullptr);
    // wide loads need every row and column start 16-byte aligned: N, M
    // multiples of 4 and 16-byte-aligned arrays (null ones are not read)
    const bool vec = !g_tune.single_scalar && a.N % 4 == 0 && a.M % 4 == 0 && aligned16(a.QdT) && aligned16(a.Qd) &&
                     aligned16(a.Gp) && aligned16(a.Qinv) && aligned16(a.Qp) && aligned16(a.GpT) &&
                     aligned16(a.QinvT) && (a.ldq & 3) == 0 && (a.ldm & 3) == 0;
    // converge mode with Qp_inv': one pass over Gp per iteration (k_solve_pipe)
    const int variant = g_tune.pipe_variant;
    if (vec && a.mode == kModeConverge && a.QinvT && pipe_route(a.N, a.M, variant)) {
        const bool big = variant != 3;
        const size_t plds = solve_pipe_lds_bytes(a.ldq, a.ldm, big);
        if (big) hipLaunchKernelGGL((k_solve_pipe<256, 2, 16, 2, true>), dim3(B), dim3(256), plds, s, a, st);
        else hipLaunchKernelGGL((k_solve_pipe<256, 2, 16, 2>), dim3(B), dim3(256), plds, s, a, st);
        g_last_batch_kernel = 1;
        return hipGetLastError();
    }
    g_last_batch_kernel = 0;
    if (a.N <= 64) {
        if (vec) hipLaunchKernelGGL((k_solve_single<64, true>), dim3(B), dim3(64), lds, s, a, st);
        else hipLaunchKernelGGL((k_solve_single<64, false>), dim3(B), dim3(64), lds, s, a, st);
    } else {
        // workgroups per CU by the register cap (3, 4 or 5).  Up to n_dual 768
        // the passes are latency-bound: more problems in flight pay, but each
        // step up costs 5-13 % per round of resident problems, so the choice
        // minimises rounds x (1 + 0.1 (occ - 3)) -- the MPC plant over 8 / 12 /
        // 16 / 24 horizon stages measured best at 5 / 5 / 4 / 5, as predicted
        // (profiles/r04/single_occ_ab*.jsonl); n_dual 896 and 1024 the same at
        // 3, 4 and 5.  single_occ 3 / 4 / 5 forces one.
        int occ = g_tune.single_occ;
        if (!occ) {
            occ = 3;
            const int cus = a.N <= 768 ? current_device_cus() : 0;
            if (cus > 0) {
                double best = 1e300;
                for (int o = 3; o <= 5; ++o) {
                    const double cost = (double)((B + (long long)cus * o - 1) / ((long long)cus * o)) * (1.0 + 0.1 * (o - 3));
                    if (cost < best - 1e-9) {
                        best = cost;
                        occ = o;
                    }
                }
            }
        }
        if (vec && occ == 5) hipLaunchKernelGGL((k_solve_single<256, true, 5>), dim3(B), dim3(256), lds, s, a, st);
        else if (vec && occ == 4) hipLaunchKernelGGL((k_solve_single<256, true, 4>), dim3(B), dim3(256), lds, s, a, st);
        else if (vec) hipLaunchKernelGGL((k_solve_single<256, true>), dim3(B), dim3(256), lds, s, a, st);
        else hipLaunchKernelGGL((k_solve_single<256, false>), dim3(B), dim3(256), lds, s, a, st);
    }
    return hipGetLastError();
}
hipError_t launch_solve_single(const SolveArgs& a, SolveState* st, hipStream_t s) {
    return launch_single_grid(1, a, st, s);
}

// path: 0 tiny (N, M <= 32), 1 LDS-staged small, 2 global-memory single,
// 3 LDS-resident mid-size
hipError_t launch_solve_batch(int B, int path, const SolveArgs& a, SolveState* st, hipStream_t s) {
    if (path == 0) return launch_tiny_grid(B, a, st, s);
    if (path == 1) return launch_small_grid(B, a, st, s);
    if (path == 3) return launch_mid_grid(B, a, st, s);
    return launch_single_grid(B, a, st, s);
}

// dst[b] (cols x rows, row-major) = transpose of src[b] (rows x cols), per problem
__global__ void __launch_bounds__(256) k_transpose_b(const float* __restrict__ src, int rows, int cols,
                                                     float* __restrict__ dst) {
    __shared__ float tile[32][33];
    const size_t b = blockIdx.z, n = (size_t)rows * cols;
    src += b * n;
    dst += b * n;
    const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int r = ty; r < 32; r += 8) {
        const int rr = r0 + r, cc = c0 + tx;
        tile[r][tx] = (rr < rows && cc < cols) ? src[(size_t)rr * cols + cc] : 0.0f;
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int cc = c0 + r, rr = r0 + tx;
        if (cc < cols && rr < rows) dst[(size_t)cc * rows + rr] = tile[tx][r];
    }
}
hipError_t launch_transpose_b(int B, const float* src, int rows, int cols, float* dst, hipStream_t s) {
    if (B <= 0 || rows <= 0 || cols <= 0) return hipSuccess;
    for (int b0 = 0; b0 < B; b0 += 65535) {
        const int nb = (B - b0) < 65535 ? (B - b0) : 65535;
        hipLaunchKernelGGL(k_transpose_b, dim3(cdiv(cols, 32), cdiv(rows, 32), nb), dim3(256), 0, s,
                           src + (size_t)b0 * rows * cols, rows, cols, dst + (size_t)b0 * rows * cols);
    }
    return hipGetLastError();
}

// sym[b] = 1 iff problem b's row-major Qd (N x N, stride N*N) equals its
// transpose bit for bit (preset to 1; 32 x 32 tiles through LDS).
__global__ void __launch_bounds__(256) k_check_symmetric(const float* __restrict__ Qd, int N, int* __restrict__ sym) {
    __shared__ unsigned tile[32][33];
    const int b = blockIdx.z;
    const int bi = blockIdx.y, bj = blockIdx.x;
    if (bj < bi) return;  // each pair of tiles once
    const unsigned* q = reinterpret_cast<const unsigned*>(Qd) + (size_t)b * N * N;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int r = ty; r < 32; r += 8) {  // tile (bj, bi) transposed into LDS
        const int i = bj * 32 + r, j = bi * 32 + tx;
        tile[tx][r] = (i < N && j < N) ? q[(size_t)i * N + j] : 0u;
    }
    __syncthreads();
    int bad = 0;
    for (int r = ty; r < 32; r += 8) {
        const int i = bi * 32 + r, j = bj * 32 + tx;
        if (i < N && j < N && q[(size_t)i * N + j] != tile[r][tx]) bad = 1;
    }
    if (__syncthreads_or(bad) && threadIdx.x == 0) atomicAnd(sym + b, 0);
}
// The same for N % 4 == 0 and a 16-byte-aligned Qd: one workgroup per (problem,
// 64-row band bi) walks the tile pairs (bi, bj >= bi) with 16-byte loads, so
// the grid is B x N/64 workgroups instead of B x (N/32)^2 (most of which had
// nothing to do).
__global__ void __launch_bounds__(256) k_check_symmetric4(const float* __restrict__ Qd, int N, int* __restrict__ sym) {
    __shared__ unsigned tile[64][65];
    const int b = blockIdx.y, bi = blockIdx.x;
    const unsigned* q = reinterpret_cast<const unsigned*>(Qd) + (size_t)b * N * N;
    const int nt = (N + 63) / 64;
    const int tc = (threadIdx.x & 15) * 4, tr = threadIdx.x >> 4;  // 16 rows x 4 columns per pass
    int bad = 0;
    for (int bj = bi; bj < nt; ++bj) {
#pragma unroll
        for (int pss = 0; pss < 4; ++pss) {  // tile (bj, bi), transposed into LDS
            const int r = tr + 16 * pss, i = bj * 64 + r, j = bi * 64 + tc;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (i < N && j < N) v = *reinterpret_cast<const uint4*>(q + (size_t)i * N + j);
            tile[tc + 0][r] = v.x;
            tile[tc + 1][r] = v.y;
            tile[tc + 2][r] = v.z;
            tile[tc + 3][r] = v.w;
        }
        __syncthreads();
#pragma unroll
        for (int pss = 0; pss < 4; ++pss) {  // against tile (bi, bj)
            const int r = tr + 16 * pss, i = bi * 64 + r, j = bj * 64 + tc;
            if (i < N && j < N) {
                const uint4 v = *reinterpret_cast<const uint4*>(q + (size_t)i * N + j);
                bad |= (v.x != tile[r][tc + 0]) | (v.y != tile[r][tc + 1]) | (v.z != tile[r][tc + 2]) |
                       (v.w != tile[r][tc + 3]);
            }
        }
        __syncthreads();
    }
    if (__syncthreads_or(bad) && threadIdx.x == 0) atomicAnd(sym + b, 0);
}
hipError_t launch_check_symmetric(int B, const float* Qd, int N, int* sym, hipStream_t s) {
    if (B <= 0 || N <= 0) return hipSuccess;
    const bool wide = N % 4 == 0 && ((uintptr_t)Qd & 15) == 0;
    hipError_t e = hipSuccess;
    for (int b0 = 0; b0 < B && e == hipSuccess; b0 += 65535) {
        const int nb = (B - b0) < 65535 ? (B - b0) : 65535;
        e = hipMemsetAsync(sym + b0, 0x01, sizeof(int) * nb, s);  // bytes 0x01: nonzero = symmetric
        if (e != hipSuccess) break;
        if (wide)
            hipLaunchKernelGGL(k_check_symmetric4, dim3(cdiv(N, 64), nb), dim3(256), 0, s, Qd + (size_t)b0 * N * N, N,
                               sym + b0);
        else
            hipLaunchKernelGGL(k_check_symmetric, dim3(cdiv(N, 32), cdiv(N, 32), nb), dim3(256), 0, s,
                               Qd + (size_t)b0 * N * N, N, sym + b0);
        e = hipGetLastError();
    }
    return e;
}

__global__ void k_extract_state(int B, const SolveState* __restrict__ st, long long* __restrict__ h,
                                int* __restrict__ status) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    if (h) h[b] = st[b].h;
    if (status) status[b] = st[b].status;
}
// every problem at the reference's start: h = 1, nothing decided (SolveState{})
__global__ void k_init_state(int B, SolveState* __restrict__ st) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    SolveState z{};
    z.h = 1;
    st[b] = z;
}
hipError_t launch_state_init(int B, SolveState* st, hipStream_t s) {
    hipLaunchKernelGGL(k_init_state, dim3(cdiv(B, 256)), dim3(256), 0, s, B, st);
    return hipGetLastError();
}
hipError_t launch_extract_state(int B, const SolveState* st, long long* h, int* status, hipStream_t s) {
    hipLaunchKernelGGL(k_extract_state, dim3(cdiv(B, 256)), dim3(256), 0, s, B, st, h, status);
    return hipGetLastError();
}

}  // namespace pqp
