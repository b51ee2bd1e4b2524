// pqp_wide.hip -- converge mode of ONE large problem spread over many
// workgroups (solveQuadraticDual, PQP_CPU.c:694-750).
//
// The one-workgroup solver (k_solve_single) moves every byte of Qd, Gp and
// Qp_inv through a single CU each iteration, so it runs at one CU's fetch
// rate.  Here one iteration is a short chain of launches, replayed from a
// hipGraph:
//
//   K1  tmp = Gp'Y + Fp          and   (Y'Qd)            [two jobs, one launch]
//   K2  U = -(Qp_inv tmp)
//   K3  Gp U vs Kp (feasibility) and   (U'Qp)            [two jobs]
//   K4  costs Jp, Jd, the gap tests, the cap; h += 1 if the update follows
//   K5  updateY2 (k_split_relay)
//
// Every launch first reads the solve's status word and returns at once when
// the solve has finished, so a graph of C iterations can be replayed until
// the status says Done/Capped.  Each product of K1-K3 is a column-access
// mat-vec out[j] = sum_k A[k][j] x[k] with k in order from +0.0f on one lane
// per output (the reference's matrixMultiply order), spread over W waves as
// in k_split_relay: wave g % W owns the k-segment g, multiplies it by x ahead
// of time, and adds it to the running sums handed over through LDS.
#include "pqp_device.h"
#include "pqp_launch.h"

#pragma clang fp contract(off)

namespace pqp {

namespace {

inline int cdivw(long long a, long long b) { return (int)((a + b - 1) / b); }

// dst (cols x rows, row-major) = transpose of src (rows x cols, row-major)
__global__ void __launch_bounds__(256) k_transpose(const float* __restrict__ src, int rows, int cols,
                                                   float* __restrict__ dst) {
    __shared__ float tile[32][33];
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

// K4: the rest of terminate() (PQP_CPU.c:673-687) and the loop control.
// The four dot products of computeCost (:648-666) -- (Y'Qd).Y, Fd.Y,
// (U'Qp).U, Fp.U -- are sums in k order on one lane each (waves 0-3); their
// products are formed by all 256 threads into LDS a chunk at a time, so the
// summing lanes read LDS instead of waiting on one global load per term
// (one lane walking Fd from global memory took ~200 us at n_dual = 1500).
// Folding this launch into the last workgroup of K3 behind an agent-scope
// fence and a counter measured 1-5 us slower per iteration.
constexpr int kDecideChunk = 1024;
__global__ void __launch_bounds__(256) k_wide_decide(WideArgs a) {
    SolveState* st = a.st;
    if (st->status != kStatusContinue) return;
    __shared__ __attribute__((aligned(16))) float prod[4][kDecideChunk];
    __shared__ float sJ[4];
    const int tid = threadIdx.x, wave = tid >> 6;
    const int feasible = *a.flag;  // checkFeas :677
    int stop = 0;
    if (feasible) {
        // wave w sums dot w: 0 quad_dual, 1 lin_dual, 2 quad_primal, 3 lin_primal
        const float* rowv[4] = {a.tq, a.Fd, a.tu, a.Fp};
        const float* zv[4] = {a.Y, a.Y, a.U, a.U};
        const int nv[4] = {a.N, a.N, a.M, a.M};
        float acc = 0.0f;
        const int nmax = a.N > a.M ? a.N : a.M;
        for (int c0 = 0; c0 < nmax; c0 += kDecideChunk) {
            for (int e = tid; e < 4 * kDecideChunk; e += 256) {
                const int d = e / kDecideChunk, k = c0 + e % kDecideChunk;
                prod[d][e % kDecideChunk] = (k < nv[d]) ? rowv[d][k] * zv[d][k] : 0.0f;
            }
            __syncthreads();
            if ((tid & 63) == 0) {
                const int n = (nv[wave] - c0) < kDecideChunk ? (nv[wave] - c0) : kDecideChunk;
                for (int k = 0; k < n; ++k) acc += prod[wave][k];  // :652-657, k in order
            }
            __syncthreads();
        }
        if ((tid & 63) == 0) sJ[wave] = acc;
        __syncthreads();
        float Jd = 0.0f, Jp = 0.0f;
        Jd = (float)((double)Jd + 0.5 * (double)sJ[0]);
        Jd += sJ[1];
        Jd += a.Md[0] / 2;
        Jp = (float)((double)Jp + 0.5 * (double)sJ[2]);
        Jp += sJ[3];
        Jp += a.Mp[0] / 2;
        stop = gap_stop(Jp, Jd) ? 1 : 0;  // the three gap tests :681-685
        if (tid == 0) {
            st->Jp = Jp;
            st->Jd = Jd;
            st->have_costs = 1;
        }
    }
    if (tid == 0) {
        if (stop)
            st->status = kStatusDone;
        else if (*a.max_updates > 0 && st->h - 1 >= *a.max_updates)
            st->status = kStatusCapped;
        else
            st->h += 1;  // the updateY2 that follows (:718-720)
        *a.flag = 1;     // re-armed for the next checkFeas
    }
}

template <int W, int S>
__global__ void __launch_bounds__(64 * W) k_gemv_relay(GemvJobs J) {
    if (J.gate && *J.gate != kStatusContinue) return;  // the solve has finished
    // LDS: [64] hand-off words, then x (zero-padded to whole segments)
    extern __shared__ __attribute__((aligned(16))) float lds[];
    unsigned long long* slot = reinterpret_cast<unsigned long long*>(lds);
    float* xs = lds + 128;
    const bool second = (int)blockIdx.x >= J.wgs0;
    const GemvJob jb = second ? J.job[1] : J.job[0];
    const int wg = second ? (int)blockIdx.x - J.wgs0 : (int)blockIdx.x;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = wg * 64 + lane;
    const bool live = j < jb.n_out;
    const int jc = live ? j : jb.n_out - 1;  // idle lanes re-read a valid column
    const int n_in = jb.n_in;
    const int G = (n_in + S - 1) / S;
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef float f2v __attribute__((ext_vector_type(2)));
    float q[S];
    auto load_seg = [&](int g) {
        const int nk = n_in - g * S;  // wave-uniform; k >= n_in is +0 and not loaded
        const float* col = jb.A + (size_t)g * S * jb.lda + jc;
#pragma unroll
        for (int t = 0; t < S; ++t) q[t] = (t < nk) ? col[(size_t)t * jb.lda] : 0.0f;
    };
    if (w < G) load_seg(w);  // independent of x: in flight while x is staged
    {
        const int t = threadIdx.x, n_lds = G * S;
        for (int b = 0; b < n_lds; b += 64 * W * 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = b + 64 * W * u + t;
                v[u] = (k < n_in) ? jb.x[k] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = b + 64 * W * u + t;
                if (k < n_lds) xs[k] = v[u];
            }
        }
        if (w == 0) slot[lane] = 0ull;  // segment 0 starts from +0.0f
    }
    __syncthreads();
    float acc = 0.0f;
    bool stale = false;
    for (int g = w; g < G; g += W) {
#pragma unroll
        for (int t0 = 0; t0 < S; t0 += 16) {  // x read 16 values at a time so the LDS reads overlap
            f4v xv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) xv[u] = *reinterpret_cast<const f4v*>(xs + g * S + t0 + 4 * u);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = t0 + 4 * u;
                const f2v lo = f2v{q[t], q[t + 1]} * f2v{xv[u].x, xv[u].y};
                const f2v hi = f2v{q[t + 2], q[t + 3]} * f2v{xv[u].z, xv[u].w};
                q[t] = lo.x;
                q[t + 1] = lo.y;
                q[t + 2] = hi.x;
                q[t + 3] = hi.y;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = t0 + 4 * u;
                asm volatile("" : "+v"(q[t]), "+v"(q[t + 1]), "+v"(q[t + 2]), "+v"(q[t + 3]));
            }
        }
        const unsigned long long h = relay_wait(slot, lane, g, J.spin_max, stale);
        __builtin_amdgcn_s_setprio(3);
        acc = __uint_as_float((unsigned)h);
#pragma unroll
        for (int t = 0; t < S; ++t) acc += q[t];  // matrixMultiply :88-100, k in order
        __hip_atomic_store(slot + lane, ((unsigned long long)(g + 1) << 32) | __float_as_uint(acc), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_s_setprio(0);
        if (g + W < G) load_seg(g + W);
    }
    if (w == (G - 1) % W && live) {
        switch (jb.epi) {
            case kEpiAdd: jb.out[j] = acc + 1.0f * jb.add[j]; break;  // matrixAdd(tmp, Fp, 1) :356
            case kEpiNeg: jb.out[j] = -acc; break;                    // U = -U :358
            case kEpiFeas: {                                          // compare :334-343
                const float kp = jb.add[j];
                if (acc > kp + max_ref((float)(kTol * kp), (float)kTol)) atomicAnd(J.flag, 0);
                jb.out[j] = acc;
                break;
            }
            default: jb.out[j] = acc;
        }
    }
    relay_report(stale, J.err, lane);
}

// ---------------------------------------------------------------------------
// Gauss_Jordan (PQP_CPU.c:251-326) of one large matrix over many workgroups:
// one launch per pivot, one workgroup per row.  Each element still sees the
// reference's operations in the reference's order (the pivots in sequence,
// row j's factor read before row j changes), so the inverse is bit-identical.
// ---------------------------------------------------------------------------
// the one bubble pass on column 0 (:280-289) decides swaps from column-0
// values only: replay it on them to get the final row order
__global__ void k_gj_order(const float* __restrict__ A, int n, int* __restrict__ perm) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int r = 0; r < n; ++r) perm[r] = r;
    for (int r = n - 1; r > 0; --r) {
        if (A[(size_t)perm[r - 1] * n] < A[(size_t)perm[r] * n]) {
            const int t = perm[r];
            perm[r] = perm[r - 1];
            perm[r - 1] = t;
        }
    }
}
// [A | I] (:262-276) with the rows in that order
__global__ void __launch_bounds__(256) k_gj_fill(const float* __restrict__ A, int n, const int* __restrict__ perm,
                                                 float* __restrict__ aug) {
    const int r = blockIdx.x, src = perm[r], w = 2 * n;
    for (int c = threadIdx.x; c < w; c += 256)
        aug[(size_t)r * w + c] = (c < n) ? A[(size_t)src * n + c] : ((c == n + src) ? 1.0f : 0.0f);
}
// pivot p (:291-305): row r -= row p * (aug[r][p] / aug[p][p]) for r != p
__global__ void __launch_bounds__(256) k_gj_pivot(float* __restrict__ aug, int n, int p) {
    const int r = blockIdx.x, w = 2 * n;
    if (r == p) return;
    float* row = aug + (size_t)r * w;
    const float* prow = aug + (size_t)p * w;
    const float f = row[p] / prow[p];  // every thread reads row[p] before any thread writes it
    __syncthreads();
    for (int c = threadIdx.x; c < w; c += 256) row[c] -= prow[c] * f;
}
// the row scaling (:307-314) and the extraction of the right half (:316-322)
__global__ void __launch_bounds__(256) k_gj_finish(const float* __restrict__ aug, int n, float* __restrict__ res) {
    const int r = blockIdx.x, w = 2 * n;
    const float d = aug[(size_t)r * w + r];
    for (int c = threadIdx.x; c < n; c += 256) res[(size_t)r * n + c] = aug[(size_t)r * w + n + c] / d;
}

// start of a converge-mode solve: SolveState (h = 1, Continue), the
// feasibility flag, the update cap, and Y = 1000 (initMat, PQP_CPU.c:710)
__global__ void k_wide_init(SolveState* st, int* flag, long long* cap, long long max_updates, float* Y, int N) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) {
        SolveState z{};
        z.h = 1;
        z.status = kStatusContinue;
        *st = z;
        *flag = 1;
        *cap = max_updates;
    }
    for (int i = t; i < N; i += gridDim.x * blockDim.x) Y[i] = 1000.0f;
}

}  // namespace

hipError_t launch_wide_init(SolveState* st, int* flag, long long* cap, long long max_updates, float* Y, int N,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_wide_init, dim3(cdivw(N, 256) < 64 ? cdivw(N, 256) : 64), dim3(256), 0, s, st, flag, cap,
                       max_updates, Y, N);
    return hipGetLastError();
}

hipError_t launch_transpose(const float* src, int rows, int cols, float* dst, hipStream_t s) {
    if (rows <= 0 || cols <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_transpose, dim3(cdivw(cols, 32), cdivw(rows, 32)), dim3(256), 0, s, src, rows, cols, dst);
    return hipGetLastError();
}


template <int W, int S>
static hipError_t gemv_launch(GemvJobs J, int n_in, hipStream_t s) {
    const size_t lds = sizeof(float) * ((size_t)cdivw(n_in, S) * S + 128);
    const int wgs1 = J.job[1].A ? cdivw(J.job[1].n_out, 64) : 0;
    hipLaunchKernelGGL((k_gemv_relay<W, S>), dim3(J.wgs0 + wgs1), dim3(64 * W), lds, s, J);
    return hipGetLastError();
}

hipError_t launch_gemv_relay(const GemvJobs& jobs, hipStream_t s) {
    GemvJobs J = jobs;
    J.wgs0 = cdivw(J.job[0].n_out, 64);
    J.spin_max = g_tune.relay_spin_max;
    int n_in = J.job[0].n_in;
    if (J.job[1].A && J.job[1].n_in > n_in) n_in = J.job[1].n_in;
    return gemv_launch<8, 32>(J, n_in, s);
}


hipError_t launch_gauss_jordan_wide(const float* A, float* aug, int* perm, float* res, int n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gj_order, dim3(1), dim3(64), 0, s, A, n, perm);
    hipLaunchKernelGGL(k_gj_fill, dim3(n), dim3(256), 0, s, A, n, perm, aug);
    for (int p = 0; p < n; ++p) hipLaunchKernelGGL(k_gj_pivot, dim3(n), dim3(256), 0, s, aug, n, p);
    hipLaunchKernelGGL(k_gj_finish, dim3(n), dim3(256), 0, s, aug, n, res);
    return hipGetLastError();
}

hipError_t launch_wide_decide(const WideArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_wide_decide, dim3(1), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace pqp
