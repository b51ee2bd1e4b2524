// pqp_tiny.hip -- ONE small problem (N, M <= 32: the bundled example, configs[1])
// solved by one launch whose results go straight to pinned host memory.
//
//   k_solve_quintet  converge mode (solveQuadraticDual, PQP_CPU.c:694-750) on
//                 five waves of one workgroup, pipelined over iterates:
//                   wave A      updateY2 (:603-618): Y_{h+1} from Y_h, nothing else
//                   waves B0/B1 terminate()'s N-long sums of the even / odd
//                               iterates: Gp'Y + Fp (computeUfromY :354-355),
//                               (Y'Qd).Y and Fd.Y (computeCost :652-657, Jd)
//                   waves C0/C1 the M-side chain of the even / odd iterates:
//                               U = -Qp_inv t (:356-359), checkFeas (:632-641),
//                               U'Qp.U and Fp.U (Jp), the gap tests (:680-686);
//                               decisions are taken in iterate order
//                 updateY2 needs only Y_h, not terminate()'s verdict, so A runs
//                 ahead of the decision (at most kRing iterates) and B, C follow;
//                 iterates past the stopping one are discarded.  Vectors pass
//                 through LDS rings indexed by the iterate; each wave publishes
//                 its progress in one LDS word, a release store after its data
//                 (a consumer's load of the word is an acquire: LDS operations
//                 of one wave may complete out of order, and relaxed words lost
//                 a race on cold launches).  LDS is never read where this
//                 launch did not write it (padding of y and t is zeroed first:
//                 a NaN left by an earlier kernel made 0 * NaN a NaN U).  Every
//                 wait is bounded: an expired wait ends the launch with an error
//                 word instead of a hang.
//   k_fixed_one   fixed mode (while(h < NUM_ITER) updateY2, the testing/
//                 harness loop) on one wave.  Where every lane's split row
//                 (lane 2i + side: Qdn_theta / Qdp_theta row i) has at most P
//                 nonzero entries, the update sums only those, in k order, with
//                 y gathered by ds_bpermute: a skipped entry is +-0, and with
//                 every y_k finite +-0 * y_k is +-0, which added to a sum that
//                 starts at +0.0f (and so is never -0) changes nothing -- the
//                 result is the reference's bit for bit.  The first non-finite
//                 y moves the rest of the solve to the dense form, where every
//                 term is summed (so a NaN or inf propagates as in the
//                 reference).
//
// Both write Y, U and the SolveState to the device buffers (for a resumed
// launch) and, when SolveArgs::hout is set, to pinned host memory, so a solve
// is one launch and one stream synchronisation: no copy kernels.
#include "pqp_device.h"
#include "pqp_launch.h"

#pragma clang fp contract(off)

namespace pqp {
namespace {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float rdl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
// this row's y_i (lane 2i) on both lanes 2i, 2i + 1: DPP quad_perm [0,0,2,2]
__device__ __forceinline__ float own_y(float yk) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(yk), 0xA0, 0xF, 0xF, true));
}
// the partner lane's value (lane ^ 1): DPP quad_perm [1,0,3,2]
__device__ __forceinline__ float partner(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}
// Progress words between the waves of one workgroup (LDS): a consumer's load
// is an acquire and a producer's store a release at workgroup scope, so the
// data a word covers is written before it and read after it (the compiler may
// neither hoist a ring read above the wait nor sink a ring write below the
// publish); the value is made wave-uniform (readfirstlane) so every wait is a
// scalar branch, not an exec-mask loop.
__device__ __forceinline__ int lds_ld(const int* p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_after_wait() { __asm__ volatile("" ::: "memory"); }
__device__ __forceinline__ void lds_publish(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

constexpr int kRing = 8;             // iterates in flight between wave A and the decision
constexpr int kStopWord = 0x7fffffff;  // `decided` once wave C has ended the solve
constexpr int kSpinMax = 1 << 24;    // polls per wait (~0.5 s) before the launch gives up

// split row i of Qdn_theta (side 0) / Qdp_theta (side 1) incl. Theta
// (computeTheta :503-519, computeQdp/Qdn_theta :524-537) and Fdn / Fdp
// (:703-704), for lane 2i + side; zero on lanes >= 2N
template <int NMAX>
__device__ __forceinline__ void split_row(const SolveArgs& A, int lane, float (&mat)[NMAX], float& fd_own) {
    const int N = A.N, i = lane >> 1, side = lane & 1;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) mat[k] = 0.0f;
    fd_own = 0.0f;
    if (i < N) {
        float th = 0.0f;
        for (int k = 0; k < N; ++k) th += max_ref(0.0f, -A.Qd[i * N + k]) * 1.0f;
        th = max_ref(th, 5.0f);
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
            if (k < N) {
                const float q = A.Qd[i * N + k];
                const float t = (i == k) ? th : 0.0f;
                mat[k] = (side ? max_ref(0.0f, q) : max_ref(0.0f, -q)) + 1.0f * t;
            }
        }
        const float f = A.Fd[i];
        fd_own = side ? max_ref(0.0f, f) : max_ref(0.0f, -f);
    }
}

// one dense update on one wave: y_k on lane 2k, broadcast by v_readlane into
// packed products, the sum in k order, num (even lane) / den (odd lane)
template <int NMAX>
__device__ __forceinline__ float update_dense(const float (&mat)[NMAX], float fd_own, float yk, bool own_row) {
    const float yi = own_y(yk);
    float p[NMAX];
#pragma unroll
    for (int k = 0; k < NMAX; k += 2) {
        const f2v pr = f2v{mat[k], mat[k + 1]} * f2v{rdl(yk, 2 * k), rdl(yk, 2 * k + 2)};
        p[k] = pr.x;
        p[k + 1] = pr.y;
    }
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) acc += p[k];  // :608-609, k in order
    const float v = acc + 1.0f * fd_own;        // :611 / :612
    const float den = partner(v);
    const float yn = v / den * yi;              // :594
    return own_row ? yn : 0.0f;                 // lanes past 2N (and odd lanes) hold +0
}

// the same update summing only this lane's P nonzero entries (k order), y by
// ds_bpermute from lane 2k (byte address sa = 8k)
template <int P>
__device__ __forceinline__ float update_sparse(const float (&sc)[12], const int (&sa)[12], float fd_own, float yk,
                                               bool own_row) {
    const float yi = own_y(yk);
    float acc = 0.0f;
#pragma unroll
    for (int s = 0; s < P; ++s) acc += sc[s] * __int_as_float(__builtin_amdgcn_ds_bpermute(sa[s], __float_as_int(yk)));
    const float v = acc + 1.0f * fd_own;
    const float den = partner(v);
    const float yn = v / den * yi;
    return own_row ? yn : 0.0f;
}

// this lane's nonzero split entries in k order (at most 12 kept) as
// coefficients sc and bpermute byte addresses sa (y_k on lane 2k), compacted
// through LDS (a per-lane slot index) rather than a select per (k, slot);
// returns the lane's count (> 12: the dense form is needed).  Unused slots:
// coefficient 0 on this row's own y, which adds +0 for a finite y.
template <int NMAX>
__device__ __forceinline__ int sparse_lists(const float (&mat)[NMAX], int lane, int N, float (&lsc)[12][64],
                                            int (&lsa)[12][64], float (&sc)[12], int (&sa)[12]) {
    const int i = lane >> 1;
#pragma unroll
    for (int s = 0; s < 12; ++s) {
        lsc[s][lane] = 0.0f;
        lsa[s][lane] = (i < N ? 2 * i : 0) * 4;
    }
    int nnz = 0;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {
        if (mat[k] != 0.0f || mat[k] != mat[k]) {  // nonzero or NaN: summed
            if (nnz < 12) {
                lsc[nnz][lane] = mat[k];
                lsa[nnz][lane] = 8 * k;
            }
            ++nnz;
        }
    }
#pragma unroll
    for (int s = 0; s < 12; ++s) {
        sc[s] = lsc[s][lane];
        sa[s] = lsa[s][lane];
    }
    return nnz;
}
// the largest count over the wave (wave-uniform)
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

// Y, the state and the error word to the device (for a resumed launch) and to
// the pinned host buffer (layout kTinyOut*, pqp_launch.h)
__device__ __forceinline__ void write_out(const SolveArgs& A, SolveState* st, int tid, const float* Y, int N,
                                          const SolveState& s, int err) {
    for (int k = tid; k < N; k += 64) A.Y[k] = Y[k];
    if (tid == 0) {
        *st = s;
        *reinterpret_cast<int*>(reinterpret_cast<char*>(st) + kTinyDevErr) = err;  // pqp_launch.h
    }
    if (A.hout) {
        // host memory (fine-grained): system-scope write-through stores of the
        // data, their completion (vmcnt), then the launch's tag -- the host
        // takes the buffer only with its own tag (a full system fence here, an
        // L2 write-back, cost 11 us per launch: profiles/r05/bundled_ab_r05x.json)
        int* hy = static_cast<int*>(A.hout);
        for (int k = tid; k < N; k += 64)
            __hip_atomic_store(hy + k, __float_as_int(Y[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (tid == 0) {
            const int* sw = reinterpret_cast<const int*>(&s);
            for (int e = 0; e < (int)(sizeof(SolveState) / 4); ++e)
                __hip_atomic_store(hy + kTinyOutStateOffset + e, sw[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(hy + kTinyOutErrOffset, err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) __hip_atomic_store(hy + kTinyOutTagOffset, A.out_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// k_fixed_one<NMAX>: fixed mode of one problem on one wave (see the header).
// ---------------------------------------------------------------------------
template <int NMAX>
__global__ void __launch_bounds__(64) k_fixed_one(SolveArgs A, SolveState* __restrict__ st) {
    SolveState s0 = A.fresh ? SolveState{1, kStatusContinue, 0, 0.0f, 0.0f, 0, 0} : *st;
    if (s0.status == kStatusDone || s0.status == kStatusCapped) return;
    __shared__ float yout[NMAX];
    const int N = A.N;
    const int lane = threadIdx.x, i = lane >> 1, side = lane & 1;
    const bool own_row = !side && i < N;
    float mat[NMAX], fd_own;
    split_row<NMAX>(A, lane, mat, fd_own);
    __shared__ float lsc[12][64];
    __shared__ int lsa[12][64];
    float sc[12];
    int sa[12];
    const int nnz = sparse_lists<NMAX>(mat, lane, N, lsc, lsa, sc, sa);
    const int pmax = wave_max(nnz);  // the widest lane decides the form
    float yk = 0.0f;
    if (own_row) yk = s0.resume ? A.Y[i] : 1000.0f;  // initMat(Y, 1000) :710
    long long h = s0.h;
    const long long left = A.num_iter - h;             // while(h < NUM_ITER)
    const long long todo = left < A.chunk ? left : A.chunk;
    int n = todo > 0 ? (int)todo : 0;
    int dense_from = 0;  // updates done in the sparse form
    if (!(A.tiny_flags & kTinyDense) && pmax <= 12) {
        // the sparse form while every y is finite.  Blocks of 8 updates test
        // the finiteness of each update's input once per block (a per-lane
        // flag beside the chain, not a branch on it; round 6); a block that met
        // a non-finite y is done again from its start in the dense form.  The
        // last < 8 updates test before each update.
#define PQP_SPARSE_LOOP(PP)                                                   \
    while (dense_from + 8 <= n) {                                             \
        const float y_blk = yk;                                               \
        bool nf = false;                                                      \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) {                       \
            nf |= !__builtin_isfinite(yk);                                    \
            yk = update_sparse<PP>(sc, sa, fd_own, yk, own_row);              \
        }                                                                     \
        if (__any(nf)) {                                                      \
            yk = y_blk;                                                       \
            break;                                                            \
        }                                                                     \
        dense_from += 8;                                                      \
    }                                                                         \
    if (dense_from + 8 > n)                                                   \
        for (; dense_from < n; ++dense_from) {                                \
            if (__any(!__builtin_isfinite(yk))) break;                        \
            yk = update_sparse<PP>(sc, sa, fd_own, yk, own_row);              \
        }
        if (pmax <= 2) {
            PQP_SPARSE_LOOP(2)
        } else if (pmax <= 4) {
            PQP_SPARSE_LOOP(4)
        } else if (pmax <= 8) {
            PQP_SPARSE_LOOP(8)
        } else {
            PQP_SPARSE_LOOP(12)
        }
#undef PQP_SPARSE_LOOP
    }
    for (int u = dense_from; u < n; ++u) yk = update_dense<NMAX>(mat, fd_own, yk, own_row);
    h += n;
    if (own_row) yout[i] = yk;
    __syncthreads();
    SolveState s = s0;
    s.h = h;
    s.status = h >= A.num_iter ? kStatusDone : kStatusContinue;
    s.resume = 1;
    write_out(A, st, lane, yout, N, s, 0);
}

// ---------------------------------------------------------------------------
// k_solve_quintet<NMAX, MMAX>: converge mode of one problem on five waves (see
// the header): A the update (its own SIMD), B0 / B1 the N-long sums of the
// even / odd iterates (sharing a SIMD: waves 0 and 4 of a workgroup are
// placed on one, profiles/r02/persist_probes/simd_map_probe.txt), C0 / C1
// the M-side chain and the decision of the even / odd iterates (decisions
// are taken in iterate order: C_p decides r once r - 1 is decided).  A takes
// the sparse update form while every y is finite (as k_fixed_one).  B and C
// form their products ahead of the add chains (sched_barrier); B's
// (Y'Qd).Y terms come back through LDS (a v_readlane costs ~10 clocks and an
// add reading its SGPR ~6.5 here, profiles/r05/trio_trace_*.json).
// N + M < 64, N, M <= 32.
// ---------------------------------------------------------------------------
template <int NMAX, int MMAX, int NP>
struct QuintetLds {
    float y[kRing][NMAX];   // Y_h            (A -> B, and the output)
    float t[kRing][MMAX];   // Gp'Y_h + Fp    (B -> C)
    float s2[kRing];        // (Y_h'Qd).Y_h   (B -> C)
    float lind[kRing];      // Fd.Y_h         (B -> C)
    float q[NP][NMAX];      // B_p's (Y'Qd)_j y_j terms, read back as broadcasts
    float lsc[12][64];      // A's sparse lists (setup)
    int lsa[12][64];
    SolveState out;         // the final state (by the deciding wave), written out by A after the barrier
    float jp, jd;           // costs of the last decided feasible iterate
    int have;
    int a_h, b_h[NP], decided;  // iterates (relative to the launch's first) published by A, B_p; decided by the C_p
    int h_end, err;
};

// NP (round 6): the B and C roles on NP waves each, iterate r on B_{r mod NP}
// and C_{r mod NP} -- 2 (five waves), 3 or 4 (seven / nine: each B / C wave
// has NP iterates' time for its own)
template <int NMAX, int MMAX, bool TRACE, int NP = 2, bool A_CACHE = false, int ABLK = 1>
__global__ void __launch_bounds__(64 * (1 + 2 * NP)) k_solve_quintet(SolveArgs A, SolveState* __restrict__ st) {
    static_assert(NMAX % 4 == 0 && MMAX % 4 == 0 && NMAX <= 32 && MMAX <= 32, "one wave per role");
    static_assert(NP >= 2 && NP <= 4, "two to four B / C waves");
    static_assert(!TRACE || NP == 2, "the timeline's layout is the five-wave one");
    constexpr int NT = 64 * (1 + 2 * NP);
    SolveState s0 = A.fresh ? SolveState{1, kStatusContinue, 0, 0.0f, 0.0f, 0, 0} : *st;
    if (s0.status == kStatusDone || s0.status == kStatusCapped) return;
    __shared__ __attribute__((aligned(16))) QuintetLds<NMAX, MMAX, NP> S;
    const int N = A.N, M = A.M;
    const int tid = threadIdx.x, lane = tid & 63;
    // roles by hardware wave (waves w and w + 4 share a SIMD): 0 / 4 B0 / B1,
    // 1 A, 2 / 3 C0 / C1; beyond, odd waves C_p and even ones B_p (NP = 3: 5 C2
    // beside A, 6 B2 beside C0; NP = 4: 7 C3 beside C1, 8 B3).  Role numbers
    // (the five-wave timeline's): 0 A, 1 B0, else the hardware wave
    const int hw = tid >> 6;
    const int role = hw == 1 ? 0 : (hw == 0 ? 1 : hw);
    const bool is_b = hw == 0 || (hw >= 4 && !(hw & 1));
    const int bpar = hw == 0 ? 0 : hw / 2 - 1;                     // B's parity
    const int cpar = hw == 2 ? 0 : (hw == 3 ? 1 : (hw - 1) / 2);   // C's parity
    // padding y_k, t_j = +0: C reads all MMAX entries of t (times qinv's zero
    // padding), and LDS holds whatever the previous kernel left -- a NaN there
    // made 0 * NaN a NaN U (seen after kernels that ran on non-finite data)
    for (int k = tid; k < kRing * NMAX; k += NT) (&S.y[0][0])[k] = 0.0f;
    for (int k = tid; k < kRing * MMAX; k += NT) (&S.t[0][0])[k] = 0.0f;
    if (tid == 0) {
        S.a_h = -1;
        for (int p = 0; p < NP; ++p) S.b_h[p] = -1;
        S.decided = -1;
        S.h_end = 0;
        S.err = 0;
        S.have = 0;
        S.out = s0;
    }
    __syncthreads();
    const long long h0 = s0.h;
    const int spin_max = (A.tiny_flags & kTinyStall) ? (1 << 14) : kSpinMax;
    // TRACE: each wave's shader clocks in total and inside its waits
    unsigned long long t_start = TRACE ? __builtin_amdgcn_s_memtime() : 0, t_wait = 0, t_w0 = 0;
    int n_iter = 0;
#define QT_WAIT_BEGIN() \
    if (TRACE) t_w0 = __builtin_amdgcn_s_memtime();
#define QT_WAIT_END()                                  \
    if (TRACE) {                                       \
        t_wait += __builtin_amdgcn_s_memtime() - t_w0; \
        ++n_iter;                                      \
    }

    if (role == 0) {
        // ---------------- wave A: updateY2 ----------------
        float mat[NMAX], fd_own;
        split_row<NMAX>(A, lane, mat, fd_own);
        float sc[12];
        int sa[12];
        const int pmax = wave_max(sparse_lists<NMAX>(mat, lane, N, S.lsc, S.lsa, sc, sa));
        bool sparse = !(A.tiny_flags & kTinyDense) && pmax <= 4;
        const int i = lane >> 1;
        const bool own_row = !(lane & 1) && i < N;
        float yk = 0.0f;
        if (own_row) yk = s0.resume ? A.Y[i] : 1000.0f;  // initMat(Y, 1000) :710
        if (own_row) S.y[0][i] = yk;
        lds_publish(&S.a_h, 0);
        int d_seen = -1;
        for (int r = 1;; r += ABLK) {
            // ABLK updates per pass.  The sparse form only while every input y
            // is finite (the skipped +-0 terms are then exact): one test per
            // pass, a per-lane flag beside the chain (round 6); a pass that met
            // a non-finite y is done again densely from its start
            float yb[ABLK];
            if (sparse) {
                const float y_blk = yk;
                bool nf = false;
#pragma unroll
                for (int j = 0; j < ABLK; ++j) {
                    nf |= !__builtin_isfinite(yk);
                    if (pmax <= 2) yk = update_sparse<2>(sc, sa, fd_own, yk, own_row);
                    else yk = update_sparse<4>(sc, sa, fd_own, yk, own_row);
                    yb[j] = yk;
                }
                if (__any(nf)) {
                    sparse = false;
                    yk = y_blk;
#pragma unroll
                    for (int j = 0; j < ABLK; ++j) yb[j] = yk = update_dense<NMAX>(mat, fd_own, yk, own_row);
                }
            } else {
#pragma unroll
                for (int j = 0; j < ABLK; ++j) yb[j] = yk = update_dense<NMAX>(mat, fd_own, yk, own_row);
            }
            // room in the ring: iterate r - kRing decided (or the solve over).
            // The last decision seen is kept and the word read again only when
            // it leaves no room (round 6, A_CACHE, the default: bundled converge
            // 0.1144 -> 0.1045 ms per solve): no LDS round trip on the update's
            // path while A runs ahead.  A learns of the stop when the ring
            // fills (at most kRing discarded updates).
            // (a pass of ABLK updates needs its last slot free: iterate r + ABLK - 1 - kRing decided)
            if (!A_CACHE || d_seen < r + ABLK - 1 - kRing) {
                int spin = 0;
                QT_WAIT_BEGIN()
                for (;; ++spin) {
                    d_seen = lds_ld(&S.decided);
                    if (d_seen == kStopWord || d_seen >= r + ABLK - 1 - kRing || spin > spin_max) break;
                }
                QT_WAIT_END()
                lds_after_wait();
                if (d_seen == kStopWord) break;
                if (spin > spin_max) {
                    S.err = 1;
                    break;
                }
            }
#pragma unroll
            for (int j = 0; j < ABLK; ++j)
                if (own_row) S.y[(r + j) & (kRing - 1)][i] = yb[j];
            lds_publish(&S.a_h, r + ABLK - 1);
        }
    } else if (is_b) {
        // ---------------- waves B0 / B1: the N-long sums of terminate(Y_h) ----------------
        // lane j < N: Qd column j -> (Y'Qd)_j (computeCost :652); lane N + j:
        // Gp column j -> (Gp'Y)_j (computeUfromY :354); lane N + M: Fd -> Fd.Y (:657)
        const int lf = N + M;
        float col[NMAX];
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
            float v = 0.0f;
            if (k < N) {
                if (lane < N) v = A.Qd[k * N + lane];
                else if (lane < N + M) v = A.Gp[k * M + (lane - N)];
                else if (lane == lf) v = A.Fd[k];
            }
            col[k] = v;
        }
        const bool is_t = lane >= N && lane < N + M;
        const float fp_own = is_t ? A.Fp[lane - N] : 0.0f;
        const int lown = lane < NMAX ? lane : 0;
        const int bp = bpar;
        int a_seen = -1;
        unsigned long long ph[4] = {0, 0, 0, 0}, tm = 0;  // TRACE: clocks per phase of B's iterate
#define QT_MARK(k)                                          \
    if (TRACE) {                                            \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        ph[k] += t_ - tm;                                   \
        tm = t_;                                            \
    }
        for (int r = bp;; r += NP) {
            if (TRACE) tm = __builtin_amdgcn_s_memtime();
            if (a_seen < r) {
                int spin = 0;
                bool over = false;
                QT_WAIT_BEGIN()
                for (;; ++spin) {
                    a_seen = lds_ld(&S.a_h);
                    if (a_seen >= r) break;
                    if (lds_ld(&S.decided) == kStopWord || spin > spin_max) {
                        if (spin > spin_max) S.err = 1;
                        over = true;
                        break;
                    }
                }
                QT_WAIT_END()
                if (over) break;
            }
            lds_after_wait();
            QT_MARK(0)
            const int slot = r & (kRing - 1);
            f4v y4[NMAX / 4];
#pragma unroll
            for (int g = 0; g < NMAX / 4; ++g) y4[g] = *reinterpret_cast<const f4v*>(&S.y[slot][4 * g]);
            const float y_own = S.y[slot][lown];
            const float* yv = reinterpret_cast<const float*>(y4);
            float p[NMAX];
#pragma unroll
            for (int k = 0; k < NMAX; k += 2) {
                const f2v pr = f2v{col[k], col[k + 1]} * f2v{yv[k], yv[k + 1]};
                p[k] = pr.x;
                p[k + 1] = pr.y;
            }
            __builtin_amdgcn_sched_barrier(0);
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < NMAX; ++k) acc += p[k];  // k in order
            QT_MARK(1)
            if (is_t) S.t[slot][lane - N] = acc + 1.0f * fp_own;  // tmp += Fp (:355)
            if (lane == lf) S.lind[slot] = acc;
            // (Y'Qd).Y: the terms (Y'Qd)_j * y_j on lanes j, summed in j order (:655),
            // back through LDS as broadcasts
            if (lane < NMAX) S.q[bp][lane] = lane < N ? acc * y_own : 0.0f;
            // the next iterate's progress word, read while the terms travel
            if (a_seen < r + NP) a_seen = lds_ld(&S.a_h);
            f4v q4[NMAX / 4];
#pragma unroll
            for (int g = 0; g < NMAX / 4; ++g) q4[g] = *reinterpret_cast<const f4v*>(&S.q[bp][4 * g]);
            const float* qs = reinterpret_cast<const float*>(q4);
            QT_MARK(2)
            float s2 = 0.0f;
#pragma unroll
            for (int j = 0; j < NMAX; ++j) s2 += qs[j];
            if (lane == 0) S.s2[slot] = s2;
            lds_publish(&S.b_h[bp], r);
            QT_MARK(3)
        }
#undef QT_MARK
        if (TRACE && lane == 0 && A.trace && bp == 0)
            for (int k = 0; k < 4; ++k) A.trace[20 + k] = ph[k];
    } else {
        // ---------------- waves C0 / C1: the M-side chain and the decision ----------------
        // lane j < M: Qp_inv row j (U = -Qp_inv t); gq[j].x: lane i < N Gp row i
        // (checkFeas), lane N Fp (Fp.U); gq[j].y: lane k < M Qp column k (U'Qp)
        const int par = cpar;
        const bool stall = (A.tiny_flags & kTinyStall) != 0;  // error-path test: no decision ever comes
        float qinv[MMAX];
        f2v gq[MMAX];
#pragma unroll
        for (int j = 0; j < MMAX; ++j) {
            const bool jm = j < M;
            qinv[j] = (jm && lane < M) ? A.Qinv[lane * M + j] : 0.0f;
            float gx = 0.0f;
            if (jm && lane < N) gx = A.Gp[lane * M + j];
            else if (jm && lane == N) gx = A.Fp[j];
            gq[j] = f2v{gx, (jm && lane < M) ? A.Qp[j * M + lane] : 0.0f};
        }
        const float kp = lane < N ? A.Kp[lane] : 0.0f;
        const float Md = A.Md[0], Mp = A.Mp[0];
        for (int r = par; !stall; r += NP) {
            int b, spin = 0;
            bool over = false;
            QT_WAIT_BEGIN()
            for (;; ++spin) {
                b = lds_ld(&S.b_h[par]);
                if (b >= r) break;
                if (lds_ld(&S.decided) == kStopWord || spin > spin_max) {
                    if (spin > spin_max) S.err = 1;
                    over = true;
                    break;
                }
            }
            QT_WAIT_END()
            lds_after_wait();
            if (over) break;
            const int slot = r & (kRing - 1);
            f4v t4[MMAX / 4];
#pragma unroll
            for (int g = 0; g < MMAX / 4; ++g) t4[g] = *reinterpret_cast<const f4v*>(&S.t[slot][4 * g]);
            const float* tv = reinterpret_cast<const float*>(t4);
            const float s2 = S.s2[slot], lin_d = S.lind[slot];
            float pu[MMAX];
#pragma unroll
            for (int l = 0; l < MMAX; ++l) pu[l] = qinv[l] * tv[l];
            __builtin_amdgcn_sched_barrier(0);
            float ua = 0.0f;  // U = Qp_inv t, l in order (:356)
#pragma unroll
            for (int l = 0; l < MMAX; ++l) ua += pu[l];
            const float u = lane < M ? -ua : 0.0f;  // U = -U (:357-359)
            float uv[MMAX];
#pragma unroll
            for (int j = 0; j < MMAX; ++j) uv[j] = rdl(u, j);
            f2v pg[MMAX];
#pragma unroll
            for (int j = 0; j < MMAX; ++j) pg[j] = gq[j] * f2v{uv[j], uv[j]};
            __builtin_amdgcn_sched_barrier(0);
            f2v g = f2v{0.0f, 0.0f};  // .x Gp U (checkFeas :636) / Fp.U ; .y U'Qp (:652)
#pragma unroll
            for (int j = 0; j < MMAX; ++j) g += pg[j];
            const int bad = lane < N && (g.x > kp + max_ref((float)(kTol * kp), (float)kTol));
            const bool infeasible = __any(bad);
            int stop = 0;
            float Jp = 0.0f, Jd = 0.0f;
            if (!infeasible) {
                const float lin_p = rdl(g.x, N);
                const float qt = lane < M ? g.y * u : 0.0f;  // (U'Qp)_k * u_k on lane k
                float qk[MMAX];
#pragma unroll
                for (int k = 0; k < MMAX; ++k) qk[k] = rdl(qt, k);
                __builtin_amdgcn_sched_barrier(0);
                float quad = 0.0f;  // (U'Qp).U, k in order (:655)
#pragma unroll
                for (int k = 0; k < MMAX; ++k) quad += qk[k];
                Jp = (float)((double)Jp + 0.5 * (double)quad);
                Jp += lin_p;
                Jp += Mp / 2;
                Jd = (float)((double)Jd + 0.5 * (double)s2);
                Jd += lin_d;
                Jd += Md / 2;
                stop = gap_stop(Jp, Jd);  // :683-685
            }
            // decisions in iterate order: r - 1 first
            int d;
            spin = 0;
            for (;; ++spin) {
                d = lds_ld(&S.decided);
                if (d == r - 1 || d == kStopWord || spin > spin_max) break;
            }
            lds_after_wait();
            if (d != r - 1) {
                if (spin > spin_max) S.err = 1;
                break;
            }
            if (!infeasible && lane == 0) {  // the last feasible iterate's costs (:673-687)
                S.jp = Jp;
                S.jd = Jd;
                S.have = 1;
            }
            const long long h = h0 + r;
            int status = -1;
            if (stop) status = kStatusDone;
            else if (A.max_updates > 0 && h - 1 >= A.max_updates) status = kStatusCapped;
            else if (r >= A.chunk) status = kStatusContinue;
            if (status >= 0) {
                // computeUfromY wrote U on every terminate(): this one's stands
                if (lane < M) A.U[lane] = u;
                if (A.hout && lane < M)
                    __hip_atomic_store(static_cast<int*>(A.hout) + kTinyOutUOffset + lane, __float_as_int(u),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // U completed before wave A's tag
                if (lane == 0) {
                    SolveState so = s0;
                    so.h = h;
                    so.status = status;
                    so.resume = 1;
                    if (S.have) {
                        so.Jp = S.jp;
                        so.Jd = S.jd;
                        so.have_costs = 1;
                    }
                    S.out = so;
                    S.h_end = r;
                    lds_publish(&S.decided, kStopWord);
                }
                break;
            }
            lds_publish(&S.decided, r);
        }
    }
    if (TRACE && lane == 0 && A.trace) {
        A.trace[4 * role + 0] = __builtin_amdgcn_s_memtime() - t_start;
        A.trace[4 * role + 1] = t_wait;
        A.trace[4 * role + 2] = n_iter;
    }
#undef QT_WAIT_BEGIN
#undef QT_WAIT_END
    __syncthreads();
    if (role == 0) {
        const int slot = S.h_end & (kRing - 1);
        SolveState s = S.out;
        if (S.err) s.status = kStatusContinue;  // an expired wait: the host reports it (err word)
        write_out(A, st, lane, &S.y[slot][0], N, s, S.err);
    }
}

// Test hook (pqp_tune_poison_lds): every workgroup fills 64 KB of LDS with
// `bits` and leaves it there, over enough workgroups to pass through every CU:
// a later kernel that reads LDS it never wrote (padding) then sees the value.
__global__ void __launch_bounds__(256) k_poison_lds(int bits, int* __restrict__ seen) {
    __shared__ int pool[16384];
    for (int k = threadIdx.x; k < 16384; k += 256) pool[k] = bits;
    __syncthreads();
    // a read the compiler cannot predict keeps the stores
    if (pool[(threadIdx.x * 61 + blockIdx.x) & 16383] != bits) seen[0] = 1;
}

}  // namespace

hipError_t launch_poison_lds(int bits, int* seen, int cus, hipStream_t s) {
    hipLaunchKernelGGL(k_poison_lds, dim3(8 * (cus > 0 ? cus : 256)), dim3(256), 0, s, bits, seen);
    return hipGetLastError();
}

hipError_t launch_one_tiny(const SolveArgs& a, SolveState* st, hipStream_t s) {
    if (a.N > 32 || a.M > 32) return hipErrorInvalidValue;
    if (a.mode == kModeFixed) {
        if (a.N <= 8) hipLaunchKernelGGL((k_fixed_one<8>), dim3(1), dim3(64), 0, s, a, st);
        else if (a.N <= 16) hipLaunchKernelGGL((k_fixed_one<16>), dim3(1), dim3(64), 0, s, a, st);
        else if (a.N <= 24) hipLaunchKernelGGL((k_fixed_one<24>), dim3(1), dim3(64), 0, s, a, st);
        else if (a.N <= 28) hipLaunchKernelGGL((k_fixed_one<28>), dim3(1), dim3(64), 0, s, a, st);
        else hipLaunchKernelGGL((k_fixed_one<32>), dim3(1), dim3(64), 0, s, a, st);
        return hipGetLastError();
    }
    if (a.mode != kModeConverge || a.N + a.M >= 64) return hipErrorInvalidValue;
    const int np = (g_tune.tiny_np >= 2 && g_tune.tiny_np <= 4) ? g_tune.tiny_np : 3;  // B / C waves per role
#define PQP_TRIO_NP(NN, MM, NPP)                                                                                  \
    do {                                                                                                          \
        if (g_tune.tiny_apoll)                                                                                    \
            hipLaunchKernelGGL((k_solve_quintet<NN, MM, false, NPP>), dim3(1), dim3(64 * (1 + 2 * NPP)), 0, s, a, \
                               st);                                                                               \
        else if (g_tune.tiny_ablk == 1)                                                                           \
            hipLaunchKernelGGL((k_solve_quintet<NN, MM, false, NPP, true>), dim3(1), dim3(64 * (1 + 2 * NPP)), 0, \
                               s, a, st);                                                                         \
        else                                                                                                      \
            hipLaunchKernelGGL((k_solve_quintet<NN, MM, false, NPP, true, 2>), dim3(1), dim3(64 * (1 + 2 * NPP)), \
                               0, s, a, st);                                                                      \
    } while (0)
#define PQP_TRIO_MM(NN, MM)                      \
    do {                                         \
        if (np == 3) PQP_TRIO_NP(NN, MM, 3);     \
        else if (np == 4) PQP_TRIO_NP(NN, MM, 4); \
        else PQP_TRIO_NP(NN, MM, 2);             \
    } while (0)
#define PQP_TRIO_M(NN)                                                                                \
    do {                                                                                              \
        if (a.trace && a.N == 28 && a.M <= 8)                                                         \
            hipLaunchKernelGGL((k_solve_quintet<28, 8, true>), dim3(1), dim3(320), 0, s, a, st);      \
        else if (a.M <= 8) PQP_TRIO_MM(NN, 8);                                                        \
        else if (a.M <= 16) PQP_TRIO_MM(NN, 16);                                                      \
        else PQP_TRIO_MM(NN, 32);                                                                     \
    } while (0)
    if (a.N <= 8) PQP_TRIO_M(8);
    else if (a.N <= 16) PQP_TRIO_M(16);
    else if (a.N <= 24) PQP_TRIO_M(24);
    else if (a.N <= 28) PQP_TRIO_M(28);
    else PQP_TRIO_M(32);
#undef PQP_TRIO_M
#undef PQP_TRIO_MM
#undef PQP_TRIO_NP
    return hipGetLastError();
}

}  // namespace pqp
