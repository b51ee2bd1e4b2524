// pqp_converge.hip -- converge mode of ONE problem with n_dual, M <= 1024 as
// ONE persistent, pipelined launch (solveQuadraticDual, PQP_CPU.c:694-750).
//
// The reference alternates terminate(Y_u) (:673-687) and updateY2 (:603-618).
// updateY2 does not depend on terminate's answer, only on Y_u, so the two can
// overlap: the launch runs the update chain and the stages of terminate() as
// concurrent ROLES on disjoint workgroups, each looping over iterates u and
// passing vectors downstream through rings of tagged 8-byte granules
// {tag = u + 1, bits(value)} in global memory (the data is its own flag):
//
//   UPD  y_{u+1} = updateY2(y_u)             2N/32 workgroups  ring ry   [N]
//   T1   tmp_u = Gp'y_u + Fp, tq_u = y_u'Qd  (N+M)/32          rtmp [M], rtq [N]
//   T2   U_u = -(Qp_inv tmp_u)               M/32              rU   [M]
//   T3   Gp U_u vs Kp, tu_u = U_u'Qp         (N+M)/32          rfeas[wg], rtu [M]
//   DEC  the four dots of computeCost, the gap tests, the decision  (1 workgroup;
//        the N-long dots on two waves each, even and odd iterates; the M-long
//        dots skipped on an infeasible iterate, as terminate() skips them)
//
// Every output is one lane's sum over k in order from +0.0f, the reference's
// matrixMultiply order (:88-100), formed exactly as in k_split_persist: the
// stage's matrix columns stay in LDS for the whole solve (32 columns per
// workgroup), wave w of a workgroup owns a k-slice, forms its products ahead
// of its turn, adds them when the running sums arrive from wave w-1 and hands
// them on through an LDS word; the last wave applies the epilogue (Fp add,
// negation, the Kp comparison) and publishes.
//
// DEC decides iterates in order.  When terminate(y_u) passes (or u reaches the
// cap) it writes h = u + 1, Jp, Jd, copies y_u and U_u out of the rings and
// raises the control word; every waiting wave sees it and leaves.  Otherwise
// it publishes `decided = u`.  Rings are kR deep and UPD publishes y_{u+1}
// only once decided >= u + 1 - kR: every role has then finished iterate
// u + 1 - kR, so no slot is overwritten while it is still read.  Speculative
// updates past the stopping iterate are simply discarded.  Every wait is
// bounded in time (2 s): a workgroup that never gets a CU ends the launch with
// an error word instead of a hang.
//
// A launch decides at most `chunk` iterates; the host relaunches from the
// iterate it left in Yout until the status leaves Continue.
//
// Requirement: all workgroups resident at once (one per CU by their LDS); the
// host checks the count against the device's CUs.
#include "pqp_device.h"
#include "pqp_launch.h"
#include "pqp_chain.h"

#include <type_traits>

#pragma clang fp contract(off)

namespace pqp {

namespace {


constexpr int kL = kSliceLanes;  // output columns (update: row sides) per workgroup
constexpr int kP0 = 24;    // packets (4 values of k) of wave 0's slice, multiplied inside its chain
constexpr int kP1 = 36;    // packets of wave 1's slice: its products must be ready when wave 0 is done
constexpr int kPW = 49;    // packets per later slice, products formed ahead in 4 kPW VGPRs
constexpr int kLateGate = 1;
#ifndef PQP_T_POLL_SLEEP
#define PQP_T_POLL_SLEEP 4
#endif
constexpr int kTPollSleep = PQP_T_POLL_SLEEP;  // s_sleep units (64 clocks) between the T roles' and DEC's sweeps
static_assert(kP0 <= 64 && kP1 <= 64 && kPW <= 64, "a slice is at most 4 granules per lane (one sweep)");  // waves 4, 5 (sharing SIMDs with 0, 1) form products once this wave is done
constexpr int kMaxW = 7;   // waves per workgroup: the chain roles use up to 6 (K <= 1024), DEC 7
#ifndef PQP_CV_DIAG  // timing diagnostic only (wrong results): 1 UPD alone, 2 UPD + T1, 3 UPD + T1-T3; DEC decides blind
#define PQP_CV_DIAG 0
#endif
#ifndef PQP_CV_NOBP  // timing diagnostic only (with PQP_CV_DIAG): no backpressure check
#define PQP_CV_NOBP 0
#endif
#ifndef PQP_CV_UPD_INPLACE  // upd_wave: later waves read their q while they wait for y
#define PQP_CV_UPD_INPLACE 1
#endif
#ifndef PQP_CV_SLEEP0  // s_sleep units between UPD wave 0's / wave 1's / later waves' y sweeps
#define PQP_CV_SLEEP0 0  // wave 0 (the chain starts on its slice) polls back to back
#endif
#ifndef PQP_CV_SLEEP1
#define PQP_CV_SLEEP1 1
#endif
#ifndef PQP_CV_SLEEPN
#define PQP_CV_SLEEPN 4  // waves 2+ (their turn comes later) poll a quarter as often
#endif
#ifndef PQP_CONVERGE_RING
#define PQP_CONVERGE_RING 8
#endif
constexpr int kR = PQP_CONVERGE_RING;  // ring depth (iterates in flight), a power of 2
static_assert((kR & (kR - 1)) == 0, "ring slots are iterate & (kR - 1)");
constexpr int kDecW = 7;     // DEC's waves: the decision, then the dot waves (dec_dots)
constexpr int kDots = 4;     // computeCost's dots, hand-off word 1..4 of a ring slot
constexpr int kDecBufs = 8;  // product buffers: waves 1-4 one each, waves 5 and 6 two each
constexpr int kDecPer = 16;  // dot terms per lane (n <= 1024)
constexpr int kDecChunk = 256;  // dot terms per unrolled chunk
constexpr int kDecAhead = 4;    // groups of 16 terms read ahead of the adds
enum Role : int { kUpd = 0, kT1 = 1, kT2 = 2, kT3 = 3, kDec = 4 };

// slices of kP0, kP1, then kPW packets (as k_split_persist)
__host__ __device__ inline int slice0_of(int w) { return w == 0 ? 0 : (w == 1 ? kP0 : kP0 + kP1 + (w - 2) * kPW); }
__host__ __device__ inline int packets_of(int W) { return slice0_of(W); }
__host__ __device__ inline int waves_of(int KB) {
    int W = 1;
    while (packets_of(W) < KB) ++W;
    return W;
}
__host__ __device__ inline int cdiv_i(int a, int b) { return (a + b - 1) / b; }
__device__ __forceinline__ u64 granule(unsigned tag, float v) { return ((u64)tag << 32) | __float_as_uint(v); }




}  // namespace

struct CvArgs {
    int N, M;
    int g1, g2, g3, g4;                  // role boundaries: [0,g1) UPD, [g1,g2) T1, [g2,g3) T2, [g3,g4) T3, g4 DEC
    long long u0;                        // iterate this launch starts from (y_{u0} in ring slot u0 % kR)
    long long u_dec_end;                 // last iterate DEC decides in this launch
    long long u_prod_end;                // last iterate UPD produces
    long long cap;                       // max_updates (<= 0: none)
    const f4v *SPu, *A1, *A2, *A3;       // LDS-resident packets per role: [wg][KB][32]
    const float *fdpn, *Fp, *Kp, *Fd, *Md, *Mp;
    u64 *ry, *rtmp, *rtq, *rU, *rtu, *rfeas;
    SolveState* st;
    int* ctl;             // 0 running, 1 finished, 2 failed
    long long* decided;   // last iterate DEC let through
    int* err;
    float *Yout, *Uout;
    u64* trace;           // tuning: [2][iterate][kTraceIds][4] s_memrealtime, then s_memtime marks of workgroup 0 of each role
    int trace_n;
    int stall_wg;  // tuning: this workgroup never runs (error-path tests; -1: none)
    int xcds;      // > 0: the roles' workgroups on this many XCDs (blockIdx % 8 < xcds take part)
};

namespace {

__device__ __forceinline__ bool stopped(const CvArgs& a) {
    return __hip_atomic_load(a.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
__device__ __forceinline__ void fail(const CvArgs& a, int code) {
    __hip_atomic_store(a.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.ctl, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until every listed granule with on[m] carries `tag`; v[m] gets its
// value.  Every g[m] must be a valid address, on or not.  Returns false when
// the launch has been stopped or the wait timed out.
template <int NG, int SLEEP = 1>
__device__ __forceinline__ bool await_granules(const CvArgs& a, const gu64* const (&g)[NG], const bool (&on)[NG],
                                               unsigned tag, float (&v)[NG], int code) {
    Deadline dl;
    for (unsigned spins = 0;; ++spins) {
        // every address is valid (callers clamp the unused ones), so the loads
        // are unconditional: all NG in flight at once, no branch around each
        u64 x[NG];
#pragma unroll
        for (int m = 0; m < NG; ++m) x[m] = __hip_atomic_load(g[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
#pragma unroll
        for (int m = 0; m < NG; ++m) {
            v[m] = __uint_as_float((unsigned)x[m]);
            ok &= !on[m] || (unsigned)(x[m] >> 32) == tag;
        }
        if (__all(ok)) return true;
        if ((spins & 63) == 63) {
            if (stopped(a)) return false;
            if (dl.expired()) {
                fail(a, code);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(SLEEP);
    }
}

constexpr int kTraceIds = 4 * kMaxW + kDecW;
template <bool TRACE>
__device__ __forceinline__ void mark(const CvArgs& a, bool on, long long u, int id, int e) {
    if constexpr (TRACE)
        if (on && u - a.u0 < a.trace_n) {
            // chip time (100 MHz), then the shader clock in a second block: the
            // ratio over a span is the clock the launch ran at
            const size_t i = ((size_t)(u - a.u0) * kTraceIds + id) * 4 + e;
            a.trace[i] = __builtin_amdgcn_s_memrealtime();
            a.trace[(size_t)a.trace_n * kTraceIds * 4 + i] = __builtin_amdgcn_s_memtime();
        }
}

// The running sums' hand-off wait of a chain wave: a bare poll whose exit
// falls through into the adds; the launch's stop flag and the time limit are
// read every 256 polls only.  0: arrived, 1: the launch stopped, 2: timed out.
__device__ __forceinline__ int wait_sums(const CvArgs& a, const u64* src, unsigned tag, u64& h) {
    Deadline dl;
    unsigned spins = 0;
    bool ok;
#pragma clang loop unroll(disable)
    do {
        h = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ok = __all((unsigned)(h >> 32) == tag);
    } while (!ok && ((++spins & 255) != 0 || !(stopped(a) || dl.expired())));
    return ok ? 0 : (stopped(a) ? 1 : 2);
}

// UPD role, one wave: k_split_persist's update (pqp_persist.hip) on the ring.
// Per iterate u: the wave's slice of y_u from ring slot u % kR (tag u + 1),
// products ahead of its turn (waves > 0 read their q while they wait for y and
// multiply in place), the running sums through one 64-bit LDS word per lane
// and update parity ([2][W][64] words inside the hand-off area), each chain
// form running straight into its hand-off or epilogue; the last wave divides
// and publishes y_{u+1} (tag u + 2); its sweep also waits until slot
// (u + 1) % kR is free.  Waits
// also end when the launch has stopped (DEC finished or a role failed).
template <bool TRACE>
__device__ __forceinline__ void upd_wave(const CvArgs& a, int g, int w, const f4v* qs, float* ysb, int ny, u64* hs) {
    const int N = a.N;
    const int lane = threadIdx.x & 63, ll = lane & (kL - 1);
    const int p = g * kL + ll;  // row side 2i + side
    const bool live = lane < kL && p < 2 * N;
    const int row = p >> 1;
    const int KB = split_kblocks(N), W = waves_of(KB);
    const int pk0 = slice0_of(w), pk1 = slice0_of(w + 1);
    const int k0 = 4 * pk0, k1 = 4 * pk1 < N ? 4 * pk1 : N;
    const bool last = (w == W - 1);
    const float fd = live ? a.fdpn[p] : 0.0f;
    const bool tr = TRACE && a.trace && g == 0 && lane == 0;
    float yrow = 0.0f;
    int bad = 0;  // a hand-off wait that ended without the sums: 1 stopped, 2 timed out
    for (long long u = a.u0; u < a.u_prod_end; ++u) {
        const int par = (int)(u & 1);
        float* ys = ysb + par * ny;
        const unsigned tag = (unsigned)(u + 1);
        const int rslot = (int)(u & (kR - 1));
        mark<TRACE>(a, tr, u, w, 0);
        // the last wave publishes y_{u+1} into slot (u + 1) % kR: free once DEC
        // has decided u + 1 - kR.  Its sweep waits for that too (one more load
        // in the same loop: off the critical path, since the last wave waits
        // for its turn long after it has staged, and no loop of its own, which
        // made the in-place products spill)
        const bool need_bp = !PQP_CV_NOBP && last && u + 1 - kR >= a.u0;
        // ---- 1. y of this slice from the ring: every load in flight, one
        // wave-wide tag test, the exit straight into the LDS stores ----
        auto stage_y = [&]() -> bool {
            const gu64* gsrc = (const gu64*)a.ry + (size_t)rslot * N;
            int ln = lane;
            asm volatile("" : "+v"(ln));
            int kk[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) kk[m] = (k0 + 64 * m + ln < k1) ? k0 + 64 * m + ln : k1 - 1;
            const int rowc = row < N ? row : N - 1;
            u64 x[4], xo = 0;
            Deadline dl;
            unsigned spins = 0;
            bool ok;
#pragma clang loop unroll(disable)
            do {
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    x[m] = __hip_atomic_load(gsrc + kk[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (last) xo = __hip_atomic_load(gsrc + rowc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                long long dv = 0;
                if (need_bp) dv = __hip_atomic_load(a.decided, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = !need_bp || dv >= u + 1 - kR;
#pragma unroll
                for (int m = 0; m < 4; ++m) ok &= (unsigned)(x[m] >> 32) == tag;
                if (last) ok &= (unsigned)(xo >> 32) == tag;
                ok = __all(ok);
                if (!ok) {
                    if ((++spins & 63) == 0) {
                        if (stopped(a)) return false;
                        if (dl.expired()) {
                            fail(a, 1);
                            return false;
                        }
                    }
                    if (w == 0) {
                        if (PQP_CV_SLEEP0 > 0) __builtin_amdgcn_s_sleep(PQP_CV_SLEEP0);
                    } else if (w == 1) {
                        __builtin_amdgcn_s_sleep(PQP_CV_SLEEP1);
                    } else {
                        __builtin_amdgcn_s_sleep(PQP_CV_SLEEPN);
                    }
                }
            } while (!ok);
#pragma unroll
            for (int m = 0; m < 4; ++m) ys[kk[m]] = __uint_as_float((unsigned)x[m]);
            if (last) yrow = __uint_as_float((unsigned)xo);
            mark<TRACE>(a, tr, u, w, 1);
            return true;
        };
        const f4v* qw = qs + (size_t)pk0 * kL + ll;
        const f4v* yw = reinterpret_cast<const f4v*>(ys) + pk0;
        u64* sl = hs + (size_t)par * W * 64;
        // the wave's sums done: hand them on, or (last wave) finish the rows
        auto finish = [&](float acc) -> bool {
            asm volatile("" : "+v"(acc));
            mark<TRACE>(a, tr, u, w, 3);
            if (!last) {
                // (after a failed wait the next wave gets a tagged word too: it
                // stops at its next sweep)
                __hip_atomic_store(sl + w * 64 + lane, granule(tag, acc), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                __builtin_amdgcn_s_setprio(0);
                if (bad) {
                    if (bad == 2) fail(a, 10);
                    return false;
                }
                return true;
            }
            __builtin_amdgcn_s_setprio(0);
            if (bad) {
                if (bad == 2) fail(a, 10);
                return false;
            }
            const float v = acc + 1.0f * fd;  // even lane: num (:611), odd lane: den (:612)
            // the partner lane's sum by a DPP swap of lane pairs (quad_perm 1,0,3,2)
            const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
            const float yn = v / den * yrow;  // updY :594
            if (!(p & 1) && live)
                __hip_atomic_store((gu64*)a.ry + (size_t)((u + 1) & (kR - 1)) * N + row, granule(tag + 1, yn),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return true;
        };
        if (w == 0) {
            // wave 0 reads its slice's split entries while it waits for y
            f4v q0[kP0];
#pragma unroll
            for (int j = 0; j < kP0; ++j) q0[j] = qw[j * kL];
            if (!stage_y()) return;
            mark<TRACE>(a, tr, u, w, 2);
            __builtin_amdgcn_s_setprio(3);
            if (!finish(chain_qreg(0.0f, q0, yw))) return;
        } else {
            auto turn = [&](auto np) -> int {
                constexpr int NP = decltype(np)::value;
                f4v prod[NP];
                // the slice's split entries, read while the wave waits for y
#if PQP_CV_UPD_INPLACE
#pragma unroll
                for (int j = 0; j < NP; ++j) prod[j] = qw[j * kL];
#endif
                if (!stage_y()) return 1;
                if (w >= 4) {
                    // waves 4, 5 share SIMDs with waves 0, 1: their products
                    // start once wave kLateGate has handed on its sums
                    Deadline dl;
                    for (unsigned spins = 0;; ++spins) {
                        const u64 h = __hip_atomic_load(sl + kLateGate * 64 + lane, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (__all((unsigned)(h >> 32) == tag)) break;
                        if ((spins & 255) == 255) {
                            if (stopped(a)) return 1;
                            if (dl.expired()) return 2;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
#if PQP_CV_UPD_INPLACE
                slice_products_inplace(prod, yw);
#else
                slice_products(prod, qw, yw);
#endif
#pragma unroll
                for (int j = 0; j < NP; ++j) asm volatile("" : "+v"(prod[j]));
                u64 h;
                bad = wait_sums(a, sl + (w - 1) * 64 + lane, tag, h);
                float acc = __uint_as_float((unsigned)h);
                mark<TRACE>(a, tr, u, w, 2);
                __builtin_amdgcn_s_setprio(3);
#pragma unroll
                for (int j = 0; j < NP; ++j) {
                    acc += prod[j].x;  // :608-609, k in order
                    acc += prod[j].y;
                    acc += prod[j].z;
                    acc += prod[j].w;
                }
                return finish(acc) ? 0 : 3;
            };
            const int rc = (w == 1) ? turn(std::integral_constant<int, kP1>{}) : turn(std::integral_constant<int, kPW>{});
            if (rc == 2) fail(a, 10);
            if (rc) return;
        }
    }
}

// One wave of a terminate() chain role (T1, T2, T3): iterates [ub, ue].  (Its
// UPD branches are the update's earlier form; UPD now runs upd_wave.)
template <int ROLE_T, bool TRACE>
__device__ __forceinline__ void chain_wave(const CvArgs& a, int g, int w, int K, const f4v* qs, float* ysb, int ny,
                                           u64* hs) {
    constexpr int ROLE = ROLE_T;
    const int N = a.N, M = a.M;
    const int lane = threadIdx.x & 63, ll = lane & (kL - 1);
    const int c = g * kL + ll;  // output column (UPD: row side p = 2i + side)
    const int KB = split_kblocks(K), W = waves_of(KB);
    const int pk0 = slice0_of(w);
    const int pk1 = slice0_of(w + 1);
    const int k0 = 4 * pk0 < K ? 4 * pk0 : K, k1 = 4 * pk1 < K ? 4 * pk1 : K;
    const bool last = (w == W - 1);
    const u64* rx = (ROLE == kUpd || ROLE == kT1) ? a.ry : (ROLE == kT2 ? a.rtmp : a.rU);
    const int nx = (ROLE == kUpd || ROLE == kT1) ? N : M;  // ring row length of x (= K)
    // epilogue constants
    const int row = c >> 1;
    const bool upd_live = lane < kL && c < 2 * N;
    float cst = 0.0f;
    if (ROLE == kUpd && upd_live) cst = a.fdpn[c];
    if (ROLE == kT1 && lane < kL && c < M) cst = a.Fp[c];
    if (ROLE == kT3 && lane < kL && c < N) cst = a.Kp[c];
    const long long ub = a.u0;
    const long long ue = ROLE == kUpd ? a.u_prod_end - 1 : a.u_dec_end;
    float yrow = 0.0f;
    const bool tr = TRACE && a.trace && g == 0 && lane == 0;
    const int tid_ = ROLE * kMaxW + w;
    int bad = 0;  // a hand-off wait that ended without the sums (wait_sums' code), acted on after the chain
    for (long long u = ub; u <= ue; ++u) {
        const unsigned tag = (unsigned)(u + 1);
        const int slot = (int)(u & (kR - 1));
        float* ys = ysb + (int)(u & 1) * ny;
        mark<TRACE>(a, tr, u, tid_, 0);
        // UPD's last wave: the slot y_{u+1} goes to must be free (issued early, tested after the chain)
        long long dec_seen = 0;
        const bool need_bp = ROLE == kUpd && last && u + 1 - kR >= a.u0;
        if (need_bp) dec_seen = __hip_atomic_load(a.decided, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // ---- 1. x of this slice, staged in LDS (run inside each wave's own
        // branch below, so that wave 0's registered q does not stay live
        // across the other branch) ----
        auto stage_x = [&]() -> bool {
            // the slice's granules, 4 per lane with indices clamped into the
            // slice (a duplicate re-reads its last granule), + y_i for UPD's last
            // wave: every load unconditional, and the stores too (a duplicate
            // stores the same value to the same word); x past K is +0 from the
            // launch's start
            const gu64* gx = (const gu64*)rx + (size_t)slot * nx;
            int ln = lane;
            asm volatile("" : "+v"(ln));  // keeps the indices out of the registers held across iterates
            const gu64* gp[5];
            bool on[5];
            float v[5] = {};
            int kk[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                kk[m] = (k0 + 64 * m + ln < k1) ? k0 + 64 * m + ln : k1 - 1;
                gp[m] = gx + kk[m];
                on[m] = true;
            }
            const bool own = ROLE == kUpd && last;  // y_i for y_next = num/den*y_i (:594)
            gp[4] = gx + (row < N ? row : N - 1);
            on[4] = own;
            // the terminate() roles poll more slowly than the update (off its
            // critical path; fewer polls of the lines the update waits on)
            if (!await_granules<5, ROLE == kUpd ? 1 : kTPollSleep>(a, gp, on, tag, v, 1 + ROLE)) return false;
#pragma unroll
            for (int m = 0; m < 4; ++m) ys[kk[m]] = v[m];
            if (own) yrow = v[4];
            mark<TRACE>(a, tr, u, tid_, 1);
            return true;
        };
        const f4v* qw = qs + (size_t)pk0 * kL + ll;
        const f4v* yw = reinterpret_cast<const f4v*>(ys) + pk0;
        float acc = 0.0f;
        if (w == 0) {
            // wave 0 reads its slice's q while it waits for x
            f4v q0[kP0];
#pragma unroll
            for (int j = 0; j < kP0; ++j) q0[j] = qw[j * kL];
            if (!stage_x()) return;
            // ---- 2/3 (wave 0): the chain starts here, products formed inside it ----
            __builtin_amdgcn_s_setprio(3);
            acc = chain_qreg(acc, q0, yw);
        } else {
            if (!stage_x()) return;
            // ---- 2. products of the slice, ahead of the turn; 3. the running
            // sums of the previous slice, then this slice's adds ----
            auto turn = [&](auto np) -> int {
                constexpr int NP = decltype(np)::value;
                f4v prod[NP];
                if (w >= 4) {
                    // waves 4, 5 share SIMDs with waves 0, 1: their products
                    // start once wave kLateGate has handed on its sums
                    const u64* gsrc = hs + ((size_t)slot * kMaxW + kLateGate) * kL + ll;
                    Deadline dl;
                    for (unsigned spins = 0;; ++spins) {
                        const u64 h = __hip_atomic_load(gsrc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (__all((unsigned)(h >> 32) == tag)) break;
                        if ((spins & 255) == 255) {
                            if (stopped(a)) return 1;
                            if (dl.expired()) return 2;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                slice_products(prod, qw, yw);
#pragma unroll
                for (int j = 0; j < NP; ++j) asm volatile("" : "+v"(prod[j]));
                u64 h;
                bad = wait_sums(a, hs + ((size_t)slot * kMaxW + (w - 1)) * kL + ll, tag, h);
                acc = __uint_as_float((unsigned)h);
                mark<TRACE>(a, tr, u, tid_, 2);
                __builtin_amdgcn_s_setprio(3);
#pragma unroll
                for (int j = 0; j < NP; ++j) {
                    acc += prod[j].x;
                    acc += prod[j].y;
                    acc += prod[j].z;
                    acc += prod[j].w;
                }
                return 0;
            };
            const int rc = (w == 1) ? turn(std::integral_constant<int, kP1>{}) : turn(std::integral_constant<int, kPW>{});
            if (rc == 2) fail(a, 10 + ROLE);
            if (rc) return;
        }
        asm volatile("" : "+v"(acc));
        mark<TRACE>(a, tr, u, tid_, 3);
        if (!last) {
            // (after a failed wait the next wave gets a tagged word too: it
            // stops at its next sweep)
            if (lane < kL)
                __hip_atomic_store(hs + ((size_t)slot * kMaxW + w) * kL + ll, granule(tag, acc), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            __builtin_amdgcn_s_setprio(0);
            if (bad) {
                if (bad == 2) fail(a, 10 + ROLE);
                return;
            }
            continue;
        }
        __builtin_amdgcn_s_setprio(0);
        if (bad) {  // the last wave publishes nothing after a failed wait
            if (bad == 2) fail(a, 10 + ROLE);
            return;
        }
        // ---- 4. the last wave's epilogue ----
        if (ROLE == kUpd) {
            const float v = acc + 1.0f * cst;    // even lane: num (:611), odd lane: den (:612)
            // the partner lane's sum by a DPP swap of lane pairs (quad_perm 1,0,3,2)
            const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
            if (need_bp && dec_seen < u + 1 - kR) {
                Deadline dl;
                for (unsigned spins = 0;; ++spins) {
                    __builtin_amdgcn_s_sleep(2);
                    if (__hip_atomic_load(a.decided, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= u + 1 - kR)
                        break;
                    if (stopped(a)) return;
                    if ((spins & 63) == 63 && dl.expired()) {
                        fail(a, 20);
                        return;
                    }
                }
            }
            if (!(c & 1) && upd_live) {
                const float yn = v / den * yrow;  // updY :594
                __hip_atomic_store((gu64*)a.ry + (size_t)((u + 1) & (kR - 1)) * N + row, granule(tag + 1, yn),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            mark<TRACE>(a, tr, u, tid_, 3);  // the last wave's "done" is the publication of y_{u+1}
        } else if (ROLE == kT1) {
            if (lane < kL && c < M)  // matrixAdd(tmp, Fp, 1) :356
                __hip_atomic_store((gu64*)a.rtmp + (size_t)slot * M + c, granule(tag, acc + 1.0f * cst),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (lane < kL && c < M + N)  // Y'Qd (computeCost :652)
                __hip_atomic_store((gu64*)a.rtq + (size_t)slot * N + (c - M), granule(tag, acc), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else if (ROLE == kT2) {
            if (lane < kL && c < M)  // U = -U :358
                __hip_atomic_store((gu64*)a.rU + (size_t)slot * M + c, granule(tag, -acc), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {  // kT3
            // compare :334-343 (erc * Kp in double, rounded to float by max())
            const bool bad = lane < kL && c < N && acc > cst + max_ref((float)(kTol * cst), (float)kTol);
            if (lane < kL && c >= N && c < N + M)  // U'Qp (computeCost, Jp)
                __hip_atomic_store((gu64*)a.rtu + (size_t)slot * M + (c - N), granule(tag, acc), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            const bool any_bad = __any(bad);
            if (lane == 0)
                __hip_atomic_store((gu64*)a.rfeas + (size_t)slot * (a.g4 - a.g3) + g,
                                   granule(tag, any_bad ? 1.0f : 0.0f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Copy a ring row (every granule already carries `tag`) to a plain vector.
__device__ bool ring_copy(const CvArgs& a, const u64* ring, int n, int slot, unsigned tag, float* out) {
    const int lane = threadIdx.x & 63;
    for (int k0 = 0; k0 < n; k0 += 64) {
        const int k = k0 + lane;
        const gu64* gp[1] = {(const gu64*)ring + (size_t)slot * n + (k < n ? k : 0)};
        const bool on[1] = {k < n};
        float v[1];
        if (!await_granules<1>(a, gp, on, tag, v, 30)) return false;
        if (k < n) out[k] = v[0];
    }
    return true;
}

// DEC's dot waves (computeCost :648-666, k in order on every lane alike,
// broadcast LDS reads of the products; each dot handed to wave 0 through an
// LDS word).  ND = 1: dot `dot0` (1: Fd.Y, 4: (Y'Qd).Y; N terms) of every
// ustep-th iterate from ustart -- two waves per dot take the even and the odd
// iterates, so each has two periods for its gather and its N-long sum.  ND = 2:
// dots 2 ((U'Qp).U) and 3 (Fp.U), one U stream, their two M-long chains side
// by side -- also on two waves, the even and the odd iterates (one wave for
// both parities was the bound of an all-feasible solve).
template <int ND, bool TRACE>
__device__ __forceinline__ void dec_dots(const CvArgs& a, int d, int dot0, float* pr0, float* pr1, long long ustart,
                                         int ustep, u64* dres) {
    const int N = a.N, M = a.M;
    const int lane = threadIdx.x & 63;
    const bool tr = TRACE && a.trace && lane == 0;
    const int n = (dot0 == 1 || dot0 == 4) ? N : M;
    const int nc = kDecChunk * cdiv_i(n, kDecChunk);
    const u64* ra = dot0 == 4 ? a.rtq : (dot0 == 2 ? a.rtu : nullptr);  // ring operand (or the constant below)
    const float* fa = ND == 2 ? a.Fp : (dot0 == 1 ? a.Fd : nullptr);   // ND = 2: dot 3's Fp
    const u64* rb = (dot0 == 1 || dot0 == 4) ? a.ry : a.rU;
    for (int k = n + lane; k < nc + 32; k += 64) {  // +0 tail: adds nothing to a sum that is never -0
        pr0[k] = 0.0f;
        if (ND == 2) pr1[k] = 0.0f;
    }
    float fav[kDecPer];  // the constant operand (Fd, Fp), loaded once
#pragma unroll
    for (int m = 0; m < kDecPer; ++m) {
        const int k = 64 * m + lane;
        fav[m] = (fa && k < n) ? fa[k] : 0.0f;
    }
    // the granules of iterate uu, every load in flight (unused lanes re-read
    // element 0); the next iterate's are issued before this iterate's sum
    u64 x[2 * kDecPer];
    // ND = 2 also reads T3's feasibility words of the iterate (one per lane,
    // G3 <= 64): computeCost runs only on a feasible iterate (terminate :677),
    // so the two sums are skipped on an infeasible one (wave 0 ignores them)
    const int G3 = a.g4 - a.g3;
    u64 xf = 0;
    auto issue = [&](long long uu) {
        const int sl = (int)(uu & (kR - 1));
        if (ND == 2)
            xf = __hip_atomic_load((const gu64*)a.rfeas + (size_t)sl * G3 + (lane < G3 ? lane : 0), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        const gu64* gb = (const gu64*)rb + (size_t)sl * n;
        const gu64* ga = (const gu64*)(ra ? ra : rb) + (size_t)sl * n;
#pragma unroll
        for (int m = 0; m < kDecPer; ++m) {
            const int k = 64 * m + lane;
            x[m] = __hip_atomic_load(gb + (k < n ? k : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (ra) {
#pragma unroll
            for (int m = 0; m < kDecPer; ++m) {
                const int k = 64 * m + lane;
                x[kDecPer + m] = __hip_atomic_load(ga + (k < n ? k : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    };
    if (ustart <= a.u_dec_end) issue(ustart);
    for (long long u = ustart; u <= a.u_dec_end; u += ustep) {
        const unsigned tag = (unsigned)(u + 1);
        const int slot = (int)(u & (kR - 1));
        mark<TRACE>(a, tr, u, 4 * kMaxW + d, 0);
        // products into LDS once every granule of the lane carries the tag
        {
            Deadline dl;
            for (unsigned spins = 0;; ++spins) {
                bool ok = true;
#pragma unroll
                for (int m = 0; m < kDecPer; ++m) {
                    const bool in = 64 * m + lane < n;
                    ok &= !in || (unsigned)(x[m] >> 32) == tag;
                    if (ra) ok &= !in || (unsigned)(x[kDecPer + m] >> 32) == tag;
                }
                if (ND == 2) ok &= lane >= G3 || (unsigned)(xf >> 32) == tag;
                if (__all(ok)) break;
                if ((spins & 63) == 63) {
                    if (stopped(a)) return;
                    if (dl.expired()) {
                        fail(a, 40 + d);
                        return;
                    }
                }
                __builtin_amdgcn_s_sleep(kTPollSleep);
                issue(u);
            }
#pragma unroll
            for (int m = 0; m < kDecPer; ++m) {
                const int k = 64 * m + lane;
                const float vb = __uint_as_float((unsigned)x[m]);
                if (k < n) {
                    if (ND == 2) {
                        pr0[k] = __uint_as_float((unsigned)x[kDecPer + m]) * vb;  // (U'Qp)[k] * U[k]
                        pr1[k] = fav[m] * vb;                                     // Fp[k] * U[k]
                    } else {
                        pr0[k] = (ra ? __uint_as_float((unsigned)x[kDecPer + m]) : fav[m]) * vb;
                    }
                }
            }
        }
        const bool skip = ND == 2 && __any(lane < G3 && __uint_as_float((unsigned)xf) != 0.0f);  // infeasible
        if (u + ustep <= a.u_dec_end) issue(u + ustep);
        mark<TRACE>(a, tr, u, 4 * kMaxW + d, 1);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // :652-657, k in order.  Chunks of kDecChunk terms, each fully unrolled
        // (a loop back-edge waits for every read in flight); the reads run
        // kDecAhead groups of 16 ahead of the adds.
        float acc0 = 0.0f, acc1 = 0.0f;
        const f4v* p0 = reinterpret_cast<const f4v*>(pr0);
        const f4v* p1 = reinterpret_cast<const f4v*>(pr1);
        constexpr int AH = ND == 2 ? 2 : kDecAhead;  // two chains: fewer groups ahead (registers)
        for (int c4 = 0; c4 < (skip ? 0 : nc / 4); c4 += kDecChunk / 4) {
            f4v R[AH + 1][4];
            f4v S[ND == 2 ? AH + 1 : 1][4];
#pragma unroll
            for (int g0 = 0; g0 < AH; ++g0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    R[g0][j] = p0[c4 + 4 * g0 + j];
                    if constexpr (ND == 2) S[g0][j] = p1[c4 + 4 * g0 + j];
                }
            }
#pragma unroll
            for (int gi = 0; gi < kDecChunk / 16; ++gi) {
                if (gi + AH < kDecChunk / 16) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        R[(gi + AH) % (AH + 1)][j] = p0[c4 + 4 * (gi + AH) + j];
                        if constexpr (ND == 2) S[(gi + AH) % (AH + 1)][j] = p1[c4 + 4 * (gi + AH) + j];
                    }
                }
                asm volatile("" : "+v"(acc0), "+v"(acc1)::"memory");  // the reads issue before the adds
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f4v r = R[gi % (AH + 1)][j];
                    acc0 += r.x;
                    if constexpr (ND == 2) acc1 += S[gi % (AH + 1)][j].x;
                    acc0 += r.y;
                    if constexpr (ND == 2) acc1 += S[gi % (AH + 1)][j].y;
                    acc0 += r.z;
                    if constexpr (ND == 2) acc1 += S[gi % (AH + 1)][j].z;
                    acc0 += r.w;
                    if constexpr (ND == 2) acc1 += S[gi % (AH + 1)][j].w;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        mark<TRACE>(a, tr, u, 4 * kMaxW + d, 2);
        if (lane == 0) {
            __hip_atomic_store(dres + (size_t)slot * kDecW + dot0, granule(tag, acc0), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
            if (ND == 2)
                __hip_atomic_store(dres + (size_t)slot * kDecW + 3, granule(tag, acc1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// DEC: wave 0 gathers the feasibility words of T3, receives the four dots
// from waves 1-6 (dec_dots) and decides (terminate :673-687, loop control
// :716-724), so the decision of iterate u overlaps the dots of u + 1.
template <bool TRACE>
__device__ void decide_role(const CvArgs& a, float* lds) {
    const int N = a.N, M = a.M;
    const int lane = threadIdx.x & 63, d = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nmax = kDecChunk * cdiv_i(N > M ? N : M, kDecChunk);
    float* prb = lds;  // [kDecBufs][nmax + 32] products (+ 32: prefetch past the end)
    u64* dres = reinterpret_cast<u64*>(lds + (size_t)kDecBufs * (nmax + 32));  // [kR][kDecW] hand-off words
    for (int e = threadIdx.x; e < kR * kDecW; e += blockDim.x) dres[e] = 0ull;
    __syncthreads();
    if (d >= kDecW) return;
    if (PQP_CV_DIAG && d != 0) return;
    const bool tr = TRACE && a.trace && lane == 0;
    if (d == 0) {
        SolveState* st = a.st;
        float Jp = st->Jp, Jd = st->Jd;
        int have = st->have_costs;
        const float Md = a.Md[0], Mp = a.Mp[0];
        const int G3 = a.g4 - a.g3;
        for (long long u = a.u0; u <= a.u_dec_end; ++u) {
            const unsigned tag = (unsigned)(u + 1);
            const int slot = (int)(u & (kR - 1));
            mark<TRACE>(a, tr, u, 4 * kMaxW, 0);
            bool bad = PQP_CV_DIAG != 0;  // checkFeas (:677): any T3 workgroup with a row over its bound
            for (int k0 = 0; k0 < (PQP_CV_DIAG ? 0 : G3); k0 += 64) {
                const int k = k0 + lane;
                const gu64* gp[1] = {(const gu64*)a.rfeas + (size_t)slot * G3 + (k < G3 ? k : 0)};
                const bool on[1] = {k < G3};
                float v[1] = {0.0f};
                if (!await_granules<1>(a, gp, on, tag, v, 50)) return;
                bad |= k < G3 && v[0] != 0.0f;
            }
            const bool feasible = !__any(bad);
            mark<TRACE>(a, tr, u, 4 * kMaxW, 1);
            float s1 = 0.0f, s2 = 0.0f, s3 = 0.0f, s4 = 0.0f;
            if (!PQP_CV_DIAG) {
                Deadline dl;
                u64 h = 0;
                const bool mine = lane >= 1 && lane <= kDots;
                for (unsigned spins = 0;; ++spins) {
                    if (mine)
                        h = __hip_atomic_load(dres + (size_t)slot * kDecW + lane, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (__all(!mine || (unsigned)(h >> 32) == tag)) break;
                    if ((spins & 255) == 255) {
                        if (stopped(a)) return;
                        if (dl.expired()) {
                            fail(a, 51);
                            return;
                        }
                    }
                }
                const float hv = __uint_as_float((unsigned)h);
                s1 = __shfl(hv, 1);
                s2 = __shfl(hv, 2);
                s3 = __shfl(hv, 3);
                s4 = __shfl(hv, 4);
            }
            mark<TRACE>(a, tr, u, 4 * kMaxW, 2);
            int stop = 0;
            if (feasible) {
                Jd = 0.0f;  // computeCost :648-666 (J += 0.5 * tmp[0] in double)
                Jd = (float)((double)Jd + 0.5 * (double)s4);
                Jd += s1;
                Jd += Md / 2;
                Jp = 0.0f;
                Jp = (float)((double)Jp + 0.5 * (double)s2);
                Jp += s3;
                Jp += Mp / 2;
                have = 1;
                stop = gap_stop(Jp, Jd) ? 1 : 0;  // the three gap tests :681-685
            }
            const bool capped = a.cap > 0 && u >= a.cap;
            if (stop || capped || u == a.u_dec_end) {
                // finished (y_u, U_u) or the end of this launch's chunk (y_{u+1}, U_u)
                const bool fin = stop || capped;
                if (!ring_copy(a, a.ry, N, (int)((fin ? u : u + 1) & (kR - 1)), fin ? tag : tag + 1, a.Yout))
                    return;
                if (!PQP_CV_DIAG && !ring_copy(a, a.rU, M, slot, tag, a.Uout)) return;
                if (lane == 0) {
                    st->h = fin ? u + 1 : u + 2;
                    st->status = stop ? kStatusDone : (capped ? kStatusCapped : kStatusContinue);
                    st->Jp = Jp;
                    st->Jd = Jd;
                    st->have_costs = have;
                    __hip_atomic_store(a.ctl, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                }
                return;
            }
            if (lane == 0) __hip_atomic_store(a.decided, u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            mark<TRACE>(a, tr, u, 4 * kMaxW, 3);
        }
        return;
    }
    // ---- waves 1..6: the dots, each on two parity waves ----
    auto buf = [&](int i) { return prb + (size_t)i * (nmax + 32); };
    const long long ue = a.u0 + ((a.u0 & 1) ? 1 : 0);  // first even iterate
    const long long uo = a.u0 + ((a.u0 & 1) ? 0 : 1);  // first odd iterate
    switch (d) {
        case 1: dec_dots<1, TRACE>(a, d, 1, buf(0), nullptr, ue, 2, dres); break;
        case 2: dec_dots<1, TRACE>(a, d, 1, buf(1), nullptr, uo, 2, dres); break;
        case 3: dec_dots<1, TRACE>(a, d, 4, buf(2), nullptr, ue, 2, dres); break;
        case 4: dec_dots<1, TRACE>(a, d, 4, buf(3), nullptr, uo, 2, dres); break;
        case 5: dec_dots<2, TRACE>(a, d, 2, buf(4), buf(5), ue, 2, dres); break;
        default: dec_dots<2, TRACE>(a, d, 2, buf(6), buf(7), uo, 2, dres); break;
    }
}

// TRACE: the timeline instantiation (pqp_tune_trace("converge", ...)); the default one
// carries no trace branches.
template <bool TRACE>
__global__ void __launch_bounds__(64 * kMaxW, 1) k_converge_persist(CvArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    int b = blockIdx.x;
    const int tid = threadIdx.x;
    if (a.xcds > 0) {  // packed onto a.xcds XCDs (round-robin placement): the rest leave at once
        if ((b & 7) >= a.xcds) return;
        b = (b >> 3) * a.xcds + (b & 7);
        if (b > a.g4) return;  // past the G = g4 + 1 workgroups (G not a multiple of xcds)
    }
    if (b == a.stall_wg) return;  // as if not resident: the other roles' waits expire into err
    if (b >= a.g4) {
        decide_role<TRACE>(a, lds);
        return;
    }
    const int role = b < a.g1 ? kUpd : (b < a.g2 ? kT1 : (b < a.g3 ? kT2 : kT3));
    if (PQP_CV_DIAG && PQP_CV_DIAG != 3 && role != kUpd && !(PQP_CV_DIAG == 2 && role == kT1)) return;
    const int g = b - (role == kUpd ? 0 : role == kT1 ? a.g1 : role == kT2 ? a.g2 : a.g3);
    const int K = (role == kUpd || role == kT1) ? a.N : a.M;
    const f4v* src = role == kUpd ? a.SPu : role == kT1 ? a.A1 : role == kT2 ? a.A2 : a.A3;
    const int KB = split_kblocks(K), W = waves_of(KB), KP = packets_of(W);
    const int Kmax = a.N > a.M ? a.N : a.M, KPmax = packets_of(waves_of(split_kblocks(Kmax)));
    f4v* qs = reinterpret_cast<f4v*>(lds);                 // [KP][32] this workgroup's packets
    float* ysb = lds + (size_t)KPmax * kL * 4;             // [2][4 KPmax] x by iterate parity
    u64* hs = reinterpret_cast<u64*>(ysb + 2 * KPmax * 4);  // [kR][kMaxW][32] hand-off words
    {
        const f4v* s = src + (size_t)g * KB * kL;
        for (int e = tid; e < KP * kL; e += blockDim.x) qs[e] = (e < KB * kL) ? s[e] : f4v{0.0f, 0.0f, 0.0f, 0.0f};
        for (int e = tid; e < kR * kMaxW * kL; e += blockDim.x) hs[e] = 0ull;
        // x past K (read by the last packet's products) stays +0: zeroed once in
        // both parity buffers
        for (int e = tid; e < 2 * (KPmax * 4 - K); e += blockDim.x) ysb[(e & 1) * KPmax * 4 + K + (e >> 1)] = 0.0f;
    }
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (w >= W) return;
    const int ny = KPmax * 4;
    if (role == kUpd) {  // k_split_persist's update form
        upd_wave<TRACE>(a, g, w, qs, ysb, ny, hs);
        return;
    }
    switch (role) {
        case kT1: chain_wave<kT1, TRACE>(a, g, w, K, qs, ysb, ny, hs); break;
        case kT2: chain_wave<kT2, TRACE>(a, g, w, K, qs, ysb, ny, hs); break;
        default: chain_wave<kT3, TRACE>(a, g, w, K, qs, ysb, ny, hs); break;
    }
}

// packets of stage columns [col0, col0 + ncols): column j of the job is
// A[k][j] = trans ? src[j * ld + k] : src[k * ld + j], k < K (+0 beyond)
__global__ void __launch_bounds__(256) k_pack_cols(const float* __restrict__ src, int ld, int trans, int K,
                                                   int ncols, int col0, int KB, f4v* __restrict__ dst) {
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;  // (kb, j), j fastest
    if (e >= (long long)KB * ncols) return;
    const int kb = (int)(e / ncols), j = (int)(e % ncols);
    float v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int k = 4 * kb + t;
        v[t] = k < K ? (trans ? src[(size_t)j * ld + k] : src[(size_t)k * ld + j]) : 0.0f;
    }
    const int c = col0 + j;
    dst[((size_t)(c / kL) * KB + kb) * kL + (c % kL)] = f4v{v[0], v[1], v[2], v[3]};
}

// ring slot of y_{u0} <- Y, control words for a launch
__global__ void k_converge_init(const float* __restrict__ Y, int N, long long u0, u64* ry, int* ctl,
                                long long* decided, int* err) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = t; k < N; k += gridDim.x * blockDim.x)
        ry[(size_t)(u0 & (kR - 1)) * N + k] = granule((unsigned)(u0 + 1), Y[k]);
    if (t == 0) {
        *ctl = 0;
        *err = 0;
        *decided = u0 - 1;
    }
}

}  // namespace


// Geometry of the launch for (N, M); 0 when it does not apply.
int converge_persist_wgs(int N, int M, int* g) {
    if (N < 1 || M < 1 || N > 1024 || M > 1024) return 0;
    const int g1 = cdiv_i(2 * N, kL);
    const int g2 = g1 + cdiv_i(N + M, kL);
    const int g3 = g2 + cdiv_i(M, kL);
    const int g4 = g3 + cdiv_i(N + M, kL);
    if (g) {
        g[0] = g1;
        g[1] = g2;
        g[2] = g3;
        g[3] = g4;
    }
    return g4 + 1;
}

size_t converge_persist_lds_bytes(int N, int M) {
    const int Kmax = N > M ? N : M;
    const int KPmax = packets_of(waves_of(split_kblocks(Kmax)));
    const size_t chain = sizeof(float) * ((size_t)KPmax * kL * 4 + (size_t)2 * KPmax * 4) + sizeof(u64) * kR * kMaxW * kL;
    const size_t dec = sizeof(float) * (size_t)kDecBufs * (kDecChunk * cdiv_i(Kmax, kDecChunk) + 32) +
                       sizeof(u64) * kR * kDecW;
    return chain > dec ? chain : dec;
}

size_t converge_ring_words(int N, int M) {
    int g[4];
    converge_persist_wgs(N, M, g);
    return (size_t)kR * (2 * (size_t)N + 3 * (size_t)M + (size_t)(g[3] - g[2]));
}

size_t converge_stage_floats(int N, int M, int stage) {
    int g[4];
    converge_persist_wgs(N, M, g);
    const int KBn = split_kblocks(N), KBm = split_kblocks(M);
    switch (stage) {
        case 1: return (size_t)(g[1] - g[0]) * KBn * kL * 4;
        case 2: return (size_t)(g[2] - g[1]) * KBm * kL * 4;
        default: return (size_t)(g[3] - g[2]) * KBm * kL * 4;
    }
}

// Build the three stage packet arrays (buffers zeroed by the caller).
hipError_t launch_converge_pack(const float* Qd, const float* Gp, const float* Qinv, const float* Qp, int N, int M,
                                float* A1, float* A2, float* A3, hipStream_t s) {
    const int KBn = split_kblocks(N), KBm = split_kblocks(M);
    auto pack = [&](const float* src, int ld, int trans, int K, int KB, int ncols, int col0, float* dst) {
        const long long n = (long long)KB * ncols;
        hipLaunchKernelGGL(k_pack_cols, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, ld, trans, K, ncols,
                           col0, KB, reinterpret_cast<f4v*>(dst));
    };
    pack(Gp, M, 0, N, KBn, M, 0, A1);       // tmp = Gp'Y   (:354): A[k][j] = Gp[k][j]
    pack(Qd, N, 0, N, KBn, N, M, A1);       // Y'Qd         (:652): A[k][j] = Qd[k][j]
    pack(Qinv, M, 1, M, KBm, M, 0, A2);     // Qp_inv tmp   (:357): A[k][i] = Qp_inv[i][k]
    pack(Gp, M, 1, M, KBm, N, 0, A3);       // Gp U         (:636): A[k][i] = Gp[i][k]
    pack(Qp, M, 0, M, KBm, M, N, A3);       // U'Qp         (:652): A[k][j] = Qp[k][j]
    return hipGetLastError();
}

// Workgroups of k_converge_persist one CU can hold at once (LDS-bound: 1),
// for the residency check of the host (converge_persist_fits).
int converge_persist_per_cu(int N, int M) {
    const int W = waves_of(split_kblocks(N > M ? N : M));
    const int threads = 64 * (W > kDecW ? W : kDecW);
    int per = 0;
    const void* kern = g_tune.converge_trace ? reinterpret_cast<const void*>(&k_converge_persist<true>)
                                        : reinterpret_cast<const void*>(&k_converge_persist<false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, threads, converge_persist_lds_bytes(N, M)) !=
        hipSuccess)
        return 0;
    return per;
}

hipError_t launch_converge_persist(const ConvergeLaunch& L, hipStream_t s) {
    int g[4];
    const int G = converge_persist_wgs(L.N, L.M, g);
    if (G == 0) return hipErrorInvalidValue;
    u64* ring = static_cast<u64*>(L.rings);
    CvArgs a{};
    a.N = L.N;
    a.M = L.M;
    a.g1 = g[0];
    a.g2 = g[1];
    a.g3 = g[2];
    a.g4 = g[3];
    a.u0 = L.u0;
    a.cap = L.cap;
    long long dec_end = L.u0 + L.chunk - 1;
    if (L.cap > 0 && dec_end > L.cap) dec_end = L.cap;
    a.u_dec_end = dec_end;
    a.u_prod_end = (L.cap > 0 && dec_end == L.cap) ? dec_end : dec_end + 1;
    a.SPu = reinterpret_cast<const f4v*>(L.SP);
    a.A1 = reinterpret_cast<const f4v*>(L.A1);
    a.A2 = reinterpret_cast<const f4v*>(L.A2);
    a.A3 = reinterpret_cast<const f4v*>(L.A3);
    a.fdpn = L.fdpn;
    a.Fp = L.Fp;
    a.Kp = L.Kp;
    a.Fd = L.Fd;
    a.Md = L.Md;
    a.Mp = L.Mp;
    a.ry = ring;
    a.rtmp = a.ry + (size_t)kR * L.N;
    a.rtq = a.rtmp + (size_t)kR * L.M;
    a.rU = a.rtq + (size_t)kR * L.N;
    a.rtu = a.rU + (size_t)kR * L.M;
    a.rfeas = a.rtu + (size_t)kR * L.M;
    a.st = L.st;
    a.ctl = L.ctl;
    a.decided = L.decided;
    a.err = L.err;
    a.Yout = L.Y;
    a.Uout = L.U;
    a.trace = g_tune.converge_trace;
    a.trace_n = g_tune.converge_trace_n;
    a.stall_wg = g_tune.persist_stall_wg;
    // the G workgroups packed onto x XCDs (x * 32 >= G): 6 by default (n_dual
    // 1024, M 512, 177 workgroups: 3.939 -> 3.921 us per iterate against all
    // eight, profiles/r06/converge_xcd_ab_r06n.json); converge_xcds 8 spreads them
    {
        const int want = g_tune.converge_xcds > 0 ? g_tune.converge_xcds : 6;
        a.xcds = (want < 8 && want * 32 >= G) ? want : 0;
    }
    const int grid = a.xcds ? 8 * ((G + a.xcds - 1) / a.xcds) : G;
    hipError_t e = hipMemsetAsync(ring, 0, sizeof(u64) * converge_ring_words(L.N, L.M), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_converge_init, dim3(4), dim3(256), 0, s, L.Y, L.N, L.u0, a.ry, L.ctl, L.decided, L.err);
    const int W = waves_of(split_kblocks(L.N > L.M ? L.N : L.M));
    const int threads = 64 * (W > kDecW ? W : kDecW);
    if (a.trace)
        hipLaunchKernelGGL(k_converge_persist<true>, dim3(grid), dim3(threads), converge_persist_lds_bytes(L.N, L.M),
                           s, a);
    else
        hipLaunchKernelGGL(k_converge_persist<false>, dim3(grid), dim3(threads), converge_persist_lds_bytes(L.N, L.M),
                           s, a);
    return hipGetLastError();
}

}  // namespace pqp
