// pqp_persist.hip -- fixed-iteration mode of ONE problem of n_dual <= 1024
// (BASELINE configs[2]) as ONE persistent launch: every update of the solve
// runs inside the kernel, the split matrices stay in LDS for the whole solve,
// and the iterate moves between workgroups through tagged 8-byte granules in
// global memory instead of through a kernel boundary per update.
//
// What one update is (PQP_CPU.c:603-618, updateY2 over the stored split
// matrices Qdn_theta / Qdp_theta, :524-537):
//   acc_p = sum_{k=0..N-1} S_p[k] * y[k]  (sequential, from +0.0f)
//   num_i = acc_{2i} + 1.0f * Fdn_i ; den_i = acc_{2i+1} + 1.0f * Fdp_i
//   y_next[i] = num_i / den_i * y[i]                             (updY :594)
// with lane p = 2i + side owning row side p (the k_split_relay layout, 32
// row sides per workgroup).  Only the adds form the sequential chain; the
// products are rounded one by one exactly as in the reference (q * y, no FMA).
//
// Geometry: workgroup b owns row sides [32b, 32b + 32) = rows [16b, 16b + 16);
// its W waves split the k range into slices of 24, 36, then 49 packets
// (4 values of k each): wave 1's slice is short so that its products are
// ready when wave 0 hands over (waves 0 and 1 see y at about the same time).
// Per update:
//   1. wave w fetches y[k] of its slice: the initial iterate from Y0, later
//      the granules {tag = update, bits(y)} published by the producing
//      workgroups (agent-scope relaxed 8-byte loads, `global_load_dwordx2 sc1`,
//      repeated until every tag matches -- the data is its own flag);
//   2. forms its slice's products q * y in registers (q from LDS; wave 0
//      reads its q while it waits for y; waves 4 and 5, which share SIMDs
//      with waves 0 and 1, start their products once wave 1 is done);
//   3. waits for wave w-1's running sums (one 64-bit LDS word per lane:
//      tag and sum), adds its products in k order, hands the sums on (wave 0
//      starts the chain as soon as its slice is staged and forms its products
//      inside it);
//   4. the last wave adds Fdn/Fdp, divides, multiplies by y_i and publishes
//      y_next[i] as a granule (`global_store_dwordx2 sc1`); the last update
//      also writes Yout.
// Granules, LDS hand-off words and y slices are double-buffered by update
// parity; the tags make every wait exact (see the hazard notes in
// k_split_persist).  Every wait is bounded in time: a workgroup that never
// gets a slot ends the launch with an error word instead of a hang.
//
// Requirement: all G = ceil(2N / 32) workgroups resident at once (one per CU
// by their LDS; G <= 64 of the 256 CUs).
#include "pqp_device.h"
#include "pqp_launch.h"
#include "pqp_chain.h"

#include <type_traits>

namespace pqp {

namespace {


constexpr int kPLanes = kSliceLanes;  // row sides per workgroup
#ifndef PQP_PERSIST_SLICES  // A/B builds: -DPQP_PERSIST_SLICES=P0,P1,PW
#define PQP_PERSIST_SLICES 24, 36, 49
#endif
constexpr int kSlices[3] = {PQP_PERSIST_SLICES};
constexpr int kPW0 = kSlices[0];  // packets (4 values of k) of wave 0's slice: multiplied inside its add chain
constexpr int kPW1 = kSlices[1];  // packets of wave 1's slice: its products must be ready when wave 0 is done
constexpr int kPW = kSlices[2];   // packets per later slice: their products are formed ahead, in 4 * kPW VGPRs
static_assert(kPW0 + kPW1 + 4 * kPW >= 256, "six waves must cover n_dual 1024");
static_assert(kPW0 <= 64 && kPW1 <= 64 && kPW <= 64, "a slice is at most 4 granules per lane (one sweep)");
constexpr int kLateGate = 1; // waves 4, 5 form their products once this wave has handed on its sums
constexpr int kPMaxWaves = 6;
#ifndef PQP_PS_SLEEP0  // s_sleep units between wave 0's / wave 1's / later waves' y sweeps
#define PQP_PS_SLEEP0 0  // wave 0 (the chain starts on its slice) polls back to back
#endif
#ifndef PQP_PS_SLEEP1
#define PQP_PS_SLEEP1 1
#endif
#ifndef PQP_PS_SLEEPN
#define PQP_PS_SLEEPN 4  // waves 2+ (their turn comes later) poll a quarter as often
#endif


__device__ __forceinline__ void fail(int* err, int code) {
    __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until every lane's 64-bit LDS word carries the tag `want` in its high
// half (a hand-off word of another wave).  `doze`: s_sleep between polls, for
// waits off the critical path.  False when the wait's time limit expired.
__device__ __forceinline__ bool lds_wait(u64* word, unsigned want, bool doze, u64* out = nullptr) {
    Deadline dl;
    for (unsigned spins = 0;; ++spins) {
        const u64 h = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__all((unsigned)(h >> 32) == want)) {
            if (out) *out = h;
            return true;
        }
        if ((spins & 255) == 255 && dl.expired()) return false;
        if (doze) __builtin_amdgcn_s_sleep(1);
    }
}

// The running sums' hand-off wait on the critical path: a bare poll whose
// exit falls through into the adds, bounded by a spin count (each poll is an
// LDS round trip of >= 64 clocks, so 2^25 polls last >= 0.9 s) instead of the
// clock.  False when the bound ran out.
constexpr unsigned kHandoffSpins = 1u << 25;
__device__ __forceinline__ bool lds_wait_sums(u64* word, unsigned want, u64& h) {
    unsigned spins = 0;
#pragma clang loop unroll(disable)
    do {
        h = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } while (!__all((unsigned)(h >> 32) == want) && ++spins < kHandoffSpins);
    return spins < kHandoffSpins;
}




}  // namespace


// waves: slices of kPW0, kPW1, then kPW packets
__host__ __device__ inline int persist_slice0(int w) { return w == 0 ? 0 : (w == 1 ? kPW0 : kPW0 + kPW1 + (w - 2) * kPW); }
__host__ __device__ inline int persist_packets(int W) { return persist_slice0(W); }
__host__ __device__ inline int persist_waves_of(int KB) {
    int W = 1;
    while (persist_packets(W) < KB) ++W;
    return W;
}
int persist_waves(int N) { return persist_waves_of(split_kblocks(N)); }
int persist_max_n() {
    const int n = 4 * persist_packets(kPMaxWaves);
    return n > 1024 ? 1024 : n;
}
// LDS: the workgroup's packets zero-padded to whole slices (so every wave runs
// the same unguarded loops: a +0 packet times y = +0 adds exactly nothing to a
// sum that is never -0), y by update parity, two hand-off words per lane and wave
size_t persist_lds_bytes(int N) {
    const int W = persist_waves(N), KP = persist_packets(W);
    return sizeof(float) * ((size_t)KP * kPLanes * 4 + (size_t)2 * KP * 4) + sizeof(u64) * 2 * W * 64;
}

// SP: the k_build_split layout with lw = 32 (workgroup-major packets).
// gran: 2 * N granules, zeroed before the launch.  err: zeroed before the launch.
// TRACE: the timeline instantiation (pqp_tune_trace("persist", ...)); the default one
// carries no trace branches on its critical path.
template <bool TRACE>
__global__ void __launch_bounds__(64 * kPMaxWaves, 1)
    k_split_persist(const float* __restrict__ SP, const float* __restrict__ fdpn, int N, int updates,
                    const float* __restrict__ Y0, float* __restrict__ Yout, u64* gran_, int* err, u64* trace,
                    int trace_n, int stall_wg, int xcds) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    // xcds > 0 (A/B, tune persist_xcds): the grid is 8 / xcds times larger and
    // only the workgroups with blockIdx % 8 < xcds take part -- under the
    // round-robin placement of workgroups over the 8 XCDs, the solve's
    // workgroups sit on xcds XCDs (32 CUs each) instead of all eight
    int wg = blockIdx.x;
    if (xcds > 0) {
        if ((int)(blockIdx.x & 7) >= xcds) return;
        wg = (int)(blockIdx.x >> 3) * xcds + (int)(blockIdx.x & 7);
        // the padded grid's last row of participants can run past the G
        // workgroups the problem has (G not a multiple of xcds)
        if (wg >= (2 * N + kPLanes - 1) / kPLanes) return;
    }
    // tuning (error-path tests): this workgroup never runs, as if it were not
    // resident; every other one's waits expire and report through err
    if (wg == stall_wg) return;
    gu64* gran = (gu64*)gran_;
    const int KB = split_kblocks(N);
    const int W = persist_waves_of(KB);
    const int KP = persist_packets(W);            // packets incl. the zero padding
    f4v* qs = reinterpret_cast<f4v*>(lds);        // [KP][32] packets of this workgroup
    float* ysb = lds + (size_t)KP * kPLanes * 4;  // [2][4 KP] y by update parity
    u64* slot = reinterpret_cast<u64*>(ysb + 2 * KP * 4);  // [2][W][64] hand-off words
    const int ny = KP * 4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ll = lane & (kPLanes - 1);  // lanes 32..63 repeat lanes 0..31 (discarded)
    const int p = wg * kPLanes + ll;
    const bool live = lane < kPLanes && p < 2 * N;
    const int row = p >> 1;

    // this workgroup's packets -> LDS (read-only input: plain loads)
    {
        const f4v* src = reinterpret_cast<const f4v*>(SP) + (size_t)wg * KB * kPLanes;
        for (int e = tid; e < KP * kPLanes; e += blockDim.x)
            qs[e] = (e < KB * kPLanes) ? src[e] : f4v{0.0f, 0.0f, 0.0f, 0.0f};
        for (int e = tid; e < 2 * W * 64; e += blockDim.x) slot[e] = 0ull;
        // y past N (read by the last packet's products) stays +0 for the whole
        // solve: zeroed once in both parity buffers
        for (int e = tid; e < 2 * (KP * 4 - N); e += blockDim.x) ysb[(e & 1) * KP * 4 + N + (e >> 1)] = 0.0f;
    }
    const float fd = live ? fdpn[p] : 0.0f;
    __syncthreads();

    const int pk0 = persist_slice0(w);                           // first packet of this wave's slice
    const int pk1 = persist_slice0(w + 1);                       // one past its last
    const int k0 = 4 * pk0, k1 = 4 * pk1 < N ? 4 * pk1 : N;      // y[k0, k1) of the slice
    const bool last = (w == W - 1);
    float yrow = 0.0f;  // last wave: y_i of this lane's row (for y_next = num / den * y_i)
    // optional timeline (s_memtime) of workgroup 0: per update and wave,
    // {sweep start, y staged, turn (sums received), chain done}
    u64* tr = (TRACE && trace && wg == 0 && lane == 0) ? trace : nullptr;
    auto mark = [&](int u, int e) {
        if constexpr (TRACE)
            if (tr && u < trace_n) tr[((size_t)u * W + w) * 4 + e] = __builtin_amdgcn_s_memtime();
    };
    int bad = 0;  // an expired hand-off wait (code 2), reported after the update
    float yn = 0.0f;  // last wave: this lane's row of y_next
    for (int u = 0; u < updates; ++u) {
        const int par = u & 1;
        float* ys = ysb + par * ny;
        mark(u, 0);
        // ---- 1. y of this slice (k in [k0, k1)), staged in LDS ----
        auto stage_y = [&]() -> bool {
        if (u == 0) {
            for (int k = k0 + lane; k < k1; k += 64) ys[k] = Y0 ? Y0[k] : 1000.0f;  // initMat(Y, 1000) :710
            if (last) yrow = (Y0 && row < N) ? Y0[row] : 1000.0f;
        } else {
            // the sweep: the slice's granules (4 per lane, indices clamped into
            // the slice: a duplicate re-reads the slice's last granule, in the
            // same request as its neighbours) and, for the last wave, y_i of
            // this lane's row (:594); every load in flight, then one
            // wave-wide test of the tags (the data is its own flag).  No
            // per-lane conditions: the exit falls straight into the stores.
            const gu64* g = gran + (size_t)par * N;
            const unsigned tag = (unsigned)u;
            // this lane's granules, clamped into the slice; computed per call
            // (the laundered lane keeps them out of the registers held across
            // updates, where the products' 4 * kPW live)
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
                for (int m = 0; m < 4; ++m) x[m] = __hip_atomic_load(g + kk[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (last) xo = __hip_atomic_load(g + rowc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = true;
#pragma unroll
                for (int m = 0; m < 4; ++m) ok &= (unsigned)(x[m] >> 32) == tag;
                if (last) ok &= (unsigned)(xo >> 32) == tag;
                ok = __all(ok);
                if (!ok) {
                    if ((++spins & 63) == 0 && dl.expired()) return false;
                    // one sweep at a time, a short pause between them (two sweeps
                    // in flight, issued 256 to 512 clocks apart, measured 5-15 %
                    // slower: the pollers' own traffic); wave 0 without a pause
                    // and waves 2+ with 4 units: 3.58-3.64 against 3.61-3.69 us
                    // per update (profiles/r05/persist_sleep_ab*.txt)
                    if (w == 0) {
                        if (PQP_PS_SLEEP0 > 0) __builtin_amdgcn_s_sleep(PQP_PS_SLEEP0);
                    } else if (w == 1) {
                        __builtin_amdgcn_s_sleep(PQP_PS_SLEEP1);
                    } else {
                        __builtin_amdgcn_s_sleep(PQP_PS_SLEEPN);
                    }
                }
            } while (!ok);
            // duplicates store the same value to the same word
#pragma unroll
            for (int m = 0; m < 4; ++m) ys[kk[m]] = __uint_as_float((unsigned)x[m]);
            if (last) yrow = __uint_as_float((unsigned)xo);
        }
        mark(u, 1);
        return true;
        };
        // one base address per operand, the packet index as an immediate offset
        const f4v* qw = qs + (size_t)pk0 * kPLanes + ll;
        const f4v* yw = reinterpret_cast<const f4v*>(ys) + pk0;
        float acc = 0.0f;
        u64* sl = slot + (size_t)par * W * 64;
        const unsigned want = (unsigned)(u + 1);
        // the wave's sums done: hand them on, or (last wave) finish the rows.
        // Called at the end of each chain form, so that each runs straight
        // into its hand-off.  False: the launch failed (reported).
        auto finish = [&](float acc) -> bool {
            asm volatile("" : "+v"(acc));  // the mark below follows the chain
            mark(u, 3);
            if (!last) {
                __hip_atomic_store(sl + w * 64 + lane, ((u64)want << 32) | __float_as_uint(acc), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                __builtin_amdgcn_s_setprio(0);
                if (bad) {
                    fail(err, bad);
                    return false;
                }
                return true;
            }
            __builtin_amdgcn_s_setprio(0);
            // ---- 4. the last slice's wave finishes the rows ----
            const float v = acc + 1.0f * fd;  // even lane: num (:611), odd lane: den (:612)
            // the partner lane's sum by a DPP swap of lane pairs (quad_perm 1,0,3,2),
            // not an LDS permute; every lane divides (odd lanes' quotients unused)
            const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
            yn = v / den * yrow;  // :594
            if (!(p & 1) && live)
                __hip_atomic_store(gran + (size_t)(par ^ 1) * N + row, ((u64)want << 32) | __float_as_uint(yn),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (bad) {
                fail(err, bad);
                return false;
            }
            return true;
        };
        if (w == 0) {
            // wave 0 reads its slice's split entries while it waits for y:
            // its products start the chain, and then need only the y reads
            f4v q0[kPW0];
#pragma unroll
            for (int j = 0; j < kPW0; ++j) q0[j] = qs[(size_t)j * kPLanes + ll];
            if (!stage_y()) {
                fail(err, 1);
                return;
            }
            // ---- 2/3 (wave 0). the chain starts here, right after its products ----
            mark(u, 2);
            __builtin_amdgcn_s_setprio(3);
            if (!finish(chain_qreg(acc, q0, yw))) return;
        } else {
            // products ahead of the turn, the running sums of the previous
            // slice, then this slice's adds; NP = the slice's packets
            auto turn = [&](auto np) -> int {
                constexpr int NP = decltype(np)::value;
                f4v prod[NP];
                // the slice's split entries, read while the wave waits for y
                // (multiplied in place once y is staged)
#pragma unroll
                for (int j = 0; j < NP; ++j) prod[j] = qw[(size_t)j * kPLanes];
                if (!stage_y()) return 1;
                if (w >= 4) {
                    // waves 4, 5 share SIMDs with waves 0, 1: they form their
                    // products once wave kLateGate has handed on its sums, so
                    // the first waves' products and chains run alone
                    if (!lds_wait(sl + kLateGate * 64 + lane, want, true)) bad = 2;
                }
                slice_products_inplace(prod, yw);
                // pinned here: otherwise the compiler sinks the multiplies into the chain
#pragma unroll
                for (int j = 0; j < NP; ++j) asm volatile("" : "+v"(prod[j]));
                u64 h;
                // an expired wait is reported once the update's sums are handed
                // on (no branch between the sums' arrival and the first add)
                if (!lds_wait_sums(sl + (w - 1) * 64 + lane, want, h)) bad = 2;
                acc = __uint_as_float((unsigned)h);
                mark(u, 2);
                __builtin_amdgcn_s_setprio(3);
                if (TRACE && trace && wg == 0 && u < trace_n) {
                    // traced launches only: s_memtime before each seventh of
                    // the chain (stored after it), to see where a slice loses time
                    constexpr int G = 7, PG = (NP + G - 1) / G;
                    u64 t[G + 1];
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        __builtin_amdgcn_sched_barrier(0);
                        t[g] = __builtin_amdgcn_s_memtime();
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int j = g * PG; j < (g + 1) * PG && j < NP; ++j) {
                            acc += prod[j].x;  // :608-609, k in order
                            acc += prod[j].y;
                            acc += prod[j].z;
                            acc += prod[j].w;
                        }
                        asm volatile("" : "+v"(acc));
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    t[G] = __builtin_amdgcn_s_memtime();
                    __builtin_amdgcn_sched_barrier(0);
                    if (lane == 0) {
                        u64* ext = trace + (size_t)trace_n * W * 4 + ((size_t)u * W + w) * 8;
#pragma unroll
                        for (int g = 0; g < G + 1 && g < 8; ++g) ext[g] = t[g];
                    }
                    return finish(acc) ? 0 : 3;
                }
#pragma unroll
                for (int j = 0; j < NP; ++j) {
                    acc += prod[j].x;  // :608-609, k in order
                    acc += prod[j].y;
                    acc += prod[j].z;
                    acc += prod[j].w;
                }
                return finish(acc) ? 0 : 3;
            };
            const int rc = (w == 1) ? turn(std::integral_constant<int, kPW1>{}) : turn(std::integral_constant<int, kPW>{});
            if (rc) {
                if (rc == 1) fail(err, rc);  // 3: reported by finish
                return;
            }
        }
    }
    if (last && updates > 0 && !(p & 1) && live) Yout[row] = yn;
}


// Can all G workgroups of k_split_persist be resident at once?  The launch's
// waits need every producer running; a grid that cannot be co-resident would
// only end by its deadline.  Occupancy of this kernel (LDS-bound: one per CU)
// times the CUs, against G.
bool split_persist_fits(int N) {
    if (N < 1 || N > persist_max_n()) return false;
    const int G = (2 * N + kPLanes - 1) / kPLanes, threads = 64 * persist_waves(N);
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
    if (g_tune.persist_fit_cus > 0) cus = g_tune.persist_fit_cus;
    const void* kern = g_tune.persist_trace ? reinterpret_cast<const void*>(&k_split_persist<true>)
                                       : reinterpret_cast<const void*>(&k_split_persist<false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, threads, persist_lds_bytes(N)) != hipSuccess)
        return false;
    return (long long)per * cus >= G;
}

hipError_t launch_split_persist(const float* SP, const float* fdpn, int N, int updates, const float* Y0, float* Yout,
                                unsigned long long* gran, int* err, hipStream_t s) {
    if (updates <= 0) return hipSuccess;
    const int W = persist_waves(N);
    const int G = (2 * N + kPLanes - 1) / kPLanes;
    hipError_t e = hipMemsetAsync(gran, 0, sizeof(u64) * 2 * N, s);
    if (e == hipSuccess) e = hipMemsetAsync(err, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    // the G workgroups packed onto x XCDs (x * 32 >= G), the grid padded with
    // workgroups that leave at once: 4 by default (n_dual 1024, 64 workgroups:
    // 3.58 -> 3.49 ms per 1000 updates against all eight XCDs, 3.71 on two;
    // profiles/r06/persist_xcd_ab_r06l.json); persist_xcds 8 spreads them
    const int want = g_tune.persist_xcds > 0 ? g_tune.persist_xcds : 4;
    const int xcds = (want < 8 && want * 32 >= G) ? want : 0;
    const int grid = xcds ? 8 * ((G + xcds - 1) / xcds) : G;
    if (g_tune.persist_trace)
        hipLaunchKernelGGL(k_split_persist<true>, dim3(grid), dim3(64 * W), persist_lds_bytes(N), s, SP, fdpn, N,
                           updates, Y0, Yout, gran, err, g_tune.persist_trace, g_tune.persist_trace_n,
                           g_tune.persist_stall_wg, xcds);
    else
        hipLaunchKernelGGL(k_split_persist<false>, dim3(grid), dim3(64 * W), persist_lds_bytes(N), s, SP, fdpn, N,
                           updates, Y0, Yout, gran, err, nullptr, 0, g_tune.persist_stall_wg, xcds);
    return hipGetLastError();
}

}  // namespace pqp
