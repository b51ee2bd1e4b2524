// pqp_launch.h -- internal interface between the host shim (pqp_capi.cpp) and
// the kernel translation unit (pqp_kernels.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pqp {

enum SolveStatus : int { kStatusContinue = 0, kStatusDone = 1, kStatusCapped = 2 };
// SolveArgs::mode: 0 converge, 1 fixed, 2 evaluate terminate() once (no update)
enum SolveMode : int { kModeConverge = 0, kModeFixed = 1, kModeTerminate = 2 };

// Device-resident state of a (resumable) single-problem solve.
struct SolveState {
    long long h;     // reference's h of the current iterate (starts at 1)
    int status;      // SolveStatus
    int resume;      // 0: start from Y = 1000; 1: continue from SolveArgs::Y
    float Jp, Jd;    // costs of the last terminate() that passed checkFeas
    int have_costs;
    int last_stop;   // result of the last terminate() (mode 2)
};

// All device pointers.  Qd row-major N x N (Jd's Y'Qd row), QdT column-major
// (ldq) for the update, Gp row-major N x M, Qinv/Qp row-major M x M.
// Batched: workgroup b solves problem b; every array holds B problems back to
// back (row-major per problem, strides N*N, N, 1, M*M, ... ; QdT N*ldq).
struct SolveArgs {
    const float *QdT, *Qd, *theta, *Fd, *Md, *Qp, *Qinv, *Fp, *Mp, *Gp, *Kp;
    float *Y, *U;
    int N, M, ldq, ldm, mode;
    long long num_iter, max_updates, chunk;
    int* pending;  // optional: +1 per problem still running when a launch ends
    const int* sym;  // optional (k_solve_single): sym[b] != 0 when problem b's Qd is bit-symmetric
    const float *GpT, *QinvT;  // optional (k_solve_single): transposes of Gp (M x N) and Qp_inv, per problem
    int feas_split;  // k_solve_single with GpT: checkFeas decides on its first rows when one is over its bound
    unsigned long long* trace;  // optional (k_solve_mid): 16 words of phase cycle totals per traced problem
    int trace_n;                // problems traced (workgroups 0..trace_n-1)
    // one small problem in one launch (pqp_tiny.hip):
    int fresh;        // 1: start from SolveState{h = 1}, ignoring the device state (no state upload)
    void* hout;       // optional pinned host buffer (kTinyOut* layout): Y, U, state, error word
    int tiny_flags;   // kTinyDense: the fixed-mode solve sums every entry (no sparse form)
    int out_tag;      // written last to hout (kTinyOutTagOffset): the host checks it is this launch's
};
// k_fixed_one / k_solve_quintet host output: Y at 0, U at kTinyOutUOffset, the
// SolveState at kTinyOutStateOffset (floats), an int error word at kTinyOutErrOffset
constexpr int kTinyOutUOffset = 32, kTinyOutStateOffset = 64, kTinyOutErrOffset = 72, kTinyOutTagOffset = 73,
              kTinyOutFloats = 80;
static_assert(sizeof(SolveState) <= 4 * (kTinyOutErrOffset - kTinyOutStateOffset),
              "the SolveState must end before the error word of the tiny output");
static_assert(kTinyOutErrOffset < kTinyOutTagOffset && kTinyOutTagOffset < kTinyOutFloats, "tiny output layout");
// the device copy of the error word: the int right behind the handle's
// SolveState (the host reads it when the pinned output lacks the launch's tag)
constexpr int kTinyDevErr = (int)sizeof(SolveState);
constexpr int kTinyTraceWords = 24;  // k_solve_quintet's timeline: 4 words per role + 4
constexpr int kTinyDense = 1;
constexpr int kTinyStall = 2;  // error-path tests: k_solve_quintet's deciding waves never decide
constexpr int kMid2Dense = 4;  // k_solve_mid2: no band skipping (tune mid2_dense)
// one problem with N, M <= 32 (fixed mode; converge mode needs N + M < 64) in one launch
hipError_t launch_one_tiny(const SolveArgs& a, SolveState* st, hipStream_t s);
// test hook: 8 * cus workgroups each fill 64 KB of LDS with `bits` (pqp_tune_poison_lds)
hipError_t launch_poison_lds(int bits, int* seen, int cus, hipStream_t s);
hipError_t launch_transpose_b(int B, const float* src, int rows, int cols, float* dst, hipStream_t s);
// sym[b] = nonzero iff problem b's row-major Qd equals its transpose bit for bit
hipError_t launch_check_symmetric(int B, const float* Qd, int N, int* sym, hipStream_t s);

hipError_t launch_batch_iterate(int B, const float* QdT, long long qstride, int ldq, int N, const float* theta,
                                const float* Fd, int ldv, const float* Y0, float* Y, int updates, hipStream_t s);
hipError_t launch_batch_update(int B, const float* QdT, long long qstride, int ldq, int N, const float* theta,
                               const float* Fd, int ldv, const float* Yin, float* Yout, hipStream_t s);
hipError_t launch_update_split(const float* QpT, const float* QnT, int ldq, int N, const float* Fdp,
                               const float* Fdn, const float* Y, float* Ynext, hipStream_t s);
hipError_t launch_pack_colmajor(int B, const float* Qd, int N, long long in_stride, float* QdT, int ldq,
                                long long qstride, hipStream_t s);
hipError_t launch_theta(int B, const float* QdT, int ldq, long long qstride, int N, float* theta, int ldv,
                        hipStream_t s);
hipError_t launch_synth(uint32_t seed, long long inst0, int B, int N, int M, float* QdT, int ldq, long long qstride,
                        float* Fd, int ldv, float* Md, hipStream_t s);
hipError_t launch_synth_primal(uint32_t seed, long long inst0, int B, int N, int M, float* Qinv, float* Gp, float* Kp,
                               float* Fp, float* Mp, hipStream_t s);
hipError_t launch_matmul_seq(float* out, const float* A, int tA, const float* B, int tB, int a, int b, int c,
                             hipStream_t s);
hipError_t launch_axpy(float* A, const float* B, float sign, int n, hipStream_t s);
hipError_t launch_negate(float* A, int n, hipStream_t s);
hipError_t launch_compare(const float* gu, const float* Kp, int n, int* flag, hipStream_t s);
hipError_t launch_theta_rowmajor(const float* Qd, int N, float* theta_mat, hipStream_t s);
hipError_t launch_cost_finish(const float* quad, const float* lin, const float* Mc, float* J, hipStream_t s);
hipError_t launch_mp_finish(const float* t, const float* Mp6, float* Mp, hipStream_t s);
hipError_t launch_gauss_jordan(const float* A, float* aug, float* fac, float* res, int n, hipStream_t s);
size_t solve_single_lds_bytes(int ldq, int ldm, bool fused = false);
size_t solve_pipe_lds_bytes(int ldq, int ldm, bool big = false);
constexpr size_t kPipeLdsMax = 150 * 1024;
// path 2's converge-mode kernel by shape: true = k_solve_pipe (needs Qp_inv' only)
bool pipe_route(int N, int M, int variant);
extern thread_local int g_last_batch_kernel;  // the calling thread's last path-2/3 launch: 0 k_solve_single, 1 k_solve_pipe, 2 k_solve_mid, 3 k_solve_mid2
size_t solve_small_lds_bytes(int N, int M);
size_t solve_mid_lds_bytes(int N, int M, bool conv);
hipError_t launch_solve_small(const SolveArgs& a, SolveState* st, hipStream_t s);
hipError_t launch_solve_tiny(const SolveArgs& a, SolveState* st, hipStream_t s);  // N, M <= 32
// row block [row0, row0 + rows) of one large problem, fixed mode,
// multi-workgroup (stored split matrices); rows = N, row0 = 0 for a whole problem
hipError_t launch_build_split(const float* Qd, int ld, const float* theta, const float* Fd, int N, int rows,
                              int row0, int lw, float* SP, float* fdpn, hipStream_t s);
hipError_t launch_theta_rows(const float* Qd, int ld, int N, int rows, float* theta, hipStream_t s);
// gate: optional; the launch does nothing unless *gate == kStatusContinue.
// err: optional sticky device word; a relay hand-off wait that expired ORs 1
// into it
hipError_t launch_split_update(const float* SP, const float* fdpn, int N, int rows, int row0, int lw,
                               const float* Yin, float* Yout, hipStream_t s, const int* gate = nullptr,
                               int* err = nullptr);
constexpr int kRelaySpinMax = 1 << 20;  // relay hand-off wait budget in polls (~0.1-1 s)
struct Tuning {  // every tuning knob of the library (pqp_tune, include/pqp_tuning.h); defaults = production
    int relay_spin_max = kRelaySpinMax;  // relay hand-off wait budget in polls (< 0: every wait expires at once)
    int lean_min_n = 4096;  // k_lean_relay for row blocks of rows x N >= lean_min_n^2 entries
    int split_lw = 0;  // relay lanes per workgroup (0 auto, else 8/16/32/64)
    int wave_pipe_max_b = 4096;  // largest batch whose k_solve_wave launch is the software-pipelined form
    int fixed_rl_max_b = 1024;  // largest batch whose k_fixed_tiny keeps y in registers
    int wave_min_b = 1;  // converge mode of N, M <= 32 on k_solve_wave from this many problems on
    int matmul_tiled_off = 0;  // every product through k_matmul_seq
    int gj_blocked_off = 0;  // Gauss_Jordan through the one-pivot-per-sweep kernel
    int single_scalar = 0;  // k_solve_single with 4-byte loads only
    int persist_off = 0;  // fixed mode of n_dual <= 1024 through the graph-replayed relay
    int persist_stall_wg = -1;  // workgroup of each persistent launch that never runs (error-path tests; -1: none)
    unsigned long long* persist_trace = nullptr;  // k_split_persist timeline buffer (device)
    int persist_trace_n = 0;  // updates the timeline buffer holds
    int persist_fit_cus = 0;  // CU count the residency checks assume (0: the device's)
    int converge_persist_off = 0;  // converge mode through the graph chain instead of the persistent launch
    unsigned long long* mid_trace = nullptr;  // k_solve_mid phase totals buffer (device)
    int mid_trace_n = 0;  // problems it holds
    unsigned long long* converge_trace = nullptr;  // k_converge_persist timeline buffer (device)
    int converge_trace_n = 0;  // iterates the timeline buffer holds
    bool force_small = false;  // route N <= 32 to k_solve_small instead of k_solve_tiny
    bool force_single = false;  // fixed mode of a large problem on one workgroup (k_solve_single)
    int wide_min_n = 384;  // converge mode: smallest N solved over many workgroups
    long long batch_chunk = 0;  // iterates per problem per batched-solve launch (0: sized from N, M)
    int mid_off = 0;  // batched solves of mid-size N through k_solve_small / k_solve_single instead of path 3
    int mid2_pair = 0;  // k_solve_mid2's update rows: 0 by shape, 1 lane sides (v_med3_f32), 2 one lane per row
    int single_occ = 0;  // k_solve_single (wide loads) workgroups per CU by register cap: 0 by shape and batch (3 above n_dual 768), 3 / 4 / 5 forced
    int mid2_dense = 0;  // k_solve_mid2 sums every k (default: each row group's nonzero band while Y is finite)
    int mid2_min_n = 48;  // smallest N path 3 runs on k_solve_mid2 (below it k_solve_mid)
    int mid_v1 = 0;  // path 3 on k_solve_mid (terminate() after the update) instead of the pipelined k_solve_mid2
    int pipe_variant = 0;  // k_solve_pipe build: 0 (128 x 96 Gp tiles, 16 update loads per lane in flight, 2 WGs/CU), 3 (two 64 x 64 tiles in flight)
    int pipe_force = 0;  // k_solve_pipe also where M < N / 3 (where k_solve_single measured faster)
    int matmul_pk_off = 0;  // setup GEMMs on the 64 x 64 scalar-staged k_matmul_tiled instead of the packed 128 x 128 k_matmul_pk
    int pipe_off = 0;  // batched converge of large problems on k_solve_single (two passes over Gp) instead of k_solve_pipe
    int batch_opts = 0;  // pqp_batch_solve: bit 0 no fused Y'Qd, bit 1 per-call transposes, bit 4 checkFeas over every row
    long long converge_chunk = 1 << 16;  // iterates decided per persistent converge launch
    int tiny_old = 0;    // one small problem on k_fixed_tiny / k_solve_wave (state copies) instead of k_fixed_one / k_solve_quintet
    int tiny_dense = 0;  // k_fixed_one / k_solve_quintet without the sparse update form
    int iterate_kind = 0;  // pqp_batch_iterate: 0 default (k_batch_resident at N 1024, k_batch_stream at other
                           // multiples of 1024, k_batch_iterate otherwise), 1 k_batch_iterate, 2 k_batch_stream,
                           // 3 k_batch_resident without its register blocks
    int tiny_stall = 0;  // k_solve_quintet's deciding waves return at once: every wait expires (error path)
    int persist_xcds = 0;  // k_split_persist's workgroups packed onto this many XCDs (0: 4, 8: spread over all)
    int converge_xcds = 0;  // k_converge_persist's workgroups packed onto this many XCDs (0: 6, 8: spread over all)
    int tiny_apoll = 0;  // k_solve_quintet's update wave polls the decision word every update (default: only when the ring is full)
    int tiny_ablk = 0;  // k_solve_quintet's update wave: 1 = publish every update (round 6 before r06q); default 2 per pass
    int tiny_np = 0;  // k_solve_quintet's B / C waves per role: 2, 3 (0: default) or 4
    int tiny_fallback = 0;  // the host reads a tiny solve's device copies as if the pinned output were stale (tests)
    long long tiny_chunk = 0;  // iterates per one-launch tiny solve launch (0: about 2^26 element updates)
    unsigned long long* tiny_trace = nullptr;  // k_solve_quintet per-wave clocks (24 words; N = 28, M <= 8 only)
};
extern Tuning g_tune;
long long batch_chunk_for(int N, int M);  // iterates per problem per batched-solve launch (pqp_capi.cpp)
hipError_t launch_fill(float* a, float v, int n, hipStream_t s);
// packets of 4 k per row side in the split layout (k padded to a multiple of 4)
__host__ __device__ inline int split_kblocks(int N) { return (N + 3) / 4; }
// fixed mode of one problem with N <= persist_max_n() as ONE persistent launch
// (pqp_persist.hip): SP built with lw = 32; gran = 2N granules, err = 1 int
int persist_max_n();
size_t persist_lds_bytes(int N);
hipError_t launch_split_persist(const float* SP, const float* fdpn, int N, int updates, const float* Y0, float* Yout,
                                unsigned long long* gran, int* err, hipStream_t s);
bool split_persist_fits(int N);  // all of k_split_persist's workgroups co-resident on this device
size_t split_floats(int N, int rows, int lw);  // size of a row block's packed split matrices
// lean relay (k_lean_relay): Qd packets (4 B per entry, lw / 2 rows per
// workgroup) and aux[row] = {Fdn, Fdp, Theta, 0} + NaN flags; used for blocks
// of rows x N >= g_tune.lean_min_n^2 entries
bool use_lean(int N, int rows);
size_t lean_floats(int N, int rows, int lw);
size_t lean_aux_floats(int N, int rows, int lw);  // per-row words + per-(workgroup, segment) NaN flags
int lean_pick_lw(int rows);
hipError_t launch_build_lean(const float* Qd, int ld, const float* theta, const float* Fd, int N, int rows, int row0,
                             int lw, float* LP, float* aux, hipStream_t s);
hipError_t launch_lean_update(const float* LP, const float* aux, int N, int rows, int row0, int lw, const float* Yin,
                              float* Yout, hipStream_t s, const int* gate = nullptr, int* err = nullptr);
int split_pick_lw(int rows);                   // lanes per workgroup for a block of `rows`
size_t split_lds_bytes(int N);         // LDS of a row block's update (the full y)
// rows [row0, row0 + rows) of synthetic problem `inst` (row-major, ld >= N,
// columns [N, ld) zeroed) and, if Fd, its full Fd (and Md)
hipError_t launch_synth_rows(uint32_t seed, long long inst, int N, int M, int row0, int rows, float* Qrows, int ld,
                             float* Fd, float* Md, hipStream_t s);
// batched forms: grid = B problems (states st[0..B-1])
hipError_t launch_solve_batch(int B, int path, const SolveArgs& a, SolveState* st, hipStream_t s);
hipError_t launch_state_init(int B, SolveState* st, hipStream_t s);
hipError_t launch_extract_state(int B, const SolveState* st, long long* h, int* status, hipStream_t s);
hipError_t launch_matmul_seq_b(int B, float* out, const float* A, int tA, const float* Bm, int tB, int a, int b,
                               int c, long long sA, long long sB, long long sO, hipStream_t s);
hipError_t launch_axpy_b(int B, float* A, const float* Bv, float sign, int n, long long sA, long long sB,
                         hipStream_t s);
hipError_t launch_negate_b(int B, float* A, int n, long long sA, hipStream_t s);
hipError_t launch_mp_finish_b(int B, const float* t, const float* Mp6, float* Mp, long long sMp6, hipStream_t s);
hipError_t launch_gauss_jordan_b(int B, const float* A, float* aug, float* fac, float* res, int n, hipStream_t s);
// floats of one matrix's augmented workspace (`aug` holds B of them)
size_t gauss_jordan_aug_floats(int n);
// ---- converge mode of one large problem over many workgroups (pqp_wide.hip)
enum GemvEpi : int { kEpiPlain = 0, kEpiAdd = 1, kEpiNeg = 2, kEpiFeas = 3 };
// out[j] = epi( sum_k A[k * lda + j] * x[k] ), j < n_out, k = 0..n_in-1 in order
struct GemvJob {
    const float* A;
    const float* x;
    float* out;
    const float* add;  // kEpiAdd: out += 1.0f * add[j]; kEpiFeas: Kp
    int lda, n_in, n_out, epi;
};
struct WideArgs {
    SolveState* st;
    int* flag;
    const float *tq, *tu, *Y, *U, *Fd, *Fp, *Md, *Mp;
    int N, M;
    const long long* max_updates;  // device word: <= 0 means no cap (read each iteration)
};
struct GemvJobs {
    GemvJob job[2];          // job[1].A == nullptr: one job
    int wgs0;                // set by the launcher
    const int* gate;         // optional: skip unless *gate == kStatusContinue
    int* flag;               // kEpiFeas: cleared to 0 by an infeasible row
    int* err;                // optional sticky word: an expired hand-off wait ORs 1 into it
    int spin_max;            // set by the launcher (g_tune.relay_spin_max)
};
hipError_t launch_transpose(const float* src, int rows, int cols, float* dst, hipStream_t s);
hipError_t launch_gemv_relay(const GemvJobs& jobs, hipStream_t s);
hipError_t launch_wide_decide(const WideArgs& a, hipStream_t s);
hipError_t launch_wide_init(SolveState* st, int* flag, long long* cap, long long max_updates, float* Y, int N,
                            hipStream_t s);
// Gauss_Jordan of one n x n matrix, one launch per pivot (aug: 2n*n floats, perm: n ints)
hipError_t launch_gauss_jordan_wide(const float* A, float* aug, int* perm, float* res, int n, hipStream_t s);
constexpr int kGaussJordanWideMin = 64;  // n from which one matrix is inverted over many workgroups

// ---- converge mode of one problem with N, M <= 1024 as ONE persistent,
// pipelined launch (pqp_converge.hip): update and terminate() stages as
// concurrent roles exchanging tagged granules
struct ConvergeLaunch {
    int N, M;
    long long u0;     // iterate the launch starts from (its y in Y)
    long long chunk;  // iterates decided per launch at most
    long long cap;    // max_updates (<= 0: none)
    const float *SP, *A1, *A2, *A3;  // update packets (k_build_split, lw = 32) and stage packets
    const float *fdpn, *Fp, *Kp, *Fd, *Md, *Mp;
    void* rings;      // converge_ring_words() 8-byte words
    SolveState* st;
    int* ctl;
    long long* decided;
    int* err;
    float *Y, *U;     // in: y_{u0}; out: the final (or next launch's) iterate, U of the last terminate()
};
int converge_persist_wgs(int N, int M, int* g);  // workgroups of the launch (0: not applicable)
size_t converge_persist_lds_bytes(int N, int M);
int converge_persist_per_cu(int N, int M);  // k_converge_persist workgroups per CU (occupancy API)
size_t converge_ring_words(int N, int M);
size_t converge_stage_floats(int N, int M, int stage);  // stage 1..3 packet arrays
hipError_t launch_converge_pack(const float* Qd, const float* Gp, const float* Qinv, const float* Qp, int N, int M,
                                float* A1, float* A2, float* A3, hipStream_t s);
hipError_t launch_converge_persist(const ConvergeLaunch& L, hipStream_t s);

hipError_t launch_solve_single(const SolveArgs& a, SolveState* st, hipStream_t s);

}  // namespace pqp
