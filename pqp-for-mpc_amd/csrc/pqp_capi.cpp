// pqp_capi.cpp -- the C ABI of libpqp (include/pqp.h): a thin host shim that
// validates arguments, moves caller buffers to/from HBM and launches the
// gfx950 kernels of pqp_kernels.hip.  No arithmetic of the solver runs on the
// host: every drop-in function is computed on the GPU and fails loudly (status
// code, or exit(EXIT_FAILURE) for the void drop-ins) when no gfx950 device or
// kernel is available -- there is no CPU fallback.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "pqp_internal.h"
#include "pqp_launch.h"

namespace pqp {

namespace {

inline int round4(int n) { return (n + 3) & ~3; }

// RAII device allocation.
struct DevBuf {
    void* p = nullptr;
    size_t bytes_ = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    // (re)allocate; a buffer of the same size is kept (same address: no
    // hipMalloc/hipFree pair, and graphs captured over it stay valid)
    int alloc(size_t bytes) {
        if (bytes == 0) bytes = 16;
        if (p && bytes == bytes_) return PQP_OK;
        if (p) {
            (void)hipFree(p);
            p = nullptr;
            bytes_ = 0;
        }
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) {
            p = nullptr;
            return set_error(PQP_ERR_ALLOC, "hipMalloc(%zu bytes): %s", bytes, hipGetErrorString(e));
        }
        bytes_ = bytes;
        return PQP_OK;
    }
    int floats(size_t n) { return alloc(n * sizeof(float)); }
    float* f() const { return static_cast<float*>(p); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes_ = 0;
    }
};

// Verify that the current device is a gfx950 (the only code object we ship).
int ensure_device() {
    static std::mutex mu;
    static int checked[64] = {0};  // 0 unknown, 1 ok, <0 error code
    int dev = 0;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) return set_error(PQP_ERR_NO_DEVICE, "libpqp: no HIP device visible");
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return set_error(PQP_ERR_NO_DEVICE, "libpqp: cannot query the current device");
    std::lock_guard<std::mutex> lk(mu);
    if (checked[dev] == 0) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
            checked[dev] = PQP_ERR_NO_DEVICE;
        } else if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            checked[dev] = PQP_ERR_NO_DEVICE;
            return set_error(PQP_ERR_NO_DEVICE, "libpqp is built for gfx950 only; device %d is %s", dev,
                             prop.gcnArchName);
        } else {
            checked[dev] = 1;
        }
    }
    if (checked[dev] < 0) return set_error(checked[dev], "libpqp: device %d is not a usable gfx950", dev);
    return PQP_OK;
}

// The stream of the drop-ins and of handles made without one: one per host
// thread and device, so calls from different threads never share a stream
// (or a lock); the drop-ins keep no other state between calls.  A thread's
// streams are destroyed when the thread exits (short-lived caller
// threads must not leak one stream each); the loading thread's stay until the
// process ends, where the HIP runtime may already be shutting down.
static const std::thread::id g_load_thread = std::this_thread::get_id();
struct ThreadStreams {
    hipStream_t s[64] = {nullptr};
    ~ThreadStreams() {
        if (std::this_thread::get_id() == g_load_thread) return;
        for (hipStream_t& x : s)
            if (x) (void)hipStreamDestroy(x);
    }
};
hipStream_t lib_stream() {
    thread_local ThreadStreams streams;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    if (!streams.s[dev]) (void)hipStreamCreateWithFlags(&streams.s[dev], hipStreamNonBlocking);
    return streams.s[dev];
}

// Make `dev` the calling thread's current device for a scope (a handle's calls
// run on the device it was made on, whatever the caller has current), and
// restore the caller's device after.
struct DeviceGuard {
    int prev = -1;
    bool changed = false;
    explicit DeviceGuard(int dev) {
        if (dev >= 0 && hipGetDevice(&prev) == hipSuccess && prev != dev) changed = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (changed) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

int upload(DevBuf& d, const float* h, size_t n, hipStream_t s) {
    PQP_TRY(d.floats(n));
    if (n) PQP_HIP(hipMemcpyAsync(d.p, h, n * sizeof(float), hipMemcpyHostToDevice, s));
    return PQP_OK;
}
int download(float* h, const void* d, size_t n, hipStream_t s) {
    if (n) PQP_HIP(hipMemcpyAsync(h, d, n * sizeof(float), hipMemcpyDeviceToHost, s));
    return PQP_OK;
}

// ---- device compositions of the reference's helper functions -------------
int dev_matmul(float* out, const float* A, int tA, const float* B, int tB, int a, int b, int c, hipStream_t s) {
    PQP_HIP(launch_matmul_seq(out, A, tA, B, tB, a, b, c, s));
    return PQP_OK;
}

// convertToDual (PQP_CPU.c:489-498)
int dev_convert_to_dual(float* Qd, float* Fd, float* Md, const float* Qinv, const float* Gp, const float* Kp,
                        const float* Fp, const float* Mp, int N, int M, hipStream_t s) {
    DevBuf GQ, fq;
    PQP_TRY(GQ.floats((size_t)N * M));
    PQP_TRY(fq.floats(M));
    PQP_TRY(dev_matmul(GQ.f(), Gp, 0, Qinv, 0, N, M, M, s));  // Gp_Qp_inv          :492
    PQP_TRY(dev_matmul(Qd, GQ.f(), 0, Gp, 1, N, M, N, s));    // computeQd          :442
    PQP_TRY(dev_matmul(Fd, GQ.f(), 0, Fp, 0, N, M, 1, s));    // computeFd          :458
    PQP_HIP(launch_axpy(Fd, Kp, 1.0f, N, s));                  //                    :459
    PQP_TRY(dev_matmul(fq.f(), Fp, 1, Qinv, 0, 1, M, M, s));  // computeMd          :475
    PQP_TRY(dev_matmul(Md, fq.f(), 0, Fp, 0, 1, M, 1, s));    //                    :476
    PQP_HIP(launch_axpy(Md, Mp, -1.0f, 1, s));                 // Md[0] -= Mp[0]     :478
    PQP_HIP(hipStreamSynchronize(s));                          // before scratch is freed
    return PQP_OK;
}

// computeUfromY (PQP_CPU.c:352-360)
int dev_u_from_y(float* U, const float* Y, const float* Fp, const float* Gp, const float* Qinv, int N, int M,
                 hipStream_t s) {
    DevBuf t;
    PQP_TRY(t.floats(M));
    PQP_TRY(dev_matmul(t.f(), Gp, 1, Y, 0, M, N, 1, s));
    PQP_HIP(launch_axpy(t.f(), Fp, 1.0f, M, s));
    PQP_TRY(dev_matmul(U, Qinv, 0, t.f(), 0, M, M, 1, s));
    PQP_HIP(launch_negate(U, M, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

// checkFeas (PQP_CPU.c:632-641) -> host int
int dev_check_feas(const float* U, const float* Gp, const float* Kp, int N, int M, int* out, hipStream_t s) {
    DevBuf gu, flag;
    PQP_TRY(gu.floats(N));
    PQP_TRY(flag.alloc(sizeof(int)));
    const int one = 1;
    PQP_HIP(hipMemcpyAsync(flag.p, &one, sizeof(int), hipMemcpyHostToDevice, s));
    PQP_TRY(dev_matmul(gu.f(), Gp, 0, U, 0, N, M, 1, s));
    PQP_HIP(launch_compare(gu.f(), Kp, N, static_cast<int*>(flag.p), s));
    PQP_HIP(hipMemcpyAsync(out, flag.p, sizeof(int), hipMemcpyDeviceToHost, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

// computeCost (PQP_CPU.c:648-666) -> device scalar J
int dev_cost(float* J, const float* Z, const float* Q, const float* F, const float* Mc, int n, hipStream_t s) {
    DevBuf row, quad, lin;
    PQP_TRY(row.floats(n));
    PQP_TRY(quad.floats(1));
    PQP_TRY(lin.floats(1));
    PQP_TRY(dev_matmul(row.f(), Z, 1, Q, 0, 1, n, n, s));
    PQP_TRY(dev_matmul(quad.f(), row.f(), 0, Z, 0, 1, n, 1, s));
    PQP_TRY(dev_matmul(lin.f(), F, 1, Z, 0, 1, n, 1, s));
    PQP_HIP(launch_cost_finish(quad.f(), lin.f(), Mc, J, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

// computeFp (PQP_CPU.c:373-382)
int dev_compute_fp(float* Fp, const float* Fp1, const float* Fp2, const float* Fp3, const float* D, const float* x,
                   int m, int nd, int ns, hipStream_t s) {
    DevBuf t;
    PQP_TRY(t.floats(m));
    PQP_TRY(dev_matmul(Fp, Fp1, 0, D, 0, m, nd, 1, s));
    PQP_TRY(dev_matmul(t.f(), Fp2, 0, x, 0, m, ns, 1, s));
    PQP_HIP(launch_axpy(Fp, t.f(), 1.0f, m, s));
    PQP_HIP(launch_axpy(Fp, Fp3, -1.0f, m, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

// computeMp (PQP_CPU.c:395-428)
int dev_compute_mp(float* Mp, const float* Mp1, const float* Mp2, const float* Mp3, const float* Mp4,
                   const float* Mp5, const float* Mp6, const float* D, const float* x, int nd, int ns,
                   hipStream_t s) {
    DevBuf row, terms;
    PQP_TRY(row.floats(ns > nd ? ns : nd));
    PQP_TRY(terms.floats(5));
    float* T = terms.f();
    PQP_TRY(dev_matmul(row.f(), x, 1, Mp1, 0, 1, ns, ns, s));     // x' Mp1
    PQP_TRY(dev_matmul(T + 0, row.f(), 0, x, 0, 1, ns, 1, s));    //  . x
    PQP_TRY(dev_matmul(row.f(), D, 1, Mp2, 0, 1, nd, ns, s));     // D' Mp2
    PQP_TRY(dev_matmul(T + 1, row.f(), 0, x, 0, 1, ns, 1, s));    //  . x
    PQP_TRY(dev_matmul(T + 2, Mp4, 1, x, 0, 1, ns, 1, s));        // Mp4' x
    PQP_TRY(dev_matmul(row.f(), D, 1, Mp3, 0, 1, nd, nd, s));     // D' Mp3
    PQP_TRY(dev_matmul(T + 3, row.f(), 0, D, 0, 1, nd, 1, s));    //  . D
    PQP_TRY(dev_matmul(T + 4, Mp5, 1, D, 0, 1, nd, 1, s));        // Mp5' D
    PQP_HIP(launch_mp_finish(T, Mp6, Mp, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

// Gauss_Jordan (PQP_CPU.c:251-326)
int dev_gauss_jordan(float* res, const float* A, int n, hipStream_t s) {
    DevBuf aug, fac;
    PQP_TRY(aug.floats(gauss_jordan_aug_floats(n)));
    PQP_TRY(fac.floats(n));
    PQP_HIP(launch_gauss_jordan(A, aug.f(), fac.f(), res, n, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

// ---- single-problem solve ---------------------------------------------------
struct SolveOut {
    long long h = 0;
    float Jp = NAN, Jd = NAN;
    int have_costs = 0, last_stop = 0, status = 0;
    bool staged = false;  // Y (and U) already copied to the problem's pinned staging buffer
};

}  // namespace
}  // namespace pqp

// A dual problem resident in HBM, prepared once and solved any number of times
// (include/pqp.h: pqp_problem_create / _solve / _destroy).  Bound to the
// device it was made on and to its own stream; calls on one handle are
// serialized by its own lock, calls on different handles run concurrently
// (the reference's solver keeps no globals, PQP_CPU.c:694).
struct pqp_problem {
    int N = 0, M = 0;
    int dev = -1;                 // the device every call of this handle runs on
    hipStream_t stream = nullptr; // the handle's stream (owned unless the caller passed one)
    bool own_stream = false;
    std::mutex mu;
    bool small = false;  // fits k_solve_small (everything staged in LDS)
    pqp::DevBuf Qd, Fd, Md, Qp, Qinv, Fp, Mp, Gp, Kp;  // row-major device copies
    pqp::DevBuf QdT, theta;                          // large path only
    pqp::DevBuf SP, fdpn, Yb;                        // large path, fixed mode (built on first use)
    pqp::DevBuf rerr;                                // sticky relay hand-off error word (relay / graph paths)
    pqp::DevBuf SPp, fdpnp, gran, perr;              // persistent fixed mode: split matrices (lw = 32), y granules, error word
    int split_lw = 0;                                // lanes per workgroup SP was built with
    bool split_lean = false;                         // SP holds Qd packets (k_lean_relay), not the split matrices
    hipGraphExec_t graph = nullptr;                  // captured fixed-mode updates (the remainder)
    long long graph_updates = -1;
    hipGraphExec_t chunk_graph = nullptr;            // captured fixed-mode chunk of kFixedChunk updates
    bool chunk_ready = false;
    // converge mode over many workgroups (pqp_wide.hip), built on first use
    pqp::DevBuf QinvT, GpT, tM, tq, tu, gu, wflag, wcap;
    // converge mode as one persistent pipelined launch (pqp_converge.hip), built on first use
    pqp::DevBuf CA1, CA2, CA3, crings, cwords;
    hipGraphExec_t wgraph = nullptr;                 // captured chunk of converge iterations
    hipGraphExec_t wgraph_first = nullptr;           // the short first chunk
    hipGraphExec_t wgraph4 = nullptr, wgraph8 = nullptr;  // the chunks that escalate to kWideChunk
    long long wgraph_key = -1;
    long long graph_variant = -1;                    // the settings the fixed-mode graphs were captured with
    pqp::DevBuf Y, U, state;
    pqp::SolveState* hst = nullptr;                  // pinned host mirror of `state`
    float* hio = nullptr;                            // pinned staging of Y (N floats) then U (M floats)
    size_t hio_floats = 0;
    float* hin = nullptr;                            // pinned staging of small problems' inputs
    size_t hin_floats = 0;
    float* hout = nullptr;                           // pinned output of the one-launch tiny solves (kTinyOut* layout)
    unsigned out_tag = 0;                            // the last tag a tiny launch was given (1 .. 2^31 - 1)
    void* hout_dev = nullptr;                        // its device address
    ~pqp_problem() {
        if (own_stream && stream) (void)hipStreamDestroy(stream);
        if (graph) (void)hipGraphExecDestroy(graph);
        if (chunk_graph) (void)hipGraphExecDestroy(chunk_graph);
        if (wgraph) (void)hipGraphExecDestroy(wgraph);
        if (wgraph_first) (void)hipGraphExecDestroy(wgraph_first);
        if (wgraph4) (void)hipGraphExecDestroy(wgraph4);
        if (wgraph8) (void)hipGraphExecDestroy(wgraph8);
        if (hst) (void)hipHostFree(hst);
        if (hio) (void)hipHostFree(hio);
        if (hin) (void)hipHostFree(hin);
        if (hout) (void)hipHostFree(hout);
    }
};

// One row block of a large problem's stored split matrices (pqp_rowblock_*).
struct pqp_rowblock {
    int N = 0, row0 = 0, rows = 0, lw = 64;
    int dev = -1;  // the device it was made on (its calls run there)
    bool lean = false;  // SP holds Qd packets (k_lean_relay), fdpn the {Fdn, Fdp, Theta, 0} words
    pqp::DevBuf SP, fdpn;
    pqp::DevBuf err;    // sticky relay hand-off error word (pqp_rowblock_check)
};

namespace pqp {
Tuning g_tune;

namespace {

constexpr size_t kLdsBudget = 150 * 1024;
inline bool batch_unfused() { return (g_tune.batch_opts & 1) != 0; }

// Allocate the per-problem work buffers and, for the large path, the
// column-major copy and theta.  The nine input buffers must already hold the
// problem.
int problem_finish(pqp_problem& P, hipStream_t s) {
    const int N = P.N, M = P.M;
    P.small = solve_small_lds_bytes(N, M) <= kLdsBudget;
    PQP_TRY(P.Y.floats(N));
    PQP_TRY(P.U.floats(M));
    // the state, then the int error word a one-launch tiny solve stores behind it (kTinyDevErr)
    PQP_TRY(P.state.alloc(sizeof(SolveState) + 16));
    PQP_HIP(hipMemsetAsync(P.state.p, 0, sizeof(SolveState) + 16, s));
    PQP_HIP(hipMemsetAsync(P.U.p, 0, sizeof(float) * M, s));
    if (!P.hst) PQP_HIP(hipHostMalloc((void**)&P.hst, sizeof(SolveState), hipHostMallocDefault));
    if (P.hio_floats < (size_t)N + M) {
        if (P.hio) (void)hipHostFree(P.hio);
        P.hio = nullptr;
        P.hio_floats = 0;
        PQP_HIP(hipHostMalloc((void**)&P.hio, sizeof(float) * ((size_t)N + M), hipHostMallocDefault));
        P.hio_floats = (size_t)N + M;
    }
    if (!P.small) {  // Theta for the large paths (computeTheta, PQP_CPU.c:503-519)
        PQP_TRY(P.theta.floats(N));
        PQP_HIP(launch_theta_rows(P.Qd.f(), N, N, N, P.theta.f(), s));
    }
    return PQP_OK;
}

// The one-workgroup solver's column-major copy of Qd, built on first use (the
// multi-workgroup paths do not need it).
int ensure_single(pqp_problem& P, hipStream_t s) {
    if (P.QdT.p) return PQP_OK;
    const int N = P.N, M = P.M, ldq = round4(N);
    if (solve_single_lds_bytes(ldq, round4(M)) > kLdsBudget)
        return set_error(PQP_ERR_ARG,
                         "N=%d, M=%d exceeds the one-workgroup solver's LDS budget (terminate() drop-in / resumed "
                         "solves); converge and fixed mode run over many workgroups", N, M);
    PQP_TRY(P.QdT.floats((size_t)N * ldq));
    PQP_HIP(launch_pack_colmajor(1, P.Qd.f(), N, (long long)N * N, P.QdT.f(), ldq, (long long)N * ldq, s));
    return PQP_OK;
}

// Drop everything derived from a problem's data (built on first use by the
// solve paths): called before new data goes into an existing handle.
void problem_reset_derived(pqp_problem& P) {
    for (DevBuf* b : {&P.QdT, &P.theta, &P.SP, &P.fdpn, &P.Yb, &P.rerr, &P.SPp, &P.fdpnp, &P.gran, &P.perr, &P.QinvT, &P.GpT,
                      &P.tM, &P.tq, &P.tu, &P.gu, &P.wflag, &P.wcap, &P.CA1, &P.CA2, &P.CA3, &P.crings, &P.cwords})
        b->reset();
    for (hipGraphExec_t* g : {&P.graph, &P.chunk_graph, &P.wgraph, &P.wgraph_first, &P.wgraph4, &P.wgraph8})
        if (*g) {
            (void)hipGraphExecDestroy(*g);
            *g = nullptr;
        }
    P.split_lw = 0;
    P.split_lean = false;
    P.graph_updates = -1;
    P.chunk_ready = false;
    P.graph_variant = -1;
    P.wgraph_key = -1;
}

int problem_upload(pqp_problem& P, const float* qd, const float* fd, const float* md, const float* qp,
                   const float* qinv, const float* fp, const float* mp, const float* gp, const float* kp, int N, int M,
                   hipStream_t s) {
    if (P.Qd.p) {  // new data into an existing handle
        PQP_HIP(hipStreamSynchronize(s));
        problem_reset_derived(P);
    }
    P.N = N;
    P.M = M;
    const size_t nn = (size_t)N * N, mm = (size_t)M * M, nm = (size_t)N * M;
    const size_t total = nn + N + 1 + 2 * mm + M + 1 + nm + N;
    if (total <= (size_t)1 << 18) {
        // small problems: every input through one pinned staging buffer, so
        // the nine H2D copies are asynchronous DMA instead of pageable copies
        if (P.hin_floats < total) {
            if (P.hin) (void)hipHostFree(P.hin);
            P.hin = nullptr;
            P.hin_floats = 0;
            PQP_HIP(hipHostMalloc((void**)&P.hin, sizeof(float) * total, hipHostMallocDefault));
            P.hin_floats = total;
        }
        float* h = P.hin;
        auto put = [&](DevBuf& d, const float* src, size_t n) -> int {
            std::memcpy(h, src, sizeof(float) * n);
            PQP_TRY(d.floats(n));
            PQP_HIP(hipMemcpyAsync(d.p, h, sizeof(float) * n, hipMemcpyHostToDevice, s));
            h += n;
            return PQP_OK;
        };
        PQP_TRY(put(P.Qd, qd, nn));
        PQP_TRY(put(P.Fd, fd, N));
        PQP_TRY(put(P.Md, md, 1));
        PQP_TRY(put(P.Qp, qp, mm));
        PQP_TRY(put(P.Qinv, qinv, mm));
        PQP_TRY(put(P.Fp, fp, M));
        PQP_TRY(put(P.Mp, mp, 1));
        PQP_TRY(put(P.Gp, gp, nm));
        PQP_TRY(put(P.Kp, kp, N));
        return problem_finish(P, s);
    }
    PQP_TRY(upload(P.Qd, qd, (size_t)N * N, s));
    PQP_TRY(upload(P.Fd, fd, N, s));
    PQP_TRY(upload(P.Md, md, 1, s));
    PQP_TRY(upload(P.Qp, qp, (size_t)M * M, s));
    PQP_TRY(upload(P.Qinv, qinv, (size_t)M * M, s));
    PQP_TRY(upload(P.Fp, fp, M, s));
    PQP_TRY(upload(P.Mp, mp, 1, s));
    PQP_TRY(upload(P.Gp, gp, (size_t)N * M, s));
    PQP_TRY(upload(P.Kp, kp, N, s));
    return problem_finish(P, s);
}

// Run the persistent solve kernel until it reports Done/Capped.  Each launch
// is bounded (chunk updates) so no launch runs unbounded.  `resume` = start
// from P.Y instead of Y = 1000 (used by the terminate() drop-in, mode 2).
// Fixed mode of a large problem: one multi-workgroup launch per update
// (k_split_update), the stored split matrices built once per problem.
// Lanes per workgroup of the relay update of an n_dual = N problem: row sides
// of the stored split matrices, or rows of Qd for the lean relay.
int pick_lw(int N) { return use_lean(N, N) ? lean_pick_lw(N) : split_pick_lw(N); }

// The relay update's operand of the whole problem (rows 0..N-1), built on
// first use (and rebuilt if lw or the layout changes): the stored split
// matrices with lw row sides per workgroup, or, from n_dual >= g_tune.lean_min_n,
// Qd itself with lw rows per workgroup (k_lean_relay, half the bytes).
int ensure_split(pqp_problem& P, int lw, hipStream_t s) {
    const int N = P.N;
    const bool lean = use_lean(N, N);
    if (P.SP.p && P.split_lw == lw && P.split_lean == lean) return PQP_OK;
    if (split_lds_bytes(N) > kLdsBudget)
        return set_error(PQP_ERR_ARG, "multi-workgroup solve: N=%d needs more than %zu B of LDS", N, kLdsBudget);
    if (!P.theta.p) {  // small problems skip the large-path setup of problem_finish
        PQP_TRY(P.theta.floats(N));
        PQP_HIP(launch_theta_rows(P.Qd.f(), N, N, N, P.theta.f(), s));
    }
    PQP_TRY(P.Yb.floats(N));
    if (!P.rerr.p) {
        PQP_TRY(P.rerr.alloc(sizeof(int)));
        PQP_HIP(hipMemsetAsync(P.rerr.p, 0, sizeof(int), s));
    }
    if (lean) {
        PQP_TRY(P.SP.floats(lean_floats(N, N, lw)));
        PQP_TRY(P.fdpn.floats(lean_aux_floats(N, N, lw)));
        PQP_HIP(hipMemsetAsync(P.SP.p, 0, sizeof(float) * lean_floats(N, N, lw), s));
        PQP_HIP(launch_build_lean(P.Qd.f(), N, P.theta.f(), P.Fd.f(), N, N, 0, lw, P.SP.f(), P.fdpn.f(), s));
    } else {
        PQP_TRY(P.SP.floats(split_floats(N, N, lw)));
        PQP_TRY(P.fdpn.floats((size_t)2 * N));
        PQP_HIP(hipMemsetAsync(P.SP.p, 0, sizeof(float) * split_floats(N, N, lw), s));
        PQP_HIP(launch_build_split(P.Qd.f(), N, P.theta.f(), P.Fd.f(), N, N, 0, lw, P.SP.f(), P.fdpn.f(), s));
    }
    P.split_lw = lw;
    P.split_lean = lean;
    return PQP_OK;
}

// One relay update of the whole problem, a -> b, over the operand ensure_split built.
hipError_t problem_update(pqp_problem& P, int lw, const float* a, float* b, hipStream_t s, const int* gate = nullptr) {
    int* err = static_cast<int*>(P.rerr.p);
    return P.split_lean ? launch_lean_update(P.SP.f(), P.fdpn.f(), P.N, P.N, 0, lw, a, b, s, gate, err)
                        : launch_split_update(P.SP.f(), P.fdpn.f(), P.N, P.N, 0, lw, a, b, s, gate, err);
}

// The relay kernels' sticky error word: read (the caller synchronizes s
// after this call) and, when set, cleared and turned into PQP_ERR_HIP.
int relay_error_check(DevBuf& word, int* host, hipStream_t s, const char* what) {
    PQP_HIP(hipStreamSynchronize(s));
    if (*host) {
        const int code = *host;
        *host = 0;
        PQP_HIP(hipMemsetAsync(word.p, 0, sizeof(int), s));
        PQP_HIP(hipStreamSynchronize(s));
        return set_error(PQP_ERR_HIP, "%s: a relay hand-off wait expired (code %d); the result is not valid", what,
                         code);
    }
    return PQP_OK;
}

// Capture `n` dependent updates P.Y -> P.Yb -> P.Y ... into *exec (plus a
// copy back into P.Y when n is odd).
static int capture_updates(pqp_problem& P, int lw, long long n, hipGraphExec_t* exec, hipStream_t s) {
    const int N = P.N;
    if (*exec) {
        (void)hipGraphExecDestroy(*exec);
        *exec = nullptr;
    }
    hipGraph_t g = nullptr;
    PQP_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    float* a = P.Y.f();
    float* b = P.Yb.f();
    hipError_t e = hipSuccess;
    for (long long u = 0; u < n && e == hipSuccess; ++u) {
        e = problem_update(P, lw, a, b, s);
        std::swap(a, b);
    }
    if (e == hipSuccess && a != P.Y.f()) e = hipMemcpyAsync(P.Y.p, a, sizeof(float) * N, hipMemcpyDeviceToDevice, s);
    const hipError_t e2 = hipStreamEndCapture(s, &g);
    if (e != hipSuccess || e2 != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        PQP_HIP(e != hipSuccess ? e : e2);
    }
    const hipError_t e3 = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    PQP_HIP(e3);
    return PQP_OK;
}

// Fixed mode of a large problem: the relay update once per iteration, from
// hipGraphs (per-update host launch overhead would otherwise exceed the
// kernel itself): a chunk of kFixedChunk updates replayed as often as needed,
// then a graph of the remainder.
constexpr long long kFixedChunk = 256;  // even: a chunk starts and ends with the iterate in P.Y
// Fixed mode of a problem with N <= persist_max_n(): every update in ONE
// persistent launch (pqp_persist.hip), launches of at most kPersistChunk
// updates chained through P.Y.
constexpr long long kPersistChunk = 1 << 16;
// The stored split matrices in the 32-lane layout (k_build_split), built once
// per problem: the persistent fixed-mode launch and the persistent converge
// launch's update role hold them in LDS.
int ensure_persist_split(pqp_problem& P, hipStream_t s) {
    const int N = P.N;
    if (P.SPp.p) return PQP_OK;
    if (!P.theta.p) {
        PQP_TRY(P.theta.floats(N));
        PQP_HIP(launch_theta_rows(P.Qd.f(), N, N, N, P.theta.f(), s));
    }
    if (!P.Yb.p) PQP_TRY(P.Yb.floats(N));
    PQP_TRY(P.SPp.floats(split_floats(N, N, 32)));
    PQP_TRY(P.fdpnp.floats((size_t)2 * N));
    PQP_HIP(hipMemsetAsync(P.SPp.p, 0, sizeof(float) * split_floats(N, N, 32), s));
    PQP_HIP(launch_build_split(P.Qd.f(), N, P.theta.f(), P.Fd.f(), N, N, 0, 32, P.SPp.f(), P.fdpnp.f(), s));
    PQP_TRY(P.gran.alloc(sizeof(unsigned long long) * 2 * N));
    PQP_TRY(P.perr.alloc(sizeof(int)));
    return PQP_OK;
}

// Which solver the last single-problem solve ran (pqp_tune_get("last_path")), and
// how many persistent launches fell back to the relay / graph path.
enum SolvePath : int {
    kPathFixedPersist = 1, kPathFixedRelay = 2, kPathConvergePersist = 3, kPathConvergeWide = 4, kPathOneWorkgroup = 5
};
thread_local int g_last_path = 0;               // of the calling thread's last solve
std::atomic<long long> g_persist_fallbacks{0};
std::atomic<long long> g_tiny_stale{0};  // tiny solves whose pinned output did not carry their tag
// problem_run_*_persist: a wait of the persistent launch expired (its
// workgroups were not all resident); the caller falls back
constexpr int kPersistStalled = 1;

// A persistent launch needs every one of its workgroups resident at once (they
// wait on each other).  Two of them from different handles on one device could
// each get part of the CUs and wait for the rest until their deadline, so the
// persistent launches of one device run one at a time; everything else of
// different handles runs concurrently.
std::mutex& persist_lock() {
    static std::mutex mu[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    return mu[dev >= 0 && dev < 64 ? dev : 0];
}

int problem_run_fixed_persist(pqp_problem& P, long long updates, SolveOut& out, hipStream_t s) {
    const int N = P.N;
    PQP_TRY(ensure_persist_split(P, s));
    auto* gran = static_cast<unsigned long long*>(P.gran.p);
    int* err = static_cast<int*>(P.perr.p);
    PQP_HIP(launch_fill(P.Y.f(), 1000.0f, N, s));  // initMat(Y, 1000) :710
    std::lock_guard<std::mutex> one_at_a_time(persist_lock());
    for (long long done = 0; done < updates;) {
        const long long n = std::min(kPersistChunk, updates - done);
        // the launch reads its initial iterate from Yb while it writes P.Y
        PQP_HIP(hipMemcpyAsync(P.Yb.p, P.Y.p, sizeof(float) * N, hipMemcpyDeviceToDevice, s));
        PQP_HIP(launch_split_persist(P.SPp.f(), P.fdpnp.f(), N, (int)n, P.Yb.f(), P.Y.f(), gran, err, s));
        int herr = 0;
        PQP_HIP(hipMemcpyAsync(&herr, err, sizeof herr, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipStreamSynchronize(s));
        if (herr) {  // not all workgroups resident (other work on the device): fall back
            set_error(PQP_ERR_HIP, "persistent fixed-mode update: workgroup hand-off timed out (code %d); "
                      "its %d workgroups must be resident at once", herr, (2 * N + 31) / 32);
            return kPersistStalled;
        }
        done += n;
    }
    PQP_HIP(hipStreamSynchronize(s));
    out.h = updates + 1;
    out.status = kStatusDone;
    g_last_path = kPathFixedPersist;
    return PQP_OK;
}

int problem_run_fixed_split(pqp_problem& P, long long num_iter, SolveOut& out, hipStream_t s) {
    const int N = P.N;
    const long long updates = num_iter > 1 ? num_iter - 1 : 0;  // while(h < NUM_ITER)
    // one persistent launch when its workgroups can all be resident; if one of
    // its waits still expires (CUs held by other work), the solve restarts on
    // the graph-replayed relay below (fixed mode restarts from Y = 1000)
    if (!g_tune.persist_off && N <= persist_max_n() && split_persist_fits(N)) {
        const int rc = problem_run_fixed_persist(P, updates, out, s);
        if (rc != kPersistStalled) return rc;
        ++g_persist_fallbacks;
    }
    const int lw = pick_lw(N);
    PQP_TRY(ensure_split(P, lw, s));
    // every setting the captured launches bake in as an argument, the relay
    // wait budget's value included
    const long long variant = ((long long)lw << 8) | ((long long)use_lean(N, N) << 16) |
                              ((long long)(unsigned)g_tune.relay_spin_max << 24);
    if (P.graph_variant != variant) {  // kernel selection changed: recapture both
        P.graph_updates = -1;
        P.chunk_ready = false;
        P.graph_variant = variant;
    }
    const long long full = updates / kFixedChunk, rem = updates % kFixedChunk;
    if (full > 0 && !P.chunk_ready) {
        PQP_TRY(capture_updates(P, lw, kFixedChunk, &P.chunk_graph, s));
        P.chunk_ready = true;
    }
    if (rem > 0 && P.graph_updates != rem) {
        PQP_TRY(capture_updates(P, lw, rem, &P.graph, s));
        P.graph_updates = rem;
    }
    PQP_HIP(launch_fill(P.Y.f(), 1000.0f, N, s));  // initMat(Y, 1000) :710
    for (long long c = 0; c < full; ++c) PQP_HIP(hipGraphLaunch(P.chunk_graph, s));
    if (rem > 0) PQP_HIP(hipGraphLaunch(P.graph, s));
    int herr = 0;
    PQP_HIP(hipMemcpyAsync(&herr, P.rerr.p, sizeof herr, hipMemcpyDeviceToHost, s));
    PQP_TRY(relay_error_check(P.rerr, &herr, s, "fixed-mode relay update"));
    out.h = updates + 1;
    out.status = kStatusDone;
    g_last_path = kPathFixedRelay;
    return PQP_OK;
}

// Converge mode of a large problem over many workgroups (pqp_wide.hip): one
// iteration = terminate() as three multi-workgroup mat-vec launches and a
// one-workgroup decision, then the relay update.  A chunk of kWideChunk
// iterations is captured into a hipGraph and replayed until the device-side
// status leaves Continue; launches after that point return at once.
// Converge mode of a problem with N, M <= 1024 as ONE persistent launch
// (pqp_converge.hip): the update and the stages of terminate() run as
// concurrent roles, terminate(Y_u) beside the update to Y_{u+1}.  Launches
// decide at most g_tune.converge_chunk iterates each and are chained through P.Y.
bool converge_persist_fits(int N, int M) {
    if (g_tune.converge_persist_off) return false;
    const int G = converge_persist_wgs(N, M, nullptr);
    if (G == 0) return false;
    int dev = 0, cus = 0, lds = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) return false;
    if (converge_persist_lds_bytes(N, M) > (size_t)lds) return false;
    if (g_tune.persist_fit_cus > 0) cus = g_tune.persist_fit_cus;
    // every workgroup of the launch resident at once (its roles wait on each other)
    return (long long)converge_persist_per_cu(N, M) * cus >= G;
}

int problem_run_converge_persist(pqp_problem& P, long long max_updates, SolveOut& out, hipStream_t s) {
    const int N = P.N, M = P.M;
    PQP_TRY(ensure_persist_split(P, s));
    if (!P.CA1.p) {
        const size_t n1 = converge_stage_floats(N, M, 1), n2 = converge_stage_floats(N, M, 2),
                     n3 = converge_stage_floats(N, M, 3);
        PQP_TRY(P.CA1.floats(n1));
        PQP_TRY(P.CA2.floats(n2));
        PQP_TRY(P.CA3.floats(n3));
        PQP_HIP(hipMemsetAsync(P.CA1.p, 0, sizeof(float) * n1, s));
        PQP_HIP(hipMemsetAsync(P.CA2.p, 0, sizeof(float) * n2, s));
        PQP_HIP(hipMemsetAsync(P.CA3.p, 0, sizeof(float) * n3, s));
        PQP_HIP(launch_converge_pack(P.Qd.f(), P.Gp.f(), P.Qinv.f(), P.Qp.f(), N, M, P.CA1.f(), P.CA2.f(), P.CA3.f(),
                                     s));
        PQP_TRY(P.crings.alloc(sizeof(unsigned long long) * converge_ring_words(N, M)));
        PQP_TRY(P.cwords.alloc(32));  // ctl, err (int), decided (long long)
    }
    SolveState& st = *P.hst;
    st = SolveState{};
    st.h = 1;
    st.status = kStatusContinue;
    SolveState* dst = static_cast<SolveState*>(P.state.p);
    PQP_HIP(hipMemcpyAsync(dst, &st, sizeof st, hipMemcpyHostToDevice, s));
    PQP_HIP(launch_fill(P.Y.f(), 1000.0f, N, s));  // initMat(Y, 1000) :710
    char* words = static_cast<char*>(P.cwords.p);
    ConvergeLaunch L{};
    L.N = N;
    L.M = M;
    L.chunk = g_tune.converge_chunk;
    L.cap = max_updates;
    L.SP = P.SPp.f();
    L.A1 = P.CA1.f();
    L.A2 = P.CA2.f();
    L.A3 = P.CA3.f();
    L.fdpn = P.fdpnp.f();
    L.Fp = P.Fp.f();
    L.Kp = P.Kp.f();
    L.Fd = P.Fd.f();
    L.Md = P.Md.f();
    L.Mp = P.Mp.f();
    L.rings = P.crings.p;
    L.st = dst;
    L.ctl = reinterpret_cast<int*>(words);
    L.err = reinterpret_cast<int*>(words + 4);
    L.decided = reinterpret_cast<long long*>(words + 8);
    L.Y = P.Y.f();
    L.U = P.U.f();
    std::lock_guard<std::mutex> one_at_a_time(persist_lock());
    for (long long u0 = 0;;) {
        L.u0 = u0;
        PQP_HIP(launch_converge_persist(L, s));
        int herr = 0;
        // Y and U ride with the state readback (pinned staging, one sync)
        PQP_HIP(hipMemcpyAsync(P.hio, P.Y.p, sizeof(float) * N, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipMemcpyAsync(P.hio + N, P.U.p, sizeof(float) * M, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipMemcpyAsync(&st, dst, sizeof st, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipMemcpyAsync(&herr, L.err, sizeof herr, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipStreamSynchronize(s));
        if (herr) {  // not all workgroups resident: the caller re-runs the solve on the graph chain
            set_error(PQP_ERR_HIP, "persistent converge launch: a wait timed out (code %d); its %d workgroups "
                      "must be resident at once", herr, converge_persist_wgs(N, M, nullptr));
            return kPersistStalled;
        }
        if (st.status != kStatusContinue) break;
        u0 = st.h - 1;  // the next launch starts from the iterate this one left in P.Y
    }
    out.staged = true;
    out.h = st.h;
    out.status = st.status;
    out.have_costs = st.have_costs;
    out.last_stop = 0;
    g_last_path = kPathConvergePersist;
    if (st.have_costs) {
        out.Jp = st.Jp;
        out.Jd = st.Jd;
    }
    return PQP_OK;
}

constexpr int kWideChunk = 16;      // even: each replay starts and ends with the iterate in P.Y
constexpr int kWideFirstChunk = 2;  // the first replay of a solve
int problem_run_wide(pqp_problem& P, long long max_updates, SolveOut& out, hipStream_t s, bool try_persist = true) {
    const int N = P.N, M = P.M;
    if (try_persist && converge_persist_fits(N, M)) {
        const int rc = problem_run_converge_persist(P, max_updates, out, s);
        if (rc != kPersistStalled) return rc;
        ++g_persist_fallbacks;  // converge mode restarts from Y = 1000 on the graph chain
    }
    const int lw = pick_lw(N);
    PQP_TRY(ensure_split(P, lw, s));
    if (!P.QinvT.p) {
        PQP_TRY(P.QinvT.floats((size_t)M * M));
        PQP_TRY(P.GpT.floats((size_t)M * N));
        PQP_TRY(P.tM.floats(M));
        PQP_TRY(P.tq.floats(N));
        PQP_TRY(P.tu.floats(M));
        PQP_TRY(P.gu.floats(N));
        PQP_TRY(P.wflag.alloc(sizeof(int)));
        PQP_TRY(P.wcap.alloc(sizeof(long long)));
        PQP_HIP(launch_transpose(P.Qinv.f(), M, M, P.QinvT.f(), s));  // QinvT[k][i] = Qp_inv[i][k]
        PQP_HIP(launch_transpose(P.Gp.f(), N, M, P.GpT.f(), s));      // GpT[k][i] = Gp[i][k]
    }
    SolveState* dst = static_cast<SolveState*>(P.state.p);
    int* flag = static_cast<int*>(P.wflag.p);
    long long* cap = static_cast<long long*>(P.wcap.p);
    // every launch argument the capture bakes in (cap: a device word)
    const long long key = (long long)(((unsigned long long)(unsigned)g_tune.relay_spin_max << 32) |
                                      ((unsigned long long)use_lean(N, N) << 24) | (unsigned long long)(lw & 0xff));
    int* rerr = static_cast<int*>(P.rerr.p);
    if (!P.wgraph || P.wgraph_key != key) {
        if (P.wgraph) {
            (void)hipGraphExecDestroy(P.wgraph);
            P.wgraph = nullptr;
        }
        // One iteration: terminate()'s launches, then the update, each gated on
        // the status word (once an iteration stops or hits the cap, the rest do
        // nothing).  The update on a forked graph branch beside terminate()
        // measured slower and was removed in round 4.
        auto iteration = [&](const float* cur, float* nxt) -> hipError_t {
            hipError_t e = hipSuccess;
            GemvJobs j1{};  // tmp = Gp'Y + Fp (computeUfromY :354-356) and Y'Qd (computeCost :652, Jd)
            j1.job[0] = GemvJob{P.Gp.f(), cur, P.tM.f(), P.Fp.f(), M, N, M, kEpiAdd};
            j1.job[1] = GemvJob{P.Qd.f(), cur, P.tq.f(), nullptr, N, N, N, kEpiPlain};
            j1.gate = &dst->status;
            j1.err = rerr;
            if ((e = launch_gemv_relay(j1, s)) != hipSuccess) return e;
            GemvJobs j2{};  // U = -(Qp_inv tmp) (:357-358)
            j2.job[0] = GemvJob{P.QinvT.f(), P.tM.f(), P.U.f(), nullptr, M, M, M, kEpiNeg};
            j2.gate = &dst->status;
            j2.err = rerr;
            if ((e = launch_gemv_relay(j2, s)) != hipSuccess) return e;
            GemvJobs j3{};  // checkFeas (:632-641) and U'Qp (computeCost, Jp)
            j3.job[0] = GemvJob{P.GpT.f(), P.U.f(), P.gu.f(), P.Kp.f(), N, M, N, kEpiFeas};
            j3.job[1] = GemvJob{P.Qp.f(), P.U.f(), P.tu.f(), nullptr, M, M, M, kEpiPlain};
            j3.gate = &dst->status;
            j3.flag = flag;
            j3.err = rerr;
            if ((e = launch_gemv_relay(j3, s)) != hipSuccess) return e;
            const WideArgs w{dst, flag, P.tq.f(), P.tu.f(), cur, P.U.f(), P.Fd.f(), P.Fp.f(), P.Md.f(), P.Mp.f(),
                             N, M, cap};
            if ((e = launch_wide_decide(w, s)) != hipSuccess) return e;
            return problem_update(P, lw, cur, nxt, s, &dst->status);
        };
        // replays of 2, 2, 4, 8, then kWideChunk iterations: a solve that stops
        // early launches at most about as many no-op iterations as it ran
        auto capture = [&](int iters, hipGraphExec_t* exec) -> int {
            hipGraph_t g = nullptr;
            PQP_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            hipError_t e = hipSuccess;
            for (int it = 0; it < iters && e == hipSuccess; it += 2) {
                e = iteration(P.Y.f(), P.Yb.f());
                if (e == hipSuccess) e = iteration(P.Yb.f(), P.Y.f());
            }
            const hipError_t e2 = hipStreamEndCapture(s, &g);
            if (e != hipSuccess || e2 != hipSuccess) {
                if (g) (void)hipGraphDestroy(g);
                PQP_HIP(e != hipSuccess ? e : e2);
            }
            const hipError_t e3 = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            PQP_HIP(e3);
            return PQP_OK;
        };
        for (hipGraphExec_t* g : {&P.wgraph_first, &P.wgraph4, &P.wgraph8})
            if (*g) {
                (void)hipGraphExecDestroy(*g);
                *g = nullptr;
            }
        PQP_TRY(capture(kWideFirstChunk, &P.wgraph_first));
        PQP_TRY(capture(4, &P.wgraph4));
        PQP_TRY(capture(8, &P.wgraph8));
        PQP_TRY(capture(kWideChunk, &P.wgraph));
        P.wgraph_key = key;
    }
    PQP_HIP(launch_wide_init(dst, flag, cap, max_updates, P.Y.f(), N, s));
    SolveState& st = *P.hst;
    for (int launch = 0;; ++launch) {
        hipGraphExec_t g = launch < 2 ? P.wgraph_first : (launch == 2 ? P.wgraph4 : (launch == 3 ? P.wgraph8 : P.wgraph));
        PQP_HIP(hipGraphLaunch(g, s));
        PQP_HIP(hipMemcpyAsync(&st, dst, sizeof st, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipStreamSynchronize(s));
        if (st.status != kStatusContinue) break;
    }
    if ((st.h - 1) & 1)  // odd number of updates: the iterate is in Yb
        PQP_HIP(hipMemcpyAsync(P.Y.p, P.Yb.p, sizeof(float) * N, hipMemcpyDeviceToDevice, s));
    int herr = 0;
    PQP_HIP(hipMemcpyAsync(&herr, rerr, sizeof herr, hipMemcpyDeviceToHost, s));
    PQP_TRY(relay_error_check(P.rerr, &herr, s, "converge-mode relay chain"));
    g_last_path = kPathConvergeWide;
    out.h = st.h;
    out.status = st.status;
    out.have_costs = st.have_costs;
    out.last_stop = st.last_stop;
    if (st.have_costs) {
        out.Jp = st.Jp;
        out.Jd = st.Jd;
    }
    return PQP_OK;
}

// One small problem (N, M <= 32) from Y = 1000 in ONE launch (pqp_tiny.hip:
// k_fixed_one / k_solve_quintet): the kernel starts from h = 1 itself (no state
// upload) and writes Y, U, the state and its error word to pinned host memory,
// so a solve is one launch and one synchronisation, no copy kernels.
int problem_run_tiny(pqp_problem& P, int mode, long long num_iter, long long max_updates, SolveOut& out,
                     hipStream_t s) {
    const int N = P.N, M = P.M;
    if (!P.hout) {
        // fine-grained (coherent) host memory: the kernel's stores reach it
        // without a cache write-back at the kernel's end
        PQP_HIP(hipHostMalloc((void**)&P.hout, sizeof(float) * kTinyOutFloats,
                              hipHostMallocMapped | hipHostMallocCoherent));
        PQP_HIP(hipHostGetDevicePointer(&P.hout_dev, P.hout, 0));
        std::memset(P.hout, 0, sizeof(float) * kTinyOutFloats);  // tag 0: no launch's
    }
    SolveArgs a{};
    a.Qd = P.Qd.f();
    a.Fd = P.Fd.f();
    a.Md = P.Md.f();
    a.Qp = P.Qp.f();
    a.Qinv = P.Qinv.f();
    a.Fp = P.Fp.f();
    a.Mp = P.Mp.f();
    a.Gp = P.Gp.f();
    a.Kp = P.Kp.f();
    a.Y = P.Y.f();
    a.U = P.U.f();
    a.N = N;
    a.M = M;
    a.ldq = round4(N);
    a.ldm = round4(M);
    a.mode = mode;
    a.num_iter = num_iter;
    a.max_updates = max_updates;
    // iterates per launch: about 2^26 element updates (28.5 k at the bundled
    // size, so its solves stay one launch), bounded so that a long fixed-mode
    // solve or an uncapped converge solve is a sequence of launches that
    // resume from the device state, not one kernel running for minutes
    // (ADVICE r5); the tiny_chunk knob sets it for the resume tests
    const double per_update = 3.0 * N * N + 2.0 * N * M + 2.0 * M * M + 1.0;
    a.chunk = g_tune.tiny_chunk > 0 ? g_tune.tiny_chunk : std::max(1024LL, (long long)((1 << 26) / per_update));
    a.fresh = 1;
    a.hout = P.hout_dev;
    a.tiny_flags = (g_tune.tiny_dense ? kTinyDense : 0) | (g_tune.tiny_stall ? kTinyStall : 0);
    a.trace = g_tune.tiny_trace;  // k_solve_quintet timing (bundled size only): 4 words per wave
    SolveState* dst = static_cast<SolveState*>(P.state.p);
    const SolveState* hs = reinterpret_cast<const SolveState*>(P.hout + kTinyOutStateOffset);
    const int* herr = reinterpret_cast<const int*>(P.hout) + kTinyOutErrOffset;
    volatile const int* htag = reinterpret_cast<const int*>(P.hout) + kTinyOutTagOffset;
    for (;;) {
        P.out_tag = (P.out_tag + 1) & 0x7fffffffu;  // positive, never 0 (the zeroed buffer's tag)
        if (P.out_tag == 0) P.out_tag = 1;
        a.out_tag = (int)P.out_tag;
        PQP_HIP(launch_one_tiny(a, dst, s));
        // (polling hipStreamQuery instead measured 2 us slower per solve, 17.7 vs
        // 12.2 us for a bare launch: profiles/r06/doorbell_r06e.json)
        PQP_HIP(hipStreamSynchronize(s));
        if (*htag != a.out_tag || g_tune.tiny_fallback) {
            // not this launch's output (never seen so far; the tiny_fallback
            // knob forces this path in tests): read the device copies instead --
            // Y, U, the state and the error word behind it
            ++g_tiny_stale;
            PQP_HIP(hipMemcpyAsync(P.hout, P.Y.p, sizeof(float) * N, hipMemcpyDeviceToHost, s));
            if (mode == kModeConverge)
                PQP_HIP(hipMemcpyAsync(P.hout + kTinyOutUOffset, P.U.p, sizeof(float) * M, hipMemcpyDeviceToHost, s));
            PQP_HIP(hipMemcpyAsync(P.hout + kTinyOutStateOffset, dst, sizeof(SolveState), hipMemcpyDeviceToHost, s));
            PQP_HIP(hipMemcpyAsync(P.hout + kTinyOutErrOffset, reinterpret_cast<const char*>(dst) + kTinyDevErr,
                                   sizeof(int), hipMemcpyDeviceToHost, s));
            PQP_HIP(hipStreamSynchronize(s));
        }
        if (*herr) return set_error(PQP_ERR_HIP, "k_solve_quintet: a wave's hand-off wait expired (N=%d, M=%d)", N, M);
        if (hs->status != kStatusContinue) break;
        a.fresh = 0;  // (a chunk ran out) resume from the device state
    }
    std::memcpy(P.hio, P.hout, sizeof(float) * N);
    if (mode == kModeConverge) std::memcpy(P.hio + N, P.hout + kTinyOutUOffset, sizeof(float) * M);
    out.staged = true;
    out.h = hs->h;
    out.status = hs->status;
    out.have_costs = hs->have_costs;
    out.last_stop = hs->last_stop;
    if (hs->have_costs) {
        out.Jp = hs->Jp;
        out.Jd = hs->Jd;
    }
    g_last_path = kPathOneWorkgroup;
    return PQP_OK;
}

int problem_run(pqp_problem& P, int mode, long long num_iter, long long max_updates, bool resume, SolveOut& out,
                hipStream_t s) {
    const int N = P.N, M = P.M;
    if (mode == kModeFixed && !P.small && !g_tune.force_single && !resume) return problem_run_fixed_split(P, num_iter, out, s);
    if (mode == kModeConverge && !g_tune.force_single && !resume) {
        // the one-wave solver stays fastest for N, M <= 32 (0.65 us per iteration
        // at 32/16 against 2.3 on the persistent launch); from n_dual 48 up the
        // persistent launch wins (scripts/converge_crossover.py)
        const bool tiny = N <= 32 && M <= 32 && !g_tune.force_small;
        const bool wide_ok = N >= g_tune.wide_min_n && (!P.small || g_tune.wide_min_n <= 0);
        if (!tiny && converge_persist_fits(N, M)) {
            const int rc = problem_run_converge_persist(P, max_updates, out, s);
            if (rc != kPersistStalled) return rc;
            ++g_persist_fallbacks;  // the solve restarts from Y = 1000 below
            if (wide_ok) return problem_run_wide(P, max_updates, out, s, false);
        } else if (wide_ok) {
            return problem_run_wide(P, max_updates, out, s);
        }
    }
    if (!resume && !g_tune.tiny_old && N <= 32 && M <= 32 && !g_tune.force_small && !g_tune.force_single &&
        (mode == kModeFixed || (mode == kModeConverge && N + M < 64)))
        return problem_run_tiny(P, mode, num_iter, max_updates, out, s);
    if (!P.small) PQP_TRY(ensure_single(P, s));
    SolveState& st = *P.hst;
    st = SolveState{};
    st.h = 1;
    st.resume = resume ? 1 : 0;
    PQP_HIP(hipMemcpyAsync(P.state.p, &st, sizeof st, hipMemcpyHostToDevice, s));
    SolveArgs a{};
    a.QdT = P.QdT.f();
    a.Qd = P.Qd.f();
    a.theta = P.theta.f();
    a.Fd = P.Fd.f();
    a.Md = P.Md.f();
    a.Qp = P.Qp.f();
    a.Qinv = P.Qinv.f();
    a.Fp = P.Fp.f();
    a.Mp = P.Mp.f();
    a.Gp = P.Gp.f();
    a.Kp = P.Kp.f();
    a.Y = P.Y.f();
    a.U = P.U.f();
    a.N = N;
    a.M = M;
    a.ldq = round4(N);
    a.ldm = round4(M);
    a.mode = mode;
    a.num_iter = num_iter;
    a.max_updates = max_updates;
    const double per_update = (double)N * N * 3.0 + 2.0 * N * M + 2.0 * M * M + 1.0;
    const long long chunk = (long long)((double)(1 << 26) / per_update);
    a.chunk = chunk < 1 ? 1 : chunk;
    SolveState* dst = static_cast<SolveState*>(P.state.p);
    for (;;) {
        if (P.N <= 32 && P.M <= 32 && !g_tune.force_small)
            PQP_HIP(launch_solve_tiny(a, dst, s));
        else if (P.small)
            PQP_HIP(launch_solve_small(a, dst, s));
        else
            PQP_HIP(launch_solve_single(a, dst, s));
        // Y and U ride with the state readback (pinned, one sync per launch);
        // the copies of the launch that finishes are the ones that stand
        PQP_HIP(hipMemcpyAsync(P.hio, P.Y.p, sizeof(float) * N, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipMemcpyAsync(P.hio + N, P.U.p, sizeof(float) * M, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipMemcpyAsync(&st, dst, sizeof st, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipStreamSynchronize(s));
        if (st.status != kStatusContinue) break;
    }
    out.staged = true;
    out.h = st.h;
    out.status = st.status;
    out.have_costs = st.have_costs;
    out.last_stop = st.last_stop;
    g_last_path = kPathOneWorkgroup;
    if (st.have_costs) {
        out.Jp = st.Jp;
        out.Jd = st.Jd;
    }
    return PQP_OK;
}

[[noreturn]] void die(const char* fn) {
    std::fprintf(stderr, "libpqp: %s failed: %s\n", fn, pqp_last_error());
    std::exit(EXIT_FAILURE);
}

int check_dims(int N, int M) {
    if (N <= 0 || M <= 0) return set_error(PQP_ERR_ARG, "N and M must be positive (N=%d, M=%d)", N, M);
    return PQP_OK;
}

}  // namespace
}  // namespace pqp

using namespace pqp;

extern "C" {

int pqp_version(void) { return 106; }  // ABI revision: INTEGRATION.md section 6

// ---------------------------------------------------------------------------
// 2a. status-returning host API
// ---------------------------------------------------------------------------
int pqp_problem_create_on(int device, void* stream, const float* Qd, const float* Fd, const float* Md,
                          const float* Qp, const float* Qp_inv, const float* Fp, const float* Mp, const float* Gp,
                          const float* Kp, int N, int M, pqp_problem** out) {
    if (!out) return set_error(PQP_ERR_ARG, "pqp_problem_create: null handle pointer");
    *out = nullptr;
    PQP_TRY(check_dims(N, M));
    if (!Qd || !Fd || !Md || !Qp || !Qp_inv || !Fp || !Mp || !Gp || !Kp)
        return set_error(PQP_ERR_ARG, "pqp_problem_create: null input");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return set_error(PQP_ERR_NO_DEVICE, "libpqp: no HIP device visible");
    if (device < 0 && hipGetDevice(&device) != hipSuccess)
        return set_error(PQP_ERR_NO_DEVICE, "libpqp: cannot query the current device");
    if (device >= n) return set_error(PQP_ERR_ARG, "pqp_problem_create_on: device %d of %d", device, n);
    DeviceGuard on(device);
    PQP_TRY(ensure_device());
    std::unique_ptr<pqp_problem> P(new pqp_problem());
    P->dev = device;
    if (stream) {
        hipDevice_t sdev = -1;
        PQP_HIP(hipStreamGetDevice(static_cast<hipStream_t>(stream), &sdev));
        if (sdev != device)
            return set_error(PQP_ERR_ARG, "pqp_problem_create_on: the stream belongs to device %d, not %d", (int)sdev,
                             device);
        P->stream = static_cast<hipStream_t>(stream);
    } else {
        PQP_HIP(hipStreamCreateWithFlags(&P->stream, hipStreamNonBlocking));
        P->own_stream = true;
    }
    hipStream_t s = P->stream;
    int rc = problem_upload(*P, Qd, Fd, Md, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M, s);
    if (rc == PQP_OK && hipStreamSynchronize(s) != hipSuccess) rc = set_error(PQP_ERR_HIP, "problem setup failed");
    if (rc != PQP_OK) return rc;
    *out = P.release();
    return PQP_OK;
}

int pqp_problem_create(const float* Qd, const float* Fd, const float* Md, const float* Qp, const float* Qp_inv,
                       const float* Fp, const float* Mp, const float* Gp, const float* Kp, int N, int M,
                       pqp_problem** out) {
    return pqp_problem_create_on(-1, nullptr, Qd, Fd, Md, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M, out);
}

int pqp_problem_device(const pqp_problem* P) { return P ? P->dev : set_error(PQP_ERR_ARG, "pqp_problem_device: null handle"); }

int pqp_problem_solve(pqp_problem* P, int mode, long long num_iter, long long max_updates, float* Y, float* U,
                      long long* h_out, float* Jp_out, float* Jd_out) {
    if (!P || !Y) return set_error(PQP_ERR_ARG, "pqp_problem_solve: null handle or Y");
    if (mode != PQP_MODE_CONVERGE && mode != PQP_MODE_FIXED)
        return set_error(PQP_ERR_ARG, "pqp_problem_solve: unknown mode %d", mode);
    std::lock_guard<std::mutex> lk(P->mu);
    DeviceGuard on(P->dev);
    PQP_TRY(ensure_device());
    hipStream_t s = P->stream;
    SolveOut o;
    PQP_TRY(problem_run(*P, mode == PQP_MODE_CONVERGE ? kModeConverge : kModeFixed, num_iter, max_updates, false, o,
                        s));
    const bool want_u = U && mode == PQP_MODE_CONVERGE;
    if (!o.staged) {  // through the pinned staging buffer: one sync, no pageable DMA
        PQP_HIP(hipMemcpyAsync(P->hio, P->Y.p, sizeof(float) * P->N, hipMemcpyDeviceToHost, s));
        if (want_u) PQP_HIP(hipMemcpyAsync(P->hio + P->N, P->U.p, sizeof(float) * P->M, hipMemcpyDeviceToHost, s));
        PQP_HIP(hipStreamSynchronize(s));
    }
    std::memcpy(Y, P->hio, sizeof(float) * P->N);
    if (want_u) std::memcpy(U, P->hio + P->N, sizeof(float) * P->M);
    if (h_out) *h_out = o.h;
    if (Jp_out) *Jp_out = o.Jp;
    if (Jd_out) *Jd_out = o.Jd;
    if (o.status == kStatusCapped)
        return set_error(PQP_ERR_NOT_CONVERGED, "no convergence within %lld updates (h=%lld)", max_updates, o.h);
    return PQP_OK;
}

int pqp_problem_destroy(pqp_problem* P) {
    if (!P) return PQP_OK;
    {
        std::lock_guard<std::mutex> lk(P->mu);  // a solve still running on another thread ends first
        DeviceGuard on(P->dev);
        if (P->stream) (void)hipStreamSynchronize(P->stream);
    }
    DeviceGuard on(P->dev);
    delete P;
    return PQP_OK;
}

static std::mutex g_oneshot_mu;              // guards g_oneshot
static pqp_problem* g_oneshot[64] = {nullptr};  // per device: cached handle of pqp_solve_dual's tiny problems

int pqp_solve_dual(const float* Qd, const float* Fd, const float* Md, const float* Qp, const float* Qp_inv,
                   const float* Fp, const float* Mp, const float* Gp, const float* Kp, int N, int M, int mode,
                   long long num_iter, long long max_updates, float* Y, float* U, long long* h_out,
                   float* Jp_out, float* Jd_out) {
    if (mode != PQP_MODE_CONVERGE && mode != PQP_MODE_FIXED)
        return set_error(PQP_ERR_ARG, "pqp_solve_dual: unknown mode %d", mode);
    if (!Y) return set_error(PQP_ERR_ARG, "pqp_solve_dual: null Y");
    if (N >= 1 && M >= 1 && N <= 32 && M <= 32) {
        // the one-shot form of tiny problems (the reference's own call
        // pattern, solveQuadraticDual per solve) reuses one cached handle: its
        // buffers are re-filled in place (no allocations), and these problems
        // build no derived per-problem data a new Qd could leave stale
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
            return set_error(PQP_ERR_NO_DEVICE, "libpqp: cannot query the current device");
        std::lock_guard<std::mutex> lk(g_oneshot_mu);
        pqp_problem*& h = g_oneshot[dev];
        if (!h) {
            PQP_TRY(pqp_problem_create(Qd, Fd, Md, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M, &h));
        } else {
            if (!Qd || !Fd || !Md || !Qp || !Qp_inv || !Fp || !Mp || !Gp || !Kp)
                return set_error(PQP_ERR_ARG, "pqp_solve_dual: null input");
            std::lock_guard<std::mutex> lk2(h->mu);
            PQP_TRY(ensure_device());
            PQP_TRY(problem_upload(*h, Qd, Fd, Md, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M, h->stream));
        }
        return pqp_problem_solve(h, mode, num_iter, max_updates, Y, U, h_out, Jp_out, Jd_out);
    }
    pqp_problem* P = nullptr;
    PQP_TRY(pqp_problem_create(Qd, Fd, Md, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M, &P));
    const int rc = pqp_problem_solve(P, mode, num_iter, max_updates, Y, U, h_out, Jp_out, Jd_out);
    const std::string err = pqp_last_error();
    pqp_problem_destroy(P);
    restore_error(err);
    return rc;
}

int pqp_update_host(const float* Qd, const float* theta_diag, const float* Fd, const float* Y, float* Y_next,
                    int N) {
    if (N <= 0 || !Qd || !theta_diag || !Fd || !Y || !Y_next) return set_error(PQP_ERR_ARG, "pqp_update_host");
    PQP_TRY(ensure_device());
    hipStream_t s = lib_stream();
    const int ldq = round4(N);
    DevBuf dQd, dQdT, dth, dFd, dY, dYn;
    PQP_TRY(upload(dQd, Qd, (size_t)N * N, s));
    PQP_TRY(upload(dth, theta_diag, N, s));
    PQP_TRY(upload(dFd, Fd, N, s));
    PQP_TRY(upload(dY, Y, N, s));
    PQP_TRY(dYn.floats(N));
    PQP_TRY(dQdT.floats((size_t)N * ldq));
    PQP_HIP(launch_pack_colmajor(1, dQd.f(), N, (long long)N * N, dQdT.f(), ldq, (long long)N * ldq, s));
    PQP_HIP(launch_batch_update(1, dQdT.f(), (long long)N * ldq, ldq, N, dth.f(), dFd.f(), N, dY.f(), dYn.f(), s));
    PQP_TRY(download(Y_next, dYn.p, N, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

int pqp_run_example(const char* dir, void* out_file) {
    FILE* out = out_file ? static_cast<FILE*>(out_file) : stdout;
    ExampleData e;
    const int m = kRefNInput * kRefPHorizon, nd = kRefNDis * kRefPHorizon, ns = kRefNState;
    PQP_TRY(read_example(dir, m, nd, ns, e));
    const int M = m, N = 4 * m;
    PQP_TRY(ensure_device());
    hipStream_t s = lib_stream();
    DevBuf Qinv, Fp1, Fp2, Fp3, Mp1, Mp2, Mp3, Mp4, Mp5, Mp6, Gp, Kp, x, D;
    PQP_TRY(upload(Qinv, e.Qp_inv.data(), e.Qp_inv.size(), s));
    PQP_TRY(upload(Fp1, e.Fp1.data(), e.Fp1.size(), s));
    PQP_TRY(upload(Fp2, e.Fp2.data(), e.Fp2.size(), s));
    PQP_TRY(upload(Fp3, e.Fp3.data(), e.Fp3.size(), s));
    PQP_TRY(upload(Mp1, e.Mp1.data(), e.Mp1.size(), s));
    PQP_TRY(upload(Mp2, e.Mp2.data(), e.Mp2.size(), s));
    PQP_TRY(upload(Mp3, e.Mp3.data(), e.Mp3.size(), s));
    PQP_TRY(upload(Mp4, e.Mp4.data(), e.Mp4.size(), s));
    PQP_TRY(upload(Mp5, e.Mp5.data(), e.Mp5.size(), s));
    PQP_TRY(upload(Mp6, e.Mp6.data(), e.Mp6.size(), s));
    PQP_TRY(upload(Gp, e.Gp.data(), e.Gp.size(), s));
    PQP_TRY(upload(Kp, e.Kp.data(), e.Kp.size(), s));
    PQP_TRY(upload(x, e.x.data(), e.x.size(), s));
    PQP_TRY(upload(D, e.D.data(), e.D.size(), s));
    pqp_problem P;
    P.N = N;
    P.M = M;
    DevBuf Jp, Jd;
    PQP_TRY(P.Qp.floats((size_t)M * M));
    PQP_TRY(P.Fp.floats(M));
    PQP_TRY(P.Mp.floats(1));
    PQP_TRY(P.Qd.floats((size_t)N * N));
    PQP_TRY(P.Fd.floats(N));
    PQP_TRY(P.Md.floats(1));
    PQP_TRY(Jp.floats(1));
    PQP_TRY(Jd.floats(1));
    std::swap(P.Qinv.p, Qinv.p);
    std::swap(P.Gp.p, Gp.p);
    std::swap(P.Kp.p, Kp.p);
    PQP_TRY(dev_gauss_jordan(P.Qp.f(), P.Qinv.f(), M, s));                                                // :989
    PQP_TRY(dev_compute_fp(P.Fp.f(), Fp1.f(), Fp2.f(), Fp3.f(), D.f(), x.f(), m, nd, ns, s));            // :991
    PQP_TRY(dev_compute_mp(P.Mp.f(), Mp1.f(), Mp2.f(), Mp3.f(), Mp4.f(), Mp5.f(), Mp6.f(), D.f(), x.f(), nd, ns,
                           s));                                                                         // :992
    PQP_TRY(dev_convert_to_dual(P.Qd.f(), P.Fd.f(), P.Md.f(), P.Qinv.f(), P.Gp.f(), P.Kp.f(), P.Fp.f(), P.Mp.f(), N,
                                M, s));                                                                 // :994
    PQP_TRY(problem_finish(P, s));
    SolveOut o;
    PQP_TRY(problem_run(P, kModeConverge, 0, 0, false, o, s));                                          // :996
    std::fprintf(out, "Printing number of iterations = %ld\n", (long)o.h);                              // :741
    float* U = P.U.f();
    float* Y = P.Y.f();
    PQP_TRY(dev_u_from_y(U, Y, P.Fp.f(), P.Gp.f(), P.Qinv.f(), N, M, s));                                // :999
    PQP_TRY(dev_cost(Jp.f(), U, P.Qp.f(), P.Fp.f(), P.Mp.f(), M, s));                                    // :1002
    PQP_TRY(dev_cost(Jd.f(), Y, P.Qd.f(), P.Fd.f(), P.Md.f(), N, s));                                    // :1003
    std::vector<float> hU(M);
    float jp = 0, jd = 0;
    PQP_TRY(download(hU.data(), U, M, s));
    PQP_TRY(download(&jp, Jp.p, 1, s));
    PQP_TRY(download(&jd, Jd.p, 1, s));
    PQP_HIP(hipStreamSynchronize(s));
    std::fprintf(out, "Jp = %f\n", jp);
    std::fprintf(out, "Jd = %f\n", jd);
    std::fprintf(out, "Printing U*\n");
    for (int i = 0; i < M; ++i) std::fprintf(out, "\t%f\n", hU[i]);
    std::fflush(out);
    return PQP_OK;
}

// ---------------------------------------------------------------------------
// 2b. batched device API
// ---------------------------------------------------------------------------
static int check_batch(int B, int N, const void* QdT, int ldq, long long qstride, int ldv) {
    if (B <= 0 || N <= 0) return set_error(PQP_ERR_ARG, "B and N must be positive (B=%d, N=%d)", B, N);
    if (!QdT || (reinterpret_cast<uintptr_t>(QdT) & 15))
        return set_error(PQP_ERR_ARG, "QdT must be a 16-byte aligned device pointer");
    if (ldq < N || (ldq & 3)) return set_error(PQP_ERR_ARG, "ldq (%d) must be >= N (%d) and a multiple of 4", ldq, N);
    if (qstride < (long long)N * ldq || (qstride & 3))
        return set_error(PQP_ERR_ARG, "qstride (%lld) must be >= N*ldq and a multiple of 4", qstride);
    if (ldv < N) return set_error(PQP_ERR_ARG, "ldv (%d) must be >= N (%d)", ldv, N);
    return ensure_device();
}

int pqp_batch_generate(uint32_t seed, long long inst0, int B, int N, int M, float* d_QdT, int ldq,
                       long long qstride, float* d_Fd, float* d_Md, float* d_theta, int ldv, void* stream) {
    PQP_TRY(check_batch(B, N, d_QdT, ldq, qstride, ldv));
    if (M <= 0 || !d_Fd || !d_theta) return set_error(PQP_ERR_ARG, "pqp_batch_generate: bad M or null output");
    hipStream_t s = static_cast<hipStream_t>(stream);
    PQP_HIP(launch_synth(seed, inst0, B, N, M, d_QdT, ldq, qstride, d_Fd, ldv, d_Md, s));
    PQP_HIP(launch_theta(B, d_QdT, ldq, qstride, N, d_theta, ldv, s));
    return PQP_OK;
}

int pqp_batch_synth_primal(uint32_t seed, long long inst0, int B, int N, int M, float* d_Qp_inv, float* d_Gp,
                           float* d_Kp, float* d_Fp, float* d_Mp, void* stream) {
    if (B <= 0 || N <= 0 || M <= 0 || !d_Qp_inv || !d_Gp || !d_Kp || !d_Fp || !d_Mp)
        return set_error(PQP_ERR_ARG, "pqp_batch_synth_primal: bad arguments");
    PQP_TRY(ensure_device());
    PQP_HIP(launch_synth_primal(seed, inst0, B, N, M, d_Qp_inv, d_Gp, d_Kp, d_Fp, d_Mp,
                                static_cast<hipStream_t>(stream)));
    return PQP_OK;
}

int pqp_batch_pack(int B, int N, const float* d_Qd, float* d_QdT, int ldq, long long qstride, void* stream) {
    PQP_TRY(check_batch(B, N, d_QdT, ldq, qstride, N));
    if (!d_Qd) return set_error(PQP_ERR_ARG, "pqp_batch_pack: null input");
    PQP_HIP(launch_pack_colmajor(B, d_Qd, N, (long long)N * N, d_QdT, ldq, qstride, static_cast<hipStream_t>(stream)));
    return PQP_OK;
}

int pqp_batch_theta(int B, int N, const float* d_QdT, int ldq, long long qstride, float* d_theta, int ldv,
                    void* stream) {
    PQP_TRY(check_batch(B, N, d_QdT, ldq, qstride, ldv));
    if (!d_theta) return set_error(PQP_ERR_ARG, "pqp_batch_theta: null output");
    PQP_HIP(launch_theta(B, d_QdT, ldq, qstride, N, d_theta, ldv, static_cast<hipStream_t>(stream)));
    return PQP_OK;
}

int pqp_batch_update(int B, int N, const float* d_QdT, int ldq, long long qstride, const float* d_theta,
                     const float* d_Fd, int ldv, const float* d_Y, float* d_Ynext, void* stream) {
    PQP_TRY(check_batch(B, N, d_QdT, ldq, qstride, ldv));
    if (!d_theta || !d_Fd || !d_Y || !d_Ynext) return set_error(PQP_ERR_ARG, "pqp_batch_update: null pointer");
    if (d_Y == d_Ynext) return set_error(PQP_ERR_ARG, "pqp_batch_update: d_Y and d_Ynext must not alias");
    if ((size_t)ldq * sizeof(float) > 150 * 1024) return set_error(PQP_ERR_ARG, "pqp_batch_update: N too large");
    PQP_HIP(launch_batch_update(B, d_QdT, qstride, ldq, N, d_theta, d_Fd, ldv, d_Y, d_Ynext,
                                static_cast<hipStream_t>(stream)));
    return PQP_OK;
}

int pqp_batch_iterate(int B, int N, const float* d_QdT, int ldq, long long qstride, const float* d_theta,
                      const float* d_Fd, int ldv, const float* d_Y0, float* d_Y, int updates, void* stream) {
    PQP_TRY(check_batch(B, N, d_QdT, ldq, qstride, ldv));
    if (!d_theta || !d_Fd || !d_Y || updates < 0) return set_error(PQP_ERR_ARG, "pqp_batch_iterate: bad argument");
    if ((size_t)2 * ldq * sizeof(float) > 160 * 1024)
        return set_error(PQP_ERR_ARG, "pqp_batch_iterate: ldq=%d needs more than 160 KiB of LDS", ldq);
    PQP_HIP(launch_batch_iterate(B, d_QdT, qstride, ldq, N, d_theta, d_Fd, ldv, d_Y0, d_Y, updates,
                                 static_cast<hipStream_t>(stream)));
    return PQP_OK;
}

// ---------------------------------------------------------------------------
// 2d. row blocks of one large problem (row-sharded solve)
// ---------------------------------------------------------------------------
int pqp_rowblock_create(const float* d_Qd_rows, int ld, const float* d_Fd, int N, int row0, int rows, void* stream,
                        pqp_rowblock** out) {
    if (!out) return set_error(PQP_ERR_ARG, "pqp_rowblock_create: null out");
    *out = nullptr;
    if (N <= 0 || ld < N || row0 < 0 || rows < 0 || row0 + (long long)rows > N || !d_Fd || (rows > 0 && !d_Qd_rows))
        return set_error(PQP_ERR_ARG, "pqp_rowblock_create: bad arguments (N=%d ld=%d row0=%d rows=%d)", N, ld, row0,
                         rows);
    if (split_lds_bytes(N) > kLdsBudget)
        return set_error(PQP_ERR_ARG, "pqp_rowblock_create: N=%d needs more than %zu B of LDS", N, kLdsBudget);
    PQP_TRY(ensure_device());
    hipStream_t s = static_cast<hipStream_t>(stream);
    std::unique_ptr<pqp_rowblock> b(new pqp_rowblock);
    PQP_HIP(hipGetDevice(&b->dev));
    b->N = N;
    b->row0 = row0;
    b->rows = rows;
    PQP_TRY(b->err.alloc(sizeof(int)));
    PQP_HIP(hipMemsetAsync(b->err.p, 0, sizeof(int), s));
    if (rows > 0) {
        DevBuf theta;
        PQP_TRY(theta.floats(rows));
        // by the block's entries: the bytes the lean layout saves grow with
        // rows x N, the chain both layouts run with N alone
        b->lean = use_lean(N, rows);
        PQP_HIP(launch_theta_rows(d_Qd_rows, ld, N, rows, theta.f(), s));
        if (b->lean) {  // Qd rows themselves (k_lean_relay): half the bytes of the split matrices
            b->lw = lean_pick_lw(rows);
            PQP_TRY(b->SP.floats(lean_floats(N, rows, b->lw)));
            PQP_TRY(b->fdpn.floats(lean_aux_floats(N, rows, b->lw)));
            PQP_HIP(hipMemsetAsync(b->SP.p, 0, sizeof(float) * lean_floats(N, rows, b->lw), s));
            PQP_HIP(launch_build_lean(d_Qd_rows, ld, theta.f(), d_Fd, N, rows, row0, b->lw, b->SP.f(), b->fdpn.f(),
                                      s));
        } else {
            b->lw = split_pick_lw(rows);
            PQP_TRY(b->SP.floats(split_floats(N, rows, b->lw)));
            PQP_TRY(b->fdpn.floats((size_t)2 * rows));
            PQP_HIP(hipMemsetAsync(b->SP.p, 0, sizeof(float) * split_floats(N, rows, b->lw), s));
            PQP_HIP(launch_build_split(d_Qd_rows, ld, theta.f(), d_Fd, N, rows, row0, b->lw, b->SP.f(),
                                       b->fdpn.f(), s));
        }
        PQP_HIP(hipStreamSynchronize(s));  // theta is freed on return
    }
    *out = b.release();
    return PQP_OK;
}

int pqp_rowblock_update(pqp_rowblock* b, const float* d_Y, float* d_Y_rows, void* stream) {
    if (!b || !d_Y || (b->rows > 0 && !d_Y_rows)) return set_error(PQP_ERR_ARG, "pqp_rowblock_update: null argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    DeviceGuard on(b->dev);
    int* err = static_cast<int*>(b->err.p);
    if (b->lean)
        PQP_HIP(launch_lean_update(b->SP.f(), b->fdpn.f(), b->N, b->rows, b->row0, b->lw, d_Y, d_Y_rows, s, nullptr, err));
    else
        PQP_HIP(launch_split_update(b->SP.f(), b->fdpn.f(), b->N, b->rows, b->row0, b->lw, d_Y, d_Y_rows, s, nullptr,
                                    err));
    return PQP_OK;
}

int pqp_rowblock_check(pqp_rowblock* b, void* stream) {
    if (!b) return set_error(PQP_ERR_ARG, "pqp_rowblock_check: null block");
    hipStream_t s = static_cast<hipStream_t>(stream);
    DeviceGuard on(b->dev);
    int herr = 0;
    PQP_HIP(hipMemcpyAsync(&herr, b->err.p, sizeof herr, hipMemcpyDeviceToHost, s));
    return relay_error_check(b->err, &herr, s, "pqp_rowblock_update");
}

int pqp_rowblock_destroy(pqp_rowblock* b) {
    if (!b) return PQP_OK;
    DeviceGuard on(b->dev);
    delete b;
    return PQP_OK;
}

int pqp_synth_rows(uint32_t seed, long long inst, int N, int M, int row0, int rows, float* d_Qd_rows, int ld,
                   float* d_Fd, float* d_Md, void* stream) {
    if (N <= 0 || M <= 0 || ld < N || row0 < 0 || rows < 0 || row0 + (long long)rows > N || (rows > 0 && !d_Qd_rows))
        return set_error(PQP_ERR_ARG, "pqp_synth_rows: bad arguments (N=%d M=%d ld=%d row0=%d rows=%d)", N, M, ld,
                         row0, rows);
    PQP_TRY(ensure_device());
    PQP_HIP(launch_synth_rows(seed, inst, N, M, row0, rows, d_Qd_rows, ld, d_Fd, d_Md,
                              static_cast<hipStream_t>(stream)));
    return PQP_OK;
}

// ---------------------------------------------------------------------------
// 2c. batched small problems
// ---------------------------------------------------------------------------
int pqp_batch_gauss_jordan(int B, int n, const float* d_A, float* d_res, void* stream) {
    if (B <= 0 || n <= 0 || !d_A || !d_res) return set_error(PQP_ERR_ARG, "pqp_batch_gauss_jordan: bad arguments");
    PQP_TRY(ensure_device());
    hipStream_t s = static_cast<hipStream_t>(stream);
    DevBuf aug, fac;
    PQP_TRY(aug.floats((size_t)B * gauss_jordan_aug_floats(n)));
    PQP_TRY(fac.floats((size_t)B * n));
    PQP_HIP(launch_gauss_jordan_b(B, d_A, aug.f(), fac.f(), d_res, n, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

// One grow-only device workspace per device for the batched setup calls
// (the round-5 form kept one per (thread, device), so a host that
// called from many pooled threads kept one buffer per thread it ever used).
// A call holds its device's lock from the workspace request until its stream
// has synchronised, so concurrent setup calls on one device take turns (each
// one fills the device anyway); no hipMalloc / hipFree (which synchronise the
// device) per call.  pqp_release_workspaces() frees every pool; nothing frees
// them at exit (a static destructor could run after the HIP runtime is gone).
namespace {
struct SetupPool {
    std::mutex mu;
    void* buf = nullptr;
    size_t cap = 0;
};
SetupPool g_setup_pool[64];

class SetupWorkspace {
  public:
    ~SetupWorkspace() {
        if (pool_) pool_->mu.unlock();
    }
    int acquire(size_t floats, float** out) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
            return set_error(PQP_ERR_NO_DEVICE, "libpqp: cannot query the current device");
        pool_ = &g_setup_pool[dev];
        pool_->mu.lock();
        const size_t bytes = floats * sizeof(float);
        if (pool_->cap < bytes) {
            if (pool_->buf) (void)hipFree(pool_->buf);
            pool_->buf = nullptr;
            pool_->cap = 0;
            const hipError_t e = hipMalloc(&pool_->buf, bytes);
            if (e != hipSuccess) {
                pool_->buf = nullptr;
                return set_error(PQP_ERR_ALLOC, "hipMalloc(%zu bytes): %s", bytes, hipGetErrorString(e));
            }
            pool_->cap = bytes;
        }
        *out = static_cast<float*>(pool_->buf);
        return PQP_OK;
    }

  private:
    SetupPool* pool_ = nullptr;
};
}  // namespace

int pqp_release_workspaces(void) {
    int dev0 = 0;
    const bool restore = hipGetDevice(&dev0) == hipSuccess;
    int rc = PQP_OK;
    for (int d = 0; d < 64; ++d) {
        SetupPool& p = g_setup_pool[d];
        std::lock_guard<std::mutex> g(p.mu);
        if (!p.buf) continue;
        if (hipSetDevice(d) != hipSuccess || hipFree(p.buf) != hipSuccess)
            rc = set_error(PQP_ERR_HIP, "pqp_release_workspaces: hipFree on device %d failed", d);
        p.buf = nullptr;
        p.cap = 0;
    }
    if (restore) (void)hipSetDevice(dev0);
    return rc;
}

int pqp_batch_convert_to_dual(int B, int N, int M, const float* d_Qp_inv, const float* d_Gp, const float* d_Kp,
                              const float* d_Fp, const float* d_Mp, float* d_Qd, float* d_Fd, float* d_Md,
                              void* stream) {
    if (B <= 0 || N <= 0 || M <= 0 || !d_Qp_inv || !d_Gp || !d_Kp || !d_Fp || !d_Mp || !d_Qd || !d_Fd || !d_Md)
        return set_error(PQP_ERR_ARG, "pqp_batch_convert_to_dual: bad arguments");
    PQP_TRY(ensure_device());
    hipStream_t s = static_cast<hipStream_t>(stream);
    const long long nm = (long long)N * M, mm = (long long)M * M, nn = (long long)N * N;
    // Gp Qp_inv (and Fp'Qp_inv) in the device's grow-only workspace, held
    // until this call's stream has synchronised
    SetupWorkspace wsp;
    float* ws = nullptr;
    PQP_TRY(wsp.acquire((size_t)B * nm + (size_t)B * M + 64, &ws));
    float* GQ = ws;
    float* fq = ws + (((size_t)B * nm + 63) & ~(size_t)63);
    // same sequence as dev_convert_to_dual (PQP_CPU.c:489-498), problem-strided
    PQP_HIP(launch_matmul_seq_b(B, GQ, d_Gp, 0, d_Qp_inv, 0, N, M, M, nm, mm, nm, s));
    PQP_HIP(launch_matmul_seq_b(B, d_Qd, GQ, 0, d_Gp, 1, N, M, N, nm, nm, nn, s));
    PQP_HIP(launch_matmul_seq_b(B, d_Fd, GQ, 0, d_Fp, 0, N, M, 1, nm, M, N, s));
    PQP_HIP(launch_axpy_b(B, d_Fd, d_Kp, 1.0f, N, N, N, s));
    PQP_HIP(launch_matmul_seq_b(B, fq, d_Fp, 1, d_Qp_inv, 0, 1, M, M, M, mm, M, s));
    PQP_HIP(launch_matmul_seq_b(B, d_Md, fq, 0, d_Fp, 0, 1, M, 1, M, M, 1, s));
    PQP_HIP(launch_axpy_b(B, d_Md, d_Mp, -1.0f, 1, 1, 1, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

int pqp_batch_compute_fp(int B, int m, int nd, int ns, const float* d_Fp1, const float* d_Fp2, const float* d_Fp3,
                         const float* d_D, const float* d_x, float* d_Fp, void* stream) {
    if (B <= 0 || m <= 0 || nd <= 0 || ns <= 0 || !d_Fp1 || !d_Fp2 || !d_Fp3 || !d_D || !d_x || !d_Fp)
        return set_error(PQP_ERR_ARG, "pqp_batch_compute_fp: bad arguments");
    PQP_TRY(ensure_device());
    hipStream_t s = static_cast<hipStream_t>(stream);
    DevBuf t;
    PQP_TRY(t.floats((size_t)B * m));
    PQP_HIP(launch_matmul_seq_b(B, d_Fp, d_Fp1, 0, d_D, 0, m, nd, 1, 0, nd, m, s));      // Fp1 D
    PQP_HIP(launch_matmul_seq_b(B, t.f(), d_Fp2, 0, d_x, 0, m, ns, 1, 0, ns, m, s));     // Fp2 x
    PQP_HIP(launch_axpy_b(B, d_Fp, t.f(), 1.0f, m, m, m, s));
    PQP_HIP(launch_axpy_b(B, d_Fp, d_Fp3, -1.0f, m, m, 0, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

int pqp_batch_compute_mp(int B, int nd, int ns, const float* d_Mp1, const float* d_Mp2, const float* d_Mp3,
                         const float* d_Mp4, const float* d_Mp5, const float* d_Mp6, const float* d_D,
                         const float* d_x, float* d_Mp, void* stream) {
    if (B <= 0 || nd <= 0 || ns <= 0 || !d_Mp1 || !d_Mp2 || !d_Mp3 || !d_Mp4 || !d_Mp5 || !d_Mp6 || !d_D || !d_x ||
        !d_Mp)
        return set_error(PQP_ERR_ARG, "pqp_batch_compute_mp: bad arguments");
    PQP_TRY(ensure_device());
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int big = ns > nd ? ns : nd;
    DevBuf row, T;
    PQP_TRY(row.floats((size_t)B * big));
    PQP_TRY(T.floats((size_t)B * 5));
    float* R = row.f();
    float* t = T.f();
    // the five halved terms of PQP_CPU.c:400-423, term s of problem b at t[b*5 + s]
    PQP_HIP(launch_matmul_seq_b(B, R, d_x, 1, d_Mp1, 0, 1, ns, ns, ns, 0, big, s));       // x' Mp1
    PQP_HIP(launch_matmul_seq_b(B, t + 0, R, 0, d_x, 0, 1, ns, 1, big, ns, 5, s));        //  . x
    PQP_HIP(launch_matmul_seq_b(B, R, d_D, 1, d_Mp2, 0, 1, nd, ns, nd, 0, big, s));       // D' Mp2
    PQP_HIP(launch_matmul_seq_b(B, t + 1, R, 0, d_x, 0, 1, ns, 1, big, ns, 5, s));        //  . x
    PQP_HIP(launch_matmul_seq_b(B, t + 2, d_Mp4, 1, d_x, 0, 1, ns, 1, 0, ns, 5, s));      // Mp4' x
    PQP_HIP(launch_matmul_seq_b(B, R, d_D, 1, d_Mp3, 0, 1, nd, nd, nd, 0, big, s));       // D' Mp3
    PQP_HIP(launch_matmul_seq_b(B, t + 3, R, 0, d_D, 0, 1, nd, 1, big, nd, 5, s));        //  . D
    PQP_HIP(launch_matmul_seq_b(B, t + 4, d_Mp5, 1, d_D, 0, 1, nd, 1, 0, nd, 5, s));      // Mp5' D
    PQP_HIP(launch_mp_finish_b(B, t, d_Mp6, d_Mp, 0, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

// Which batched solver a problem size takes: 0 one wave / tiny workgroup
// (N, M <= 32), 3 every matrix once in LDS (k_solve_mid), 1 everything
// staged in LDS with the split copies (k_solve_small; mid_off), 2 one
// workgroup from global memory (k_solve_single; needs the prepared data of
// pqp_batch_prepare), -1 too large for any.
static int batch_path(int N, int M) {
    if (N <= 32 && M <= 32 && !g_tune.force_small) return 0;
    if (!g_tune.mid_off && solve_mid_lds_bytes(N, M, true) <= kLdsBudget) return 3;
    if (solve_small_lds_bytes(N, M) <= kLdsBudget) return 1;
    if (solve_single_lds_bytes(round4(N), round4(M), false) <= kLdsBudget) return 2;
    return -1;
}

int pqp_batch_solve_path(int N, int M) {
    if (N <= 0 || M <= 0) return set_error(PQP_ERR_ARG, "pqp_batch_solve_path: N and M must be positive");
    const int p = batch_path(N, M);
    return p < 0 ? set_error(PQP_ERR_ARG, "N=%d, M=%d exceeds the batched solvers' LDS budget", N, M) : p;
}

int pqp_batch_solve_kernel(int N, int M) {
    if (N <= 0 || M <= 0) return set_error(PQP_ERR_ARG, "pqp_batch_solve_kernel: N and M must be positive");
    return batch_path(N, M) == 2 && pipe_route(N, M, g_tune.pipe_variant) ? 1 : 0;
}

int pqp_batch_prepare(int B, int N, int M, const float* d_Qd, const float* d_Gp, const float* d_Qp_inv, float* d_QdT,
                      float* d_theta, int* d_sym, float* d_GpT, float* d_QinvT, int* all_sym_out, void* stream) {
    if (all_sym_out) *all_sym_out = 0;
    if (B <= 0 || N <= 0 || M <= 0 || !d_Qd || !d_theta || !d_sym)
        return set_error(PQP_ERR_ARG, "pqp_batch_prepare: bad arguments");
    if ((d_GpT && !d_Gp) || (d_QinvT && !d_Qp_inv))
        return set_error(PQP_ERR_ARG, "pqp_batch_prepare: a transposed copy needs its source");
    PQP_TRY(ensure_device());
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int ldq = round4(N);
    // Qd bit-symmetric in every problem (convertToDual's (Gp Qp_inv) Gp' is,
    // for a diagonal Qp_inv) and N % 4 == 0: the row-major Qd is its own
    // column-major copy, no packing pass.  The per-problem flags also gate the
    // fused Y'Qd pass of converge mode.
    PQP_HIP(launch_check_symmetric(B, d_Qd, N, d_sym, s));
    std::vector<int> hs((size_t)B);
    PQP_HIP(hipMemcpyAsync(hs.data(), d_sym, sizeof(int) * (size_t)B, hipMemcpyDeviceToHost, s));
    PQP_HIP(hipStreamSynchronize(s));
    bool all_sym = ldq == N;
    for (int v : hs) all_sym = all_sym && v != 0;
    if (all_sym_out) *all_sym_out = all_sym ? 1 : 0;
    const float* qdt = d_Qd;
    if (!all_sym) {
        if (!d_QdT)
            return set_error(PQP_ERR_NEEDS_QDT, "pqp_batch_prepare: some Qd is not bit-symmetric (or N %% 4 != 0): pass "
                                          "d_QdT ([B][N][round4(N)] floats) for its column-major copy");
        PQP_HIP(launch_pack_colmajor(B, d_Qd, N, (long long)N * N, d_QdT, ldq, (long long)N * ldq, s));
        qdt = d_QdT;
    }
    PQP_HIP(launch_theta(B, qdt, ldq, (long long)N * ldq, N, d_theta, N, s));  // computeTheta :503-519
    if (d_GpT) PQP_HIP(launch_transpose_b(B, d_Gp, N, M, d_GpT, s));
    if (d_QinvT) PQP_HIP(launch_transpose_b(B, d_Qp_inv, M, M, d_QinvT, s));
    return PQP_OK;
}

int pqp_batch_solve_prepared(int B, int N, int M, const float* d_Qd, const float* d_QdT, const float* d_theta,
                             const int* d_sym, const float* d_GpT, const float* d_QinvT, const float* d_Fd,
                             const float* d_Md, const float* d_Qp, const float* d_Qp_inv, const float* d_Fp,
                             const float* d_Mp, const float* d_Gp, const float* d_Kp, int mode, long long num_iter,
                             long long max_updates, float* d_Y, float* d_U, long long* d_h, int* d_status,
                             void* stream) {
    if (B <= 0 || N <= 0 || M <= 0 || !d_Qd || !d_Fd || !d_Y)
        return set_error(PQP_ERR_ARG, "pqp_batch_solve: bad arguments");
    if (mode != PQP_MODE_CONVERGE && mode != PQP_MODE_FIXED)
        return set_error(PQP_ERR_ARG, "pqp_batch_solve: unknown mode %d", mode);
    if (mode == PQP_MODE_CONVERGE && (!d_Md || !d_Qp || !d_Qp_inv || !d_Fp || !d_Mp || !d_Gp || !d_Kp || !d_U))
        return set_error(PQP_ERR_ARG, "pqp_batch_solve: converge mode needs every primal/dual array and U");
    PQP_TRY(ensure_device());
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int ldq = round4(N), ldm = round4(M);
    const int path = batch_path(N, M);
    if (path < 0) return set_error(PQP_ERR_ARG, "pqp_batch_solve: N=%d, M=%d exceeds the LDS budget", N, M);
    if (path == 2 && (!d_theta || !d_sym || (!d_QdT && ldq != N)))
        return set_error(PQP_ERR_ARG, "pqp_batch_solve_prepared: N=%d, M=%d needs pqp_batch_prepare's theta, "
                                      "symmetry flags and (unless every Qd is bit-symmetric) d_QdT", N, M);
    // the fused Y'Qd pass needs one more ldq-long LDS vector: only where it fits
    const bool fuse = path == 2 && !batch_unfused() && ldq == N && solve_single_lds_bytes(ldq, ldm, true) <= kLdsBudget;
    DevBuf state, pending, Udummy;
    if (!d_U) {
        PQP_TRY(Udummy.floats((size_t)B * M));
        d_U = Udummy.f();
    }
    PQP_TRY(state.alloc(sizeof(SolveState) * (size_t)B));
    PQP_TRY(pending.alloc(sizeof(int)));
    PQP_HIP(launch_state_init(B, static_cast<SolveState*>(state.p), s));
    SolveArgs a{};
    a.QdT = path == 2 ? (d_QdT ? d_QdT : d_Qd) : nullptr;
    a.Qd = d_Qd;
    a.theta = path == 2 ? d_theta : nullptr;
    a.Fd = d_Fd;
    a.Md = d_Md;
    a.Qp = d_Qp;
    a.Qinv = d_Qp_inv;
    a.sym = fuse ? d_sym : nullptr;
    a.GpT = path == 2 && mode == PQP_MODE_CONVERGE ? d_GpT : nullptr;
    a.QinvT = path == 2 && mode == PQP_MODE_CONVERGE ? d_QinvT : nullptr;
    a.feas_split = (g_tune.batch_opts & 16) ? 0 : 1;
    a.trace = g_tune.mid_trace;
    a.trace_n = g_tune.mid_trace_n;
    a.Fp = d_Fp;
    a.Mp = d_Mp;
    a.Gp = d_Gp;
    a.Kp = d_Kp;
    a.Y = d_Y;
    a.U = d_U;
    a.N = N;
    a.M = M;
    a.ldq = ldq;
    a.ldm = ldm;
    a.mode = (mode == PQP_MODE_CONVERGE) ? kModeConverge : kModeFixed;
    a.num_iter = num_iter;
    a.max_updates = max_updates;
    a.chunk = pqp::batch_chunk_for(N, M);
    a.pending = static_cast<int*>(pending.p);
    SolveState* st = static_cast<SolveState*>(state.p);
    for (;;) {
        int left = 0;
        PQP_HIP(hipMemsetAsync(pending.p, 0, sizeof(int), s));
        PQP_HIP(launch_solve_batch(B, path, a, st, s));
        PQP_HIP(hipMemcpyAsync(&left, pending.p, sizeof(int), hipMemcpyDeviceToHost, s));
        PQP_HIP(hipStreamSynchronize(s));
        if (left == 0) break;
    }
    PQP_HIP(launch_extract_state(B, st, d_h, d_status, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

int pqp_batch_solve(int B, int N, int M, const float* d_Qd, const float* d_Fd, const float* d_Md, const float* d_Qp,
                    const float* d_Qp_inv, const float* d_Fp, const float* d_Mp, const float* d_Gp, const float* d_Kp,
                    int mode, long long num_iter, long long max_updates, float* d_Y, float* d_U, long long* d_h,
                    int* d_status, void* stream) {
    if (B <= 0 || N <= 0 || M <= 0 || !d_Qd || !d_Fd || !d_Y)
        return set_error(PQP_ERR_ARG, "pqp_batch_solve: bad arguments");
    const int path = batch_path(N, M);
    if (path < 0) return set_error(PQP_ERR_ARG, "pqp_batch_solve: N=%d, M=%d exceeds the LDS budget", N, M);
    DevBuf QdT, theta, sym, GpT, QinvT;
    if (path == 2) {  // the per-problem setup, for this call only (pqp_batch_prepare keeps it across calls)
        PQP_TRY(ensure_device());
        PQP_TRY(theta.floats((size_t)B * N));
        PQP_TRY(sym.alloc(sizeof(int) * (size_t)B));
        if ((g_tune.batch_opts & 2) && mode == PQP_MODE_CONVERGE && d_Gp && d_Qp_inv) {
            PQP_TRY(GpT.floats((size_t)B * N * M));
            PQP_TRY(QinvT.floats((size_t)B * M * M));
        }
        int all_sym = 0;
        int* ps = static_cast<int*>(sym.p);
        const int rc = pqp_batch_prepare(B, N, M, d_Qd, d_Gp, d_Qp_inv, nullptr, theta.f(), ps, GpT.f(), QinvT.f(),
                                         &all_sym, stream);
        if (rc != PQP_OK && rc != PQP_ERR_NEEDS_QDT) return rc;
        if (rc == PQP_ERR_NEEDS_QDT) {  // some Qd not bit-symmetric: the column-major copy
            PQP_TRY(QdT.floats((size_t)B * N * round4(N)));
            PQP_TRY(pqp_batch_prepare(B, N, M, d_Qd, d_Gp, d_Qp_inv, QdT.f(), theta.f(), ps, GpT.f(), QinvT.f(),
                                      &all_sym, stream));
            restore_error("");  // the first call's "pass d_QdT" text is not this call's outcome
        }
    }
    return pqp_batch_solve_prepared(B, N, M, d_Qd, QdT.f(), theta.f(), static_cast<const int*>(sym.p), GpT.f(),
                                    QinvT.f(), d_Fd, d_Md, d_Qp, d_Qp_inv, d_Fp, d_Mp, d_Gp, d_Kp, mode, num_iter,
                                    max_updates, d_Y, d_U, d_h, d_status, stream);
}

// ---------------------------------------------------------------------------
// 1. drop-in entry points (reference signatures)
// ---------------------------------------------------------------------------
void solveQuadraticDual(float* Y, float* Qd, float* Fd, float* Md, float* U, float* Qp, float* Qp_inv, float* Fp,
                        float* Mp, float* Gp, float* Kp, int N, int M) {
    long long h = 0;
    long long cap = 0;  // the reference has no cap (PQP_CPU.c:718); PQP_MAX_UPDATES adds one
    if (const char* env = std::getenv("PQP_MAX_UPDATES")) cap = std::atoll(env);
    int rc = pqp_solve_dual(Qd, Fd, Md, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M, PQP_MODE_CONVERGE, 0, cap, Y, U, &h,
                            nullptr, nullptr);
    if (rc != PQP_OK && rc != PQP_ERR_NOT_CONVERGED) die("solveQuadraticDual");
    std::printf("Printing number of iterations = %ld\n", (long)h);
}

void updateY2(float* Y_next, float* Y, float* Qdp_theta, float* Qdn_theta, float* Fd, float* Fdp, float* Fdn,
              int N) {
    (void)Fd;
    auto run = [&]() -> int {
        if (N <= 0) return set_error(PQP_ERR_ARG, "updateY2: N must be positive");
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        const int ldq = round4(N);
        DevBuf qp, qn, qpT, qnT, fdp, fdn, y, yn;
        PQP_TRY(upload(qp, Qdp_theta, (size_t)N * N, s));
        PQP_TRY(upload(qn, Qdn_theta, (size_t)N * N, s));
        PQP_TRY(upload(fdp, Fdp, N, s));
        PQP_TRY(upload(fdn, Fdn, N, s));
        PQP_TRY(upload(y, Y, N, s));
        PQP_TRY(yn.floats(N));
        PQP_TRY(qpT.floats((size_t)N * ldq));
        PQP_TRY(qnT.floats((size_t)N * ldq));
        PQP_HIP(launch_pack_colmajor(1, qp.f(), N, (long long)N * N, qpT.f(), ldq, (long long)N * ldq, s));
        PQP_HIP(launch_pack_colmajor(1, qn.f(), N, (long long)N * N, qnT.f(), ldq, (long long)N * ldq, s));
        PQP_HIP(launch_update_split(qpT.f(), qnT.f(), ldq, N, fdp.f(), fdn.f(), y.f(), yn.f(), s));
        PQP_TRY(download(Y_next, yn.p, N, s));
        PQP_HIP(hipStreamSynchronize(s));
        return PQP_OK;
    };
    if (run() != PQP_OK) die("updateY2");
}

int terminate(float* Y, float* Qd, float* Fd, float* Md, float* U, float* Qp, float* Qp_inv, float* Fp, float* Mp,
              float* Gp, float* Kp, int N, int M) {
    int result = 0;
    auto run = [&]() -> int {
        PQP_TRY(check_dims(N, M));
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        pqp_problem P;
        PQP_TRY(problem_upload(P, Qd, Fd, Md, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M, s));
        PQP_HIP(hipMemcpyAsync(P.Y.p, Y, sizeof(float) * N, hipMemcpyHostToDevice, s));
        SolveOut o;
        PQP_TRY(problem_run(P, kModeTerminate, 0, 0, true, o, s));
        PQP_TRY(download(U, P.U.p, M, s));
        PQP_HIP(hipStreamSynchronize(s));
        result = o.last_stop;
        return PQP_OK;
    };
    if (run() != PQP_OK) die("terminate");
    return result;
}

void convertToDual(float* Qd, float* Fd, float* Md, float* Qp_inv, float* Gp, float* Kp, float* Fp, float* Mp, int N,
                   int M) {
    auto run = [&]() -> int {
        PQP_TRY(check_dims(N, M));
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        DevBuf qinv, gp, kp, fp, mp, qd, fd, md;
        PQP_TRY(upload(qinv, Qp_inv, (size_t)M * M, s));
        PQP_TRY(upload(gp, Gp, (size_t)N * M, s));
        PQP_TRY(upload(kp, Kp, N, s));
        PQP_TRY(upload(fp, Fp, M, s));
        PQP_TRY(upload(mp, Mp, 1, s));
        PQP_TRY(qd.floats((size_t)N * N));
        PQP_TRY(fd.floats(N));
        PQP_TRY(md.floats(1));
        PQP_TRY(dev_convert_to_dual(qd.f(), fd.f(), md.f(), qinv.f(), gp.f(), kp.f(), fp.f(), mp.f(), N, M, s));
        PQP_TRY(download(Qd, qd.p, (size_t)N * N, s));
        PQP_TRY(download(Fd, fd.p, N, s));
        PQP_TRY(download(Md, md.p, 1, s));
        PQP_HIP(hipStreamSynchronize(s));
        return PQP_OK;
    };
    if (run() != PQP_OK) die("convertToDual");
}

void computeUfromY(float* U, float* Y, float* Fp, float* Gp, float* Qp_inv, int N, int M) {
    auto run = [&]() -> int {
        PQP_TRY(check_dims(N, M));
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        DevBuf u, y, fp, gp, qinv;
        PQP_TRY(upload(y, Y, N, s));
        PQP_TRY(upload(fp, Fp, M, s));
        PQP_TRY(upload(gp, Gp, (size_t)N * M, s));
        PQP_TRY(upload(qinv, Qp_inv, (size_t)M * M, s));
        PQP_TRY(u.floats(M));
        PQP_TRY(dev_u_from_y(u.f(), y.f(), fp.f(), gp.f(), qinv.f(), N, M, s));
        PQP_TRY(download(U, u.p, M, s));
        PQP_HIP(hipStreamSynchronize(s));
        return PQP_OK;
    };
    if (run() != PQP_OK) die("computeUfromY");
}

float computeCost(float* Z, float* Q, float* F, float* Mc, int N) {
    float J = 0.0f;
    auto run = [&]() -> int {
        if (N <= 0) return set_error(PQP_ERR_ARG, "computeCost: N must be positive");
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        DevBuf z, q, f, m, j;
        PQP_TRY(upload(z, Z, N, s));
        PQP_TRY(upload(q, Q, (size_t)N * N, s));
        PQP_TRY(upload(f, F, N, s));
        PQP_TRY(upload(m, Mc, 1, s));
        PQP_TRY(j.floats(1));
        PQP_TRY(dev_cost(j.f(), z.f(), q.f(), f.f(), m.f(), N, s));
        PQP_TRY(download(&J, j.p, 1, s));
        PQP_HIP(hipStreamSynchronize(s));
        return PQP_OK;
    };
    if (run() != PQP_OK) die("computeCost");
    return J;
}

int checkFeas(float* U, float* Gp, float* Kp, int N, int M) {
    int flag = 0;
    auto run = [&]() -> int {
        PQP_TRY(check_dims(N, M));
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        DevBuf u, gp, kp;
        PQP_TRY(upload(u, U, M, s));
        PQP_TRY(upload(gp, Gp, (size_t)N * M, s));
        PQP_TRY(upload(kp, Kp, N, s));
        return dev_check_feas(u.f(), gp.f(), kp.f(), N, M, &flag, s);
    };
    if (run() != PQP_OK) die("checkFeas");
    return flag;
}

void computeTheta(float* theta, float* Qd, int N) {
    auto run = [&]() -> int {
        if (N <= 0) return set_error(PQP_ERR_ARG, "computeTheta: N must be positive");
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        DevBuf th, qd;
        PQP_TRY(upload(th, theta, (size_t)N * N, s));
        PQP_TRY(upload(qd, Qd, (size_t)N * N, s));
        PQP_HIP(launch_theta_rowmajor(qd.f(), N, th.f(), s));
        PQP_TRY(download(theta, th.p, (size_t)N * N, s));
        PQP_HIP(hipStreamSynchronize(s));
        return PQP_OK;
    };
    if (run() != PQP_OK) die("computeTheta");
}

void matrixMultiply(float* output, float* mat1, int transpose1, float* mat2, int transpose2, int a, int b, int c) {
    auto run = [&]() -> int {
        if (a <= 0 || b < 0 || c <= 0) return set_error(PQP_ERR_ARG, "matrixMultiply: bad sizes");
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        DevBuf A, B, O;
        PQP_TRY(upload(A, mat1, (size_t)a * b, s));
        PQP_TRY(upload(B, mat2, (size_t)b * c, s));
        PQP_TRY(O.floats((size_t)a * c));
        PQP_TRY(dev_matmul(O.f(), A.f(), transpose1, B.f(), transpose2, a, b, c, s));
        PQP_TRY(download(output, O.p, (size_t)a * c, s));
        PQP_HIP(hipStreamSynchronize(s));
        return PQP_OK;
    };
    if (run() != PQP_OK) die("matrixMultiply");
}

void Gauss_Jordan(float* A, float* res, int N) {
    auto run = [&]() -> int {
        if (N <= 0) return set_error(PQP_ERR_ARG, "Gauss_Jordan: N must be positive");
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        DevBuf a, r;
        PQP_TRY(upload(a, A, (size_t)N * N, s));
        PQP_TRY(r.floats((size_t)N * N));
        PQP_TRY(dev_gauss_jordan(r.f(), a.f(), N, s));
        PQP_TRY(download(res, r.p, (size_t)N * N, s));
        PQP_HIP(hipStreamSynchronize(s));
        return PQP_OK;
    };
    if (run() != PQP_OK) die("Gauss_Jordan");
}

void computeFp(float* Fp, float* Fp1, float* Fp2, float* Fp3, float* D, float* x) {
    const int m = kRefNInput * kRefPHorizon, nd = kRefNDis * kRefPHorizon, ns = kRefNState;
    auto run = [&]() -> int {
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        DevBuf fp, f1, f2, f3, d, xx;
        PQP_TRY(upload(f1, Fp1, (size_t)m * nd, s));
        PQP_TRY(upload(f2, Fp2, (size_t)m * ns, s));
        PQP_TRY(upload(f3, Fp3, m, s));
        PQP_TRY(upload(d, D, nd, s));
        PQP_TRY(upload(xx, x, ns, s));
        PQP_TRY(fp.floats(m));
        PQP_TRY(dev_compute_fp(fp.f(), f1.f(), f2.f(), f3.f(), d.f(), xx.f(), m, nd, ns, s));
        PQP_TRY(download(Fp, fp.p, m, s));
        PQP_HIP(hipStreamSynchronize(s));
        return PQP_OK;
    };
    if (run() != PQP_OK) die("computeFp");
}

void computeMp(float* Mp, float* Mp1, float* Mp2, float* Mp3, float* Mp4, float* Mp5, float* Mp6, float* D,
               float* x) {
    const int nd = kRefNDis * kRefPHorizon, ns = kRefNState;
    auto run = [&]() -> int {
        PQP_TRY(ensure_device());
        hipStream_t s = lib_stream();
        DevBuf mp, m1, m2, m3, m4, m5, m6, d, xx;
        PQP_TRY(upload(m1, Mp1, (size_t)ns * ns, s));
        PQP_TRY(upload(m2, Mp2, (size_t)nd * ns, s));
        PQP_TRY(upload(m3, Mp3, (size_t)nd * nd, s));
        PQP_TRY(upload(m4, Mp4, ns, s));
        PQP_TRY(upload(m5, Mp5, nd, s));
        PQP_TRY(upload(m6, Mp6, 1, s));
        PQP_TRY(upload(d, D, nd, s));
        PQP_TRY(upload(xx, x, ns, s));
        PQP_TRY(mp.floats(1));
        PQP_TRY(dev_compute_mp(mp.f(), m1.f(), m2.f(), m3.f(), m4.f(), m5.f(), m6.f(), d.f(), xx.f(), nd, ns, s));
        PQP_TRY(download(Mp, mp.p, 1, s));
        PQP_HIP(hipStreamSynchronize(s));
        return PQP_OK;
    };
    if (run() != PQP_OK) die("computeMp");
}

void input(float* qp_inv, float* Fp1, float* Fp2, float* Fp3, float* Mp1, float* Mp2, float* Mp3, float* Mp4,
           float* Mp5, float* Mp6, float* Gp, float* Kp, float* x, float* D, float* theta, float* Z) {
    const int m = kRefNInput * kRefPHorizon, nd = kRefNDis * kRefPHorizon, ns = kRefNState;
    if (pqp_read_example("./example", m, nd, ns, qp_inv, Fp1, Fp2, Fp3, Mp1, Mp2, Mp3, Mp4, Mp5, Mp6, Gp, Kp, x, D) !=
            PQP_OK ||
        read_unused_example("./example", ns, kRefNOutput * kRefPHorizon, nd, Z, theta) != PQP_OK)
        die("input");
}

}  // extern "C"

// ---------------------------------------------------------------------------
// tuning / diagnostics (include/pqp_tuning.h)
// ---------------------------------------------------------------------------
#include "../../include/pqp_tuning.h"

namespace {
// key -> knob of pqp::g_tune (pqp_tune / pqp_tune_get)
struct KnobRef {
    const char* key;
    int* i;
    bool* b;
    long long* ll;
};
const KnobRef* find_knob(const char* key) {
    using pqp::g_tune;
    static const KnobRef knobs[] = {
        {"relay_spin_max", &g_tune.relay_spin_max, nullptr, nullptr},
        {"lean_min_n", &g_tune.lean_min_n, nullptr, nullptr},
        {"split_lw", &g_tune.split_lw, nullptr, nullptr},
        {"wave_pipe_max_b", &g_tune.wave_pipe_max_b, nullptr, nullptr},
        {"fixed_rl_max_b", &g_tune.fixed_rl_max_b, nullptr, nullptr},
        {"wave_min_b", &g_tune.wave_min_b, nullptr, nullptr},
        {"matmul_tiled_off", &g_tune.matmul_tiled_off, nullptr, nullptr},
        {"gj_blocked_off", &g_tune.gj_blocked_off, nullptr, nullptr},
        {"single_scalar", &g_tune.single_scalar, nullptr, nullptr},
        {"persist_off", &g_tune.persist_off, nullptr, nullptr},
        {"persist_stall_wg", &g_tune.persist_stall_wg, nullptr, nullptr},
        {"persist_fit_cus", &g_tune.persist_fit_cus, nullptr, nullptr},
        {"converge_persist_off", &g_tune.converge_persist_off, nullptr, nullptr},
        {"force_small", nullptr, &g_tune.force_small, nullptr},
        {"force_single", nullptr, &g_tune.force_single, nullptr},
        {"wide_min_n", &g_tune.wide_min_n, nullptr, nullptr},
        {"batch_opts", &g_tune.batch_opts, nullptr, nullptr},
        {"mid_off", &g_tune.mid_off, nullptr, nullptr},
        {"pipe_off", &g_tune.pipe_off, nullptr, nullptr},
        {"mid_v1", &g_tune.mid_v1, nullptr, nullptr},
        {"mid2_pair", &g_tune.mid2_pair, nullptr, nullptr},
        {"mid2_min_n", &g_tune.mid2_min_n, nullptr, nullptr},
        {"mid2_dense", &g_tune.mid2_dense, nullptr, nullptr},
        {"single_occ", &g_tune.single_occ, nullptr, nullptr},
        {"matmul_pk_off", &g_tune.matmul_pk_off, nullptr, nullptr},
        {"pipe_variant", &g_tune.pipe_variant, nullptr, nullptr},
        {"pipe_force", &g_tune.pipe_force, nullptr, nullptr},
        {"batch_chunk", nullptr, nullptr, &g_tune.batch_chunk},
        {"converge_chunk", nullptr, nullptr, &g_tune.converge_chunk},
        {"tiny_old", &g_tune.tiny_old, nullptr, nullptr},
        {"tiny_dense", &g_tune.tiny_dense, nullptr, nullptr},
        {"tiny_stall", &g_tune.tiny_stall, nullptr, nullptr},
        {"tiny_fallback", &g_tune.tiny_fallback, nullptr, nullptr},
        {"tiny_np", &g_tune.tiny_np, nullptr, nullptr},
        {"tiny_ablk", &g_tune.tiny_ablk, nullptr, nullptr},
        {"tiny_apoll", &g_tune.tiny_apoll, nullptr, nullptr},
        {"persist_xcds", &g_tune.persist_xcds, nullptr, nullptr},
        {"converge_xcds", &g_tune.converge_xcds, nullptr, nullptr},
        {"tiny_chunk", nullptr, nullptr, &g_tune.tiny_chunk},
        {"iterate_kind", &g_tune.iterate_kind, nullptr, nullptr},
    };
    for (const KnobRef& k : knobs)
        if (std::strcmp(k.key, key) == 0) return &k;
    return nullptr;
}
long long knob_value(const KnobRef& k) { return k.i ? *k.i : (k.b ? (long long)*k.b : *k.ll); }
}  // namespace

namespace pqp {
// iterates per problem per batched-solve launch: about 2^28 element updates per
// problem (56 at n_dual 1024, M 512: each launch's start -- its first Gp'Y
// pass, the state, the host's check of the pending count -- cost about a
// quarter (infeasible) to 1.4 (feasible) iterates at 2^26:
// profiles/r04/pipe/launch_amortization.json), or the batch_chunk knob
long long batch_chunk_for(int N, int M) {
    if (g_tune.batch_chunk > 0) return g_tune.batch_chunk;
    const double per_update = (double)N * N * 3.0 + 2.0 * N * M + 2.0 * M * M + 1.0;
    const long long chunk = (long long)((double)(1 << 28) / per_update);
    return chunk < 1 ? 1 : chunk;
}
}  // namespace pqp

static std::mutex g_tune_mu;  // pqp_tune / pqp_tune_trace writers

extern "C" int pqp_tune(const char* key, long long value, long long* old_value) {
    // writers are serialized; readers (the launches) take no lock: the knobs
    // are test and tuning hooks that must not change while another thread is
    // inside a solve (include/pqp_tuning.h)
    std::lock_guard<std::mutex> lk(g_tune_mu);
    const KnobRef* k = key ? find_knob(key) : nullptr;
    if (!k) return pqp::set_error(PQP_ERR_ARG, "pqp_tune: unknown key '%s'", key ? key : "(null)");
    if (old_value) *old_value = knob_value(*k);
    if (std::strcmp(key, "relay_spin_max") == 0) {
        // 0 restores the default; clamped: a budget near INT_MAX would let a
        // broken hand-off spin until its counter overflows
        value = value == 0 ? pqp::kRelaySpinMax : (value > (1 << 30) ? (1 << 30) : value);
    } else if (std::strcmp(key, "converge_chunk") == 0) {
        value = value > 0 ? value : (1 << 16);
    } else if (std::strcmp(key, "persist_stall_wg") == 0) {
        value = value >= 0 ? value : -1;
    }
    if (k->i) *k->i = (int)value;
    else if (k->b) *k->b = value != 0;
    else *k->ll = value;
    return PQP_OK;
}

extern "C" int pqp_tune_get(const char* key, long long* value) {
    if (!key || !value) return pqp::set_error(PQP_ERR_ARG, "pqp_tune_get: null argument");
    if (std::strcmp(key, "last_path") == 0) {
        *value = pqp::g_last_path;
        return PQP_OK;
    }
    if (std::strcmp(key, "last_batch_kernel") == 0) {  // 1: k_solve_pipe, 0: k_solve_single (path 2)
        *value = pqp::g_last_batch_kernel;
        return PQP_OK;
    }
    if (std::strcmp(key, "tiny_stale") == 0) {  // tiny solves whose pinned output lacked their tag
        *value = pqp::g_tiny_stale;
        return PQP_OK;
    }
    if (std::strcmp(key, "persist_fallbacks") == 0) {
        *value = pqp::g_persist_fallbacks;
        return PQP_OK;
    }
    if (std::strcmp(key, "batch_chunk_for") == 0) {  // in: N << 32 | M; out: iterates per batched launch
        const long long v = *value;
        *value = pqp::batch_chunk_for((int)(v >> 32), (int)(v & 0xffffffff));
        return PQP_OK;
    }
    if (std::strcmp(key, "converge_grid") == 0) {  // in: N << 32 | M
        const long long v = *value;
        *value = pqp::converge_persist_wgs((int)(v >> 32), (int)(v & 0xffffffff), nullptr);
        return PQP_OK;
    }
    const KnobRef* k = find_knob(key);
    if (!k) return pqp::set_error(PQP_ERR_ARG, "pqp_tune_get: unknown key '%s'", key);
    *value = knob_value(*k);
    return PQP_OK;
}

extern "C" int pqp_tune_trace(const char* what, void* d_buf, int n) {
    if (!what || n < 0 || (n > 0 && !d_buf)) return pqp::set_error(PQP_ERR_ARG, "pqp_tune_trace: bad arguments");
    auto* buf = n > 0 ? static_cast<unsigned long long*>(d_buf) : nullptr;
    std::lock_guard<std::mutex> lk(g_tune_mu);
    if (std::strcmp(what, "persist") == 0) {
        pqp::g_tune.persist_trace = buf;
        pqp::g_tune.persist_trace_n = n;
    } else if (std::strcmp(what, "mid") == 0) {
        pqp::g_tune.mid_trace = buf;
        pqp::g_tune.mid_trace_n = n;
    } else if (std::strcmp(what, "tiny") == 0) {
        // k_solve_quintet<..., true> writes kTinyTraceWords words unconditionally
        if (n > 0 && n < pqp::kTinyTraceWords)
            return pqp::set_error(PQP_ERR_ARG, "pqp_tune_trace: the tiny timeline needs %d words", pqp::kTinyTraceWords);
        pqp::g_tune.tiny_trace = buf;
    } else if (std::strcmp(what, "converge") == 0) {
        pqp::g_tune.converge_trace = buf;
        pqp::g_tune.converge_trace_n = n;
    } else {
        return pqp::set_error(PQP_ERR_ARG, "pqp_tune_trace: unknown timeline '%s'", what);
    }
    return PQP_OK;
}

extern "C" int pqp_tune_poison_lds(float value) {
    PQP_TRY(pqp::ensure_device());
    hipStream_t s = pqp::lib_stream();
    int dev = 0, cus = 0;
    PQP_HIP(hipGetDevice(&dev));
    PQP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    pqp::DevBuf seen;
    PQP_TRY(seen.alloc(sizeof(int)));
    int bits;
    std::memcpy(&bits, &value, sizeof bits);
    PQP_HIP(pqp::launch_poison_lds(bits, static_cast<int*>(seen.p), cus, s));
    PQP_HIP(hipStreamSynchronize(s));
    return PQP_OK;
}

extern "C" int pqp_tune_glibc_rand(int n, int* out) {
    if (n < 0 || (n > 0 && !out)) return pqp::set_error(PQP_ERR_ARG, "pqp_tune_glibc_rand: bad arguments");
    return pqp::glibc_rand_sequence(n, out);
}
