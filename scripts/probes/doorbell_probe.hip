// Probe: what a persistent, pre-launched one-problem
// server would save per solve against the one-launch tiny solve's launch and
// synchronisation (pqp_problem_solve of the bundled problem: one launch, the
// results written by the kernel to fine-grained pinned host memory, then
// hipStreamSynchronize).
//
//   launch_sync   : launch a one-wave kernel that writes its tag to pinned
//                   host memory (system-scope store), hipStreamSynchronize,
//                   check the tag -- the per-solve overhead of today's path
//   launch_spin   : the same launch, the host spinning on the pinned tag
//                   instead of synchronising the stream
//   launch_query  : the same launch, the host polling hipStreamQuery until the
//                   stream is idle (the completion signal: the same ordering
//                   guarantee as a synchronisation), then reading the tag
//   doorbell      : ONE kernel launched once; its wave polls a doorbell word
//                   in pinned host memory (vector system-scope loads), answers
//                   each ring with a tag store to pinned memory; the host rings
//                   and spins on the answer -- the per-solve overhead of a
//                   server.  Every wait is bounded (the kernel leaves after
//                   kIdle polls without a ring, and after the last request).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 doorbell_probe.hip -o doorbell_probe
// Run:   ./doorbell_probe [requests=2000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

__device__ __forceinline__ int sys_load(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(64) k_tag(int* out, int tag) {
    if (threadIdx.x == 0) sys_store(out, tag);
}

constexpr long long kIdle = 1LL << 20;  // polls without a ring before the server leaves (about a second)

__global__ void __launch_bounds__(64) k_server(const int* bell, int* out, int requests) {
    int want = 1;
    long long idle = 0;
    while (want <= requests && idle < kIdle) {
        const int b = sys_load(bell);  // every lane loads (vector load); the value is uniform
        if (b >= want) {
            if (threadIdx.x == 0) sys_store(out, b);
            want = b + 1;
            idle = 0;
        } else {
            ++idle;
        }
    }
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 2000;
    int *hbell, *hout, *dbell, *dout;
    CK(hipHostMalloc((void**)&hbell, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&hout, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&dbell, hbell, 0));
    CK(hipHostGetDevicePointer((void**)&dout, hout, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    volatile int* vout = hout;
    volatile int* vbell = hbell;
    using clk = std::chrono::steady_clock;
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };

    // warm up
    *vout = 0;
    for (int i = 1; i <= 50; ++i) hipLaunchKernelGGL(k_tag, dim3(1), dim3(64), 0, s, dout, i);
    CK(hipStreamSynchronize(s));

    std::vector<double> t_sync, t_spin, t_bell, t_query;
    for (int i = 1; i <= R; ++i) {
        const auto a = clk::now();
        hipLaunchKernelGGL(k_tag, dim3(1), dim3(64), 0, s, dout, 100000 + i);
        CK(hipStreamSynchronize(s));
        const auto b = clk::now();
        if (*vout != 100000 + i) { fprintf(stderr, "launch_sync: tag missing\n"); return 1; }
        t_sync.push_back(us(a, b));
    }
    for (int i = 1; i <= R; ++i) {
        const auto a = clk::now();
        hipLaunchKernelGGL(k_tag, dim3(1), dim3(64), 0, s, dout, 200000 + i);
        long long spins = 0;
        while (*vout != 200000 + i && ++spins < (1LL << 32)) {}
        const auto b = clk::now();
        t_spin.push_back(us(a, b));
    }
    CK(hipStreamSynchronize(s));
    for (int i = 1; i <= R; ++i) {
        const auto a = clk::now();
        hipLaunchKernelGGL(k_tag, dim3(1), dim3(64), 0, s, dout, 300000 + i);
        hipError_t q;
        while ((q = hipStreamQuery(s)) == hipErrorNotReady) {}
        CK(q);
        const auto b = clk::now();
        if (*vout != 300000 + i) { fprintf(stderr, "launch_query: tag missing\n"); return 1; }
        t_query.push_back(us(a, b));
    }

    *vbell = 0;
    *vout = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipLaunchKernelGGL(k_server, dim3(1), dim3(64), 0, s, dbell, dout, R);
    bool ok = true;
    for (int i = 1; i <= R && ok; ++i) {
        const auto a = clk::now();
        *vbell = i;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        long long spins = 0;
        while (*vout != i) {
            if (++spins > (1LL << 33)) { ok = false; break; }
        }
        const auto b = clk::now();
        t_bell.push_back(us(a, b));
    }
    CK(hipStreamSynchronize(s));
    printf("{\"requests\": %d, \"launch_query_us\": %.2f, \"launch_sync_us\": %.2f, \"launch_spin_us\": %.2f, \"doorbell_us\": %.2f, "
           "\"doorbell_ok\": %s, \"launch_sync_p90_us\": %.2f, \"doorbell_p90_us\": %.2f}\n",
           R, median(t_query), median(t_sync), median(t_spin), t_bell.empty() ? -1.0 : median(t_bell), ok ? "true" : "false",
           [&] { auto v = t_sync; std::sort(v.begin(), v.end()); return v[v.size() * 9 / 10]; }(),
           [&] { auto v = t_bell; std::sort(v.begin(), v.end()); return v.empty() ? -1.0 : v[v.size() * 9 / 10]; }());
    return ok ? 0 : 1;
}
