// Probe: per-launch cost of a chain of dependent kernels replayed from a
// hipGraph (the single-problem update is one such launch per iteration), and
// of a grid barrier inside one persistent kernel as the alternative.
// Build: hipcc --offload-arch=gfx950 -O3 launch_probe.hip -o launch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(float* y) {
    if (threadIdx.x == 0 && blockIdx.x == 100000) y[0] = 1.0f;
}
// reads the 1024-float vector the previous launch wrote, writes its slice
__global__ void k_dep(const float* __restrict__ yin, float* __restrict__ yout) {
    __shared__ float ys[1024];
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) ys[k] = yin[k];
    __syncthreads();
    const int i = blockIdx.x * 32 + (threadIdx.x & 31);
    if (threadIdx.x < 32) yout[i] = ys[i] * 0.5f + ys[(i + 1) & 1023];
}
// persistent: `iters` rounds of (read y, write slice, grid barrier)
__global__ void k_persist(float* ya, float* yb, unsigned* bar, int iters) {
    __shared__ float ys[1024];
    float* a = ya;
    float* b = yb;
    const unsigned nb = gridDim.x;
    for (int it = 0; it < iters; ++it) {
        for (int k = threadIdx.x; k < 1024; k += blockDim.x) ys[k] = __hip_atomic_load(a + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int i = blockIdx.x * 32 + (threadIdx.x & 31);
        if (threadIdx.x < 32) __hip_atomic_store(b + i, ys[i] * 0.5f + ys[(i + 1) & 1023], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (threadIdx.x == 0) {
            __atomic_thread_fence(__ATOMIC_RELEASE);
            __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = nb * (unsigned)(it + 1);
            for (int spin = 0;; ++spin) {
                if (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
                if (spin > (1 << 16) || __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    __hip_atomic_store(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // abort all
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        if (__hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        float* t = a;
        a = b;
        b = t;
    }
}

int main() {
    float *ya, *yb;
    unsigned* bar;
    (void)hipMalloc(&ya, 4096);
    (void)hipMalloc(&yb, 4096);
    (void)hipMalloc(&bar, 8);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    (void)hipMemset(ya, 0, 4096);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const int n = 1000;
    for (int which = 0; which < 2; ++which) {
        for (int threads : {64, 512}) {
            hipGraph_t g;
            hipGraphExec_t ge;
            (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
            for (int i = 0; i < n; ++i) {
                if (which == 0)
                    hipLaunchKernelGGL(k_empty, dim3(32), dim3(threads), 0, s, ya);
                else
                    hipLaunchKernelGGL(k_dep, dim3(32), dim3(threads), 0, s, (i & 1) ? yb : ya, (i & 1) ? ya : yb);
            }
            (void)hipStreamEndCapture(s, &g);
            (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            (void)hipGraphLaunch(ge, s);
            (void)hipStreamSynchronize(s);
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a, s);
            (void)hipGraphLaunch(ge, s);
            (void)hipEventRecord(b, s);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("{\"chain\": \"%s\", \"threads\": %d, \"us_per_launch\": %.3f}\n", which ? "dep" : "empty", threads,
                   ms * 1e3 / n);
        }
    }
    for (int wgs : {32, 128}) {
        (void)hipMemsetAsync(bar, 0, 8, s);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        (void)hipEventRecord(a, s);
        hipLaunchKernelGGL(k_persist, dim3(wgs), dim3(512), 0, s, ya, yb, bar, n);
        (void)hipEventRecord(b, s);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        unsigned hb[2];
        (void)hipMemcpy(hb, bar, 8, hipMemcpyDeviceToHost);
        printf("{\"chain\": \"persistent grid barrier\", \"wgs\": %d, \"us_per_iter\": %.3f, \"count\": %u, \"aborted\": %u}\n",
               wgs, ms * 1e3 / n, hb[0], hb[1]);
    }
    return 0;
}
