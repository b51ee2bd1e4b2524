// Probe: aggregate read bandwidth when every CU streams its own slice of a
// buffer that fits the 256 MiB Infinity Cache, vs one that does not.
// Build: hipcc --offload-arch=gfx950 -O3 mall_probe.hip -o mall_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4v __attribute__((ext_vector_type(4)));

template <int U>
__global__ void __launch_bounds__(256) k_read(const f4v* __restrict__ buf, size_t per_wg, int passes, float* out) {
    const f4v* p = buf + (size_t)blockIdx.x * per_wg;
    f4v acc = {0, 0, 0, 0};
    for (int r = 0; r < passes; ++r) {
        for (size_t i = threadIdx.x; i < per_wg; i += 256 * U) {
            f4v v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = (i + 256 * u < per_wg) ? p[i + 256 * u] : f4v{0, 0, 0, 0};
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u];
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

int main() {
    const int wgs_list[] = {256, 512, 1024};
    const size_t sizes_mb[] = {64, 128, 192, 2048};
    float* out;
    hipMalloc(&out, sizeof(float) * 1024 * 256);
    for (size_t mb : sizes_mb) {
        const size_t bytes = mb << 20;
        f4v* buf;
        hipMalloc(&buf, bytes);
        hipMemset(buf, 0, bytes);
        for (int wgs : wgs_list) {
            const size_t per_wg = bytes / 16 / wgs;
            const int passes = mb >= 1024 ? 2 : 20;
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipLaunchKernelGGL(k_read<8>, dim3(wgs), dim3(256), 0, 0, buf, per_wg, 1, out);
            hipEventRecord(a);
            hipLaunchKernelGGL(k_read<8>, dim3(wgs), dim3(256), 0, 0, buf, per_wg, passes, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("{\"MiB\": %zu, \"wgs\": %d, \"passes\": %d, \"TBps\": %.3f}\n", mb, wgs, passes,
                   (double)per_wg * 16 * wgs * passes / (ms * 1e-3) / 1e12);
        }
        hipFree(buf);
    }
    return 0;
}
