// Probe: which SIMD each wave of a 6-wave workgroup runs on (HW_ID register,
// SIMD_ID bits 5:4 on gfx9), for workgroups of 1 per CU (large LDS).
// Build: hipcc --offload-arch=gfx950 -O3 simd_map_probe.hip -o simd_map_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(384) k_map(unsigned* out) {
    extern __shared__ float lds[];
    const unsigned id = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // hwreg(HW_REG_HW_ID, 0, 32)
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 6 + (threadIdx.x >> 6)] = id;
    lds[threadIdx.x] = (float)id;
}

int main() {
    unsigned* out;
    (void)hipMalloc(&out, 64 * 6 * 4);
    hipLaunchKernelGGL(k_map, dim3(64), dim3(384), 140 * 1024, 0, out);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    unsigned h[64 * 6];
    (void)hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
    for (int b = 0; b < 8; ++b) {
        printf("wg %d:", b);
        for (int w = 0; w < 6; ++w) printf(" w%d simd=%u wave=%u cu=%u", w, (h[b * 6 + w] >> 4) & 3, h[b * 6 + w] & 15,
                                           (h[b * 6 + w] >> 8) & 15);
        printf("\n");
    }
    return 0;
}
