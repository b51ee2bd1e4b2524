// Probe: the latency of one dependent v_add_f32 on gfx950 -- the floor of
// any sequential k-ordered sum, and so of one update of one problem (the
// reference's row sum is N adds in k order; configs[2] has N = 1024).
// One wave alone, a register-only chain of 64 adds per asm block, s_memtime
// around 1000 blocks; also two interleaved chains (the den / num pair of a
// row) and the same with a v_mul_f32 feeding each add (a dot's term).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 add_chain_probe.hip -o add_chain_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

#define A1(d, s) "v_add_f32 " d ", " d ", " s "\n"
#define A8(d, s) A1(d, s) A1(d, s) A1(d, s) A1(d, s) A1(d, s) A1(d, s) A1(d, s) A1(d, s)
#define A64(d, s) A8(d, s) A8(d, s) A8(d, s) A8(d, s) A8(d, s) A8(d, s) A8(d, s) A8(d, s)
#define AA8 "v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %2\n"  // one add of each chain
#define AA64 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 \
             AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8 AA8
#define MA "v_mul_f32 %1, %2, %3\n v_add_f32 %0, %0, %1\n"
#define MA8 MA MA MA MA MA MA MA MA
#define MA64 MA8 MA8 MA8 MA8 MA8 MA8 MA8 MA8

constexpr int kReps = 1000;

template <int MODE>
__global__ void __launch_bounds__(64) k_chain(float* out, unsigned long long* cyc, float x) {
    float s = threadIdx.x * 1e-7f, t = 0.5f, p = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < kReps; ++r) {
        if constexpr (MODE == 0) asm volatile(A64("%0", "%1") : "+v"(s) : "v"(x));
        else if constexpr (MODE == 1) asm volatile(AA64 : "+v"(s), "+v"(t) : "v"(x));
        else asm volatile(MA64 : "+v"(s), "=&v"(p) : "v"(x), "v"(t));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) *cyc = t1 - t0;
    out[threadIdx.x] = s + t + p;
}

template <int MODE>
double run(float* out, unsigned long long* cyc) {
    hipLaunchKernelGGL(k_chain<MODE>, dim3(1), dim3(64), 0, 0, out, cyc, 1e-9f);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_chain<MODE>, dim3(1), dim3(64), 0, 0, out, cyc, 1e-9f);
    CK(hipDeviceSynchronize());
    unsigned long long h;
    CK(hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost));
    return (double)h / (kReps * 64.0);
}

int main() {
    float* out;
    unsigned long long* cyc;
    CK(hipMalloc(&out, 4 * 64));
    CK(hipMalloc(&cyc, 8));
    printf("{\"cycles_per_dependent_add\": %.2f, \"cycles_per_add_pair_two_chains\": %.2f, "
           "\"cycles_per_mul_add_term\": %.2f}\n",
           run<0>(out, cyc), run<1>(out, cyc), run<2>(out, cyc));
    return 0;
}
