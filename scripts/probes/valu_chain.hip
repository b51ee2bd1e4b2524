// Probe: what a dependent f32 add chain costs per add on gfx950 (the horizon
// kernel's sums are such chains), one workgroup of W waves on one CU:
//   dep_add    : v_add_f32 s = s + x, each add waiting on the one before
//   dep_pk_add : v_pk_add_f32 on a packed pair, likewise
//   ind_add    : 8 independent v_add_f32 chains interleaved (issue cost)
//   mul_add    : v_mul_f32 p = a * b then s = s + p per term (a dot's term)
//   lds_b128   : ds_read_b128 issued and waited for, dependent addresses
// Cycles per operation (s_memtime, shader clock), median over waves.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 valu_chain.hip -o valu_chain
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int kReps = 1024;

template <int MODE>
__global__ void k_chain(float* out, unsigned long long* cyc, float x) {
    __shared__ float lds[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = 0.0f;
    __syncthreads();
    float s = threadIdx.x * 1e-7f, t = 1.0f;
    float a0 = s, a1 = s, a2 = s, a3 = s, a4 = s, a5 = s, a6 = s, a7 = s;
    int addr = (threadIdx.x & 63) * 16;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < kReps; ++r) {
        if constexpr (MODE == 0) {
            asm volatile(
                "v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n"
                "v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1"
                : "+v"(s) : "v"(x));
        } else if constexpr (MODE == 1) {
            asm volatile(
                "v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n"
                "v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1"
                : "+v"(*reinterpret_cast<double*>(&a0)) : "v"(*reinterpret_cast<double*>(&a2)));
        } else if constexpr (MODE == 2) {
            asm volatile(
                "v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
                "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x));
        } else if constexpr (MODE == 3) {
            float p;
            asm volatile(
                "v_mul_f32 %1, %2, %3\n v_add_f32 %0, %0, %1\n v_mul_f32 %1, %2, %3\n v_add_f32 %0, %0, %1\n"
                "v_mul_f32 %1, %2, %3\n v_add_f32 %0, %0, %1\n v_mul_f32 %1, %2, %3\n v_add_f32 %0, %0, %1\n"
                "v_mul_f32 %1, %2, %3\n v_add_f32 %0, %0, %1\n v_mul_f32 %1, %2, %3\n v_add_f32 %0, %0, %1\n"
                "v_mul_f32 %1, %2, %3\n v_add_f32 %0, %0, %1\n v_mul_f32 %1, %2, %3\n v_add_f32 %0, %0, %1"
                : "+v"(s), "=&v"(p) : "v"(x), "v"(t));
        } else {
            float v0, v1, v2, v3;
            asm volatile(
                "ds_read_b128 %1, %0\n s_waitcnt lgkmcnt(0)\n v_and_b32 %0, 0x3f0, %1\n"
                : "+v"(addr), "=v"(*reinterpret_cast<float4*>(&v0))::"memory");
            (void)v1; (void)v2; (void)v3;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = t1 - t0;
    out[threadIdx.x] = s + t + a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)addr;
}

template <int MODE>
double run(int waves, float* out, unsigned long long* cyc, int ops_per_rep) {
    hipLaunchKernelGGL(k_chain<MODE>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, 1e-9f);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(waves);
    CK(hipMemcpy(h.data(), cyc, 8 * waves, hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    return (double)h[waves / 2] / (kReps * (double)ops_per_rep);
}

int main() {
    float* out;
    unsigned long long* cyc;
    CK(hipMalloc(&out, 4 * 1024));
    CK(hipMalloc(&cyc, 8 * 16));
    printf("{");
    const int W[] = {1, 4, 8, 16};
    for (int wi = 0; wi < 4; ++wi) {
        const int w = W[wi];
        run<0>(w, out, cyc, 8);  // warm
        printf("\"w%d\": {\"dep_add\": %.2f, \"dep_pk_add\": %.2f, \"ind_add\": %.2f, \"mul_add_term\": %.2f, "
               "\"lds_b128_dep\": %.1f}%s",
               w, run<0>(w, out, cyc, 8), run<1>(w, out, cyc, 8), run<2>(w, out, cyc, 8), run<3>(w, out, cyc, 8),
               run<4>(w, out, cyc, 1), wi < 3 ? ", " : "");
    }
    printf("}\n");
    return 0;
}
