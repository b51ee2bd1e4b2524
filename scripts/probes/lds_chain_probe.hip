// Probe: a dependent fp32 add chain whose terms come from LDS (products
// formed elsewhere), the reads D packets (of 4 terms) ahead of the adds in a
// register ring, one wave per SIMD, all lanes active (one row side per lane).
// Prints clocks per add for D = 2, 4, 8, 12 and for the same chain over
// registers.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off lds_chain_probe.hip -o lds_chain_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int KP = 256;  // packets per chain (1024 terms)

template <int D>
__global__ void __launch_bounds__(256) k_lds_chain(const float* __restrict__ in, float* out, long long* clk) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    f4v* q = reinterpret_cast<f4v*>(lds);  // [KP / 4 waves ... ] one ring of packets shared by the 4 waves
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // 32 KiB of packets: [p][64 lanes] for p < 32, re-read 8 times = 256 packets
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
        const int i = e * 4;
        q[e] = f4v{in[i & 4095], in[(i + 1) & 4095], in[(i + 2) & 4095], in[(i + 3) & 4095]} * 1e-3f;
    }
    __syncthreads();
    const f4v* qw = q + lane;
    float acc = 0.0f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    f4v ring[D];
#pragma unroll
    for (int j = 0; j < D; ++j) ring[j] = qw[(j & 31) * 64];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < KP; ++j) {
        const f4v v = ring[j % D];
        if (j + D < KP) ring[j % D] = qw[((j + D) & 31) * 64];
        acc += v.x;
        acc += v.y;
        acc += v.z;
        acc += v.w;
        __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("" : "+v"(acc));
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (lane == 0) clk[blockIdx.x * 4 + w] = t1 - t0;
}

__global__ void __launch_bounds__(256) k_reg_chain(const float* __restrict__ in, float* out, long long* clk) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float p[64];
#pragma unroll
    for (int m = 0; m < 64; ++m) p[m] = in[(lane * 64 + m) & 4095] * 1e-3f;
    float acc = 0.0f;
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
        for (int m = 0; m < 64; ++m) acc += p[m];
        asm volatile("" : "+v"(p[r]));
    }
    asm volatile("" : "+v"(acc));
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (lane == 0) clk[blockIdx.x * 4 + w] = t1 - t0;
}

template <int D>
static void run(const float* in, float* out, long long* clk, int waves) {
    long long h[4];
    for (int rep = 0; rep < 3; ++rep)
        hipLaunchKernelGGL(k_lds_chain<D>, dim3(1), dim3(64 * waves), 32 * 64 * 16, 0, in, out, clk);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
    printf("{\"form\": \"lds D=%d\", \"waves\": %d, \"clk_per_add_wave0\": %.2f}\n", D, waves, h[0] / (4.0 * KP));
}

int main() {
    float *in, *out;
    long long* clk;
    (void)hipMalloc(&in, 4096 * 4);
    (void)hipMalloc(&out, 256 * 4);
    (void)hipMalloc(&clk, 4 * 8);
    float h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = 1.0f + (i % 97) * 0.01f;
    (void)hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    long long hc[4];
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_reg_chain, dim3(1), dim3(64), 0, 0, in, out, clk);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(hc, clk, sizeof hc, hipMemcpyDeviceToHost);
    printf("{\"form\": \"registers\", \"clk_per_add\": %.2f}\n", hc[0] / 1024.0);
    for (int waves : {1, 4}) {
        run<2>(in, out, clk, waves);
        run<4>(in, out, clk, waves);
        run<8>(in, out, clk, waves);
        run<12>(in, out, clk, waves);
    }
    return 0;
}
