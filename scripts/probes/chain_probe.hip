// Probe: cost per add of a dependent fp32 add chain in the forms a lane-split
// update could use (gfx950, one workgroup of 4 waves = one wave per SIMD).
//   0 plain:  acc += p[m], products in the lane's own registers
//   1 dpp:    acc += row_shr:j(p[m]) (the product of a lane j to the left; the
//             compiler puts s_nop 1 before each DPP add: VALU write -> DPP read)
//   2 nop1:   plain adds with an s_nop 1 after each (the cost of the nop alone)
//   3 lds:    acc += products read from LDS, b128, only the chain lanes active
//   4 dpp2:   two interleaved chains (acc0 += dpp(p), acc1 += dpp(q)): the other
//             chain's add covers half of each hazard
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off chain_probe.hip -o chain_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int G = 64;  // products per lane per group
template <int J>
__device__ __forceinline__ float shr(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x110 + J, 0xF, 0xF, false));
}

template <int J>
__device__ __forceinline__ void dpp_group(float& acc, const float (&p)[G]) {
#pragma unroll
    for (int m = 0; m < G; ++m) acc += shr<J>(p[m]);
}
template <int J>
__device__ __forceinline__ void dpp_group2(float& a0, float& a1, const float (&p)[G]) {
#pragma unroll
    for (int m = 0; m < G; m += 2) {
        a0 += shr<J>(p[m]);
        a1 += shr<J>(p[m + 1]);
    }
}

template <int MODE>
__global__ void __launch_bounds__(256) k_chain(const float* __restrict__ in, float* out, long long* clk) {
    __shared__ __attribute__((aligned(16))) float lds[4][16 * G * 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float p[G];
#pragma unroll
    for (int m = 0; m < G; ++m) p[m] = in[(lane * G + m) & 4095] * 0.5f;
    if (MODE == 3) {  // the wave's 16 groups of products, [group][m] per chain lane
        for (int e = lane; e < 16 * G; e += 64) lds[w][e] = in[e & 4095] * 0.5f;
    }
    __syncthreads();
    float acc = 0.0f, acc1 = 0.0f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int m = 0; m < G; ++m) acc += p[m];
            asm volatile("" : "+v"(p[r]));
        }
    } else if (MODE == 1) {
#pragma unroll
        for (int m = 0; m < G; ++m) acc += p[m];
        dpp_group<1>(acc, p); dpp_group<2>(acc, p); dpp_group<3>(acc, p); dpp_group<4>(acc, p);
        dpp_group<5>(acc, p); dpp_group<6>(acc, p); dpp_group<7>(acc, p); dpp_group<8>(acc, p);
        dpp_group<9>(acc, p); dpp_group<10>(acc, p); dpp_group<11>(acc, p); dpp_group<12>(acc, p);
        dpp_group<13>(acc, p); dpp_group<14>(acc, p); dpp_group<15>(acc, p);
    } else if (MODE == 2) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int m = 0; m < G; ++m) {
                acc += p[m];
                asm volatile("s_nop 1" : "+v"(acc));
            }
        }
    } else if (MODE == 3) {
        if ((lane & 15) == 15) {
            const float4* q = reinterpret_cast<const float4*>(lds[w]);
#pragma unroll 16
            for (int e = 0; e < 16 * G / 4; ++e) {
                const float4 v = q[e];
                acc += v.x;
                acc += v.y;
                acc += v.z;
                acc += v.w;
            }
        }
    } else {
        dpp_group2<1>(acc, acc1, p); dpp_group2<2>(acc, acc1, p); dpp_group2<3>(acc, acc1, p);
        dpp_group2<4>(acc, acc1, p); dpp_group2<5>(acc, acc1, p); dpp_group2<6>(acc, acc1, p);
        dpp_group2<7>(acc, acc1, p); dpp_group2<8>(acc, acc1, p); dpp_group2<9>(acc, acc1, p);
        dpp_group2<10>(acc, acc1, p); dpp_group2<11>(acc, acc1, p); dpp_group2<12>(acc, acc1, p);
        dpp_group2<13>(acc, acc1, p); dpp_group2<14>(acc, acc1, p); dpp_group2<15>(acc, acc1, p);
        dpp_group2<15>(acc, acc1, p);
    }
    asm volatile("" : "+v"(acc), "+v"(acc1));
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = acc + acc1;
    if (lane == 0) clk[blockIdx.x * 4 + w] = t1 - t0;
}

int main() {
    float *in, *out;
    long long* clk;
    (void)hipMalloc(&in, 4096 * 4);
    (void)hipMalloc(&out, 256 * 256 * 4);
    (void)hipMalloc(&clk, 256 * 4 * 8);
    float h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = 1.0f + (i % 97) * 0.01f;
    (void)hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const char* names[] = {"plain", "dpp", "nop1", "lds_b128", "dpp_two_chains"};
    const int adds[] = {16 * G, 16 * G, 16 * G, 16 * G, 8 * G};  // per chain
    for (int mode = 0; mode < 5; ++mode) {
        for (int wgs : {1, 128}) {
            for (int rep = 0; rep < 3; ++rep) {
                switch (mode) {
                    case 0: hipLaunchKernelGGL(k_chain<0>, dim3(wgs), dim3(256), 0, 0, in, out, clk); break;
                    case 1: hipLaunchKernelGGL(k_chain<1>, dim3(wgs), dim3(256), 0, 0, in, out, clk); break;
                    case 2: hipLaunchKernelGGL(k_chain<2>, dim3(wgs), dim3(256), 0, 0, in, out, clk); break;
                    case 3: hipLaunchKernelGGL(k_chain<3>, dim3(wgs), dim3(256), 0, 0, in, out, clk); break;
                    default: hipLaunchKernelGGL(k_chain<4>, dim3(wgs), dim3(256), 0, 0, in, out, clk); break;
                }
            }
            (void)hipDeviceSynchronize();
            long long hc[4];
            (void)hipMemcpy(hc, clk, sizeof hc, hipMemcpyDeviceToHost);
            printf("{\"form\": \"%s\", \"wgs\": %d, \"clk_per_add\": [%.2f, %.2f, %.2f, %.2f]}\n", names[mode], wgs,
                   hc[0] / (double)adds[mode], hc[1] / (double)adds[mode], hc[2] / (double)adds[mode],
                   hc[3] / (double)adds[mode]);
        }
    }
    return 0;
}
