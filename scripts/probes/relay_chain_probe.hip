// Probe: a 6-wave relay of add chains, the shape of k_split_persist's update
// (wave w adds its L products, hands the running sums to wave w + 1 through
// one 64-bit LDS word per lane; wave 0 takes over from wave 5 for the next
// round).  Reports clocks per round and per hand-off (round time minus the
// adds, measured alone) for:
//   0 spin:   every waiting wave polls its predecessor's word in a tight loop
//   1 doze:   a wave whose predecessor has not started yet (the word of the
//             wave before that is not set) sleeps between polls
//   2 prio:   as 0, the chaining wave at s_setprio 3
//   3 doze+prio
//   4 sweep:  as 0, but the waiting waves also poll a global buffer with
//             agent-scope (sc1) 8-byte loads between LDS polls, as the
//             granule sweep of the next update does (s_sleep 1 between sweeps)
//   8 bystand: pure LDS waits, but a wave that has handed on its sums polls
//             the global buffer (sc1 loads, s_sleep 1) until the round's last
//             wave is done -- the granule sweep of k_split_persist's next
//             update, running beside the later waves' chains and hand-offs
//   10 bystand+prio
//   16 products: before waiting for its turn, a wave forms 48 packets of
//             products from LDS (b128 q and y reads, v_pk_mul), as
//             k_split_persist's slices do; the chain itself is unchanged
// Grids of 1 and 64 workgroups (one per CU), the kernel's own geometry.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off relay_chain_probe.hip -o relay_chain_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 6, L = 192, kRounds = 200;

template <int MODE>
__global__ void __launch_bounds__(64 * W) k_relay(const float* __restrict__ in, float* out, long long* clk,
                                                  unsigned long long* gbuf) {
    __shared__ unsigned long long slot[W][64];
    __shared__ __attribute__((aligned(16))) float4 qlds[48 * 32 + 48];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    typedef float f2v __attribute__((ext_vector_type(2)));
    typedef float f4v __attribute__((ext_vector_type(4)));
    float p[(MODE & 16) ? 1 : L];
    if (!(MODE & 16)) {
#pragma unroll
        for (int m = 0; m < L; ++m) p[m] = in[(lane * 7 + m * 13 + w) & 4095] * 1e-3f;
    }
    f4v pr[(MODE & 16) ? L / 4 : 1];
    slot[w][lane] = 0ull;
    for (int e = threadIdx.x; e < 48 * 32 + 48; e += blockDim.x) qlds[e] = make_float4(1.0f, 2.0f, 3.0f, 4.0f);
    __syncthreads();
    float sink = 0.0f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    float acc = 0.0f;
    for (int r = 0; r < kRounds; ++r) {
        const int prev = w == 0 ? W - 1 : w - 1;
        const unsigned want = w == 0 ? (unsigned)r : (unsigned)r + 1u;  // round r of wave 5 ends with tag r
        if (MODE & 16) {  // this round's products, ahead of the turn
            const float4* qw = qlds + (lane & 31);
            const float4* yw = qlds + 48 * 32;
#pragma unroll
            for (int j = 0; j < L / 4; ++j) {
                const float4 q = qw[j * 32], y = yw[j];
                const f2v lo = f2v{q.x, q.y} * f2v{y.x, y.y};
                const f2v hi = f2v{q.z, q.w} * f2v{y.z, y.w};
                pr[j] = f4v{lo.x, lo.y, hi.x, hi.y};
            }
#pragma unroll
            for (int j = 0; j < L / 4; ++j) asm volatile("" : "+v"(pr[j]));
        }
        if (!(w == 0 && r == 0)) {
            const int prev2 = prev == 0 ? W - 1 : prev - 1;
            const unsigned want2 = prev == 0 ? want - 1u : want;  // predecessor's predecessor, same hand-off chain
            for (;;) {
                const unsigned long long h = __hip_atomic_load(&slot[prev][lane], __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                if (__all((unsigned)(h >> 32) == want)) {
                    acc = __uint_as_float((unsigned)h);
                    break;
                }
                if (MODE & 4) {
                    unsigned long long acc4 = 0;
#pragma unroll
                    for (int m = 0; m < 4; ++m)
                        acc4 += __hip_atomic_load(gbuf + blockIdx.x * 256 + 64 * m + lane, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
                    if (__all(acc4 == 12345ull)) acc += 1.0f;
                    __builtin_amdgcn_s_sleep(1);
                }
                if (MODE & 1) {
                    const unsigned long long h2 = __hip_atomic_load(&slot[prev2][lane], __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (!__all((unsigned)(h2 >> 32) == want2)) __builtin_amdgcn_s_sleep(2);
                }
            }
        }
        if (MODE & 2) __builtin_amdgcn_s_setprio(3);
        if (MODE & 16) {
#pragma unroll
            for (int j = 0; j < L / 4; ++j) {
                acc += pr[j].x;
                acc += pr[j].y;
                acc += pr[j].z;
                acc += pr[j].w;
            }
        } else {
#pragma unroll
            for (int m = 0; m < L; ++m) acc += p[m];
        }
        asm volatile("" : "+v"(acc));
        const unsigned tag = w == W - 1 ? (unsigned)r + 1u : (unsigned)r + 1u;
        __hip_atomic_store(&slot[w][lane], ((unsigned long long)tag << 32) | __float_as_uint(acc), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        if (MODE & 2) __builtin_amdgcn_s_setprio(0);
        if ((MODE & 8) && w < W - 1) {
            for (;;) {  // the next update's sweep, until the round's last wave is done
                unsigned long long acc4 = 0;
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    acc4 += __hip_atomic_load(gbuf + blockIdx.x * 256 + 64 * m + lane, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                if (__all(acc4 == 12345ull)) acc += 1.0f;
                const unsigned long long h5 = __hip_atomic_load(&slot[W - 1][lane], __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_WORKGROUP);
                if (__all((unsigned)(h5 >> 32) == (unsigned)r + 1u)) break;
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 * W + threadIdx.x] = acc + sink;
    if (lane == 0 && blockIdx.x == 0) clk[w] = t1 - t0;
}

// the adds alone: one wave, W * L adds per round
__global__ void __launch_bounds__(64) k_alone(const float* __restrict__ in, float* out, long long* clk) {
    const int lane = threadIdx.x & 63;
    float p[L];
#pragma unroll
    for (int m = 0; m < L; ++m) p[m] = in[(lane * 7 + m * 13) & 4095] * 1e-3f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    float acc = 0.0f;
    for (int r = 0; r < kRounds * W; ++r) {
#pragma unroll
        for (int m = 0; m < L; ++m) acc += p[m];
        asm volatile("" : "+v"(acc));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (lane == 0) clk[0] = t1 - t0;
}

int main() {
    float *in, *out;
    long long* clk;
    (void)hipMalloc(&in, 4096 * 4);
    (void)hipMalloc(&out, 64 * W * 4);
    (void)hipMalloc(&clk, W * 8);
    unsigned long long* gbuf;
    (void)hipMalloc(&gbuf, 64 * 256 * 8);
    (void)hipMemset(gbuf, 0, 64 * 256 * 8);
    (void)hipFree(out);
    (void)hipMalloc(&out, 64 * 64 * W * 4);
    float h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = 1.0f + (i % 97) * 0.01f;
    (void)hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    long long hc[W];
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_alone, dim3(1), dim3(64), 0, 0, in, out, clk);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    (void)hipMemcpy(hc, clk, 8, hipMemcpyDeviceToHost);
    const double add = hc[0] / (double)(kRounds * W * L);
    printf("{\"form\": \"adds alone\", \"clk_per_add\": %.3f}\n", add);
    const char* names[] = {"spin", "doze", "prio", "doze+prio", "sweep", "", "sweep+prio", "", "bystand", "", "bystand+prio", "", "", "", "", "", "products"};
    for (int mode : {0, 2, 16}) {
        for (int wgs : {1, 64}) {
            for (int rep = 0; rep < 3; ++rep) {
                switch (mode) {
                    case 0: hipLaunchKernelGGL(k_relay<0>, dim3(wgs), dim3(64 * W), 0, 0, in, out, clk, gbuf); break;
                    case 1: hipLaunchKernelGGL(k_relay<1>, dim3(wgs), dim3(64 * W), 0, 0, in, out, clk, gbuf); break;
                    case 2: hipLaunchKernelGGL(k_relay<2>, dim3(wgs), dim3(64 * W), 0, 0, in, out, clk, gbuf); break;
                    case 3: hipLaunchKernelGGL(k_relay<3>, dim3(wgs), dim3(64 * W), 0, 0, in, out, clk, gbuf); break;
                    case 4: hipLaunchKernelGGL(k_relay<4>, dim3(wgs), dim3(64 * W), 0, 0, in, out, clk, gbuf); break;
                    case 8: hipLaunchKernelGGL(k_relay<8>, dim3(wgs), dim3(64 * W), 0, 0, in, out, clk, gbuf); break;
                    case 10: hipLaunchKernelGGL(k_relay<10>, dim3(wgs), dim3(64 * W), 0, 0, in, out, clk, gbuf); break;
                    case 16: hipLaunchKernelGGL(k_relay<16>, dim3(wgs), dim3(64 * W), 0, 0, in, out, clk, gbuf); break;
                    default: hipLaunchKernelGGL(k_relay<6>, dim3(wgs), dim3(64 * W), 0, 0, in, out, clk, gbuf); break;
                }
            }
            if (hipDeviceSynchronize() != hipSuccess) return 1;
            (void)hipMemcpy(hc, clk, sizeof hc, hipMemcpyDeviceToHost);
            const double round = hc[0] / (double)kRounds;
            printf("{\"form\": \"%s\", \"wgs\": %d, \"clk_per_round\": %.1f, \"clk_per_handoff\": %.1f}\n",
                   names[mode], wgs, round, (round - W * L * add) / W);
        }
    }
    return 0;
}
