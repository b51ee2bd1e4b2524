// Probe: latency of one wave -> wave hand-off inside a workgroup (the running
// sums of k_split_persist pass from wave to wave this way).  Two waves play
// ping-pong through one LDS word, 2000 hand-offs; clocks per hand-off:
//   0 poll:    ds_read in a tight loop until the word holds the token
//   1 poll+sl: the same with s_sleep 1 between reads
//   2 wakeup:  the waiter sleeps (s_sleep 8 in a loop); the writer stores the
//              token, waits for the store (lgkmcnt 0) and issues s_wakeup
//   3 poll64:  64-lane ds_read_b64 of per-lane words + __all (the shipped form)
// Build: hipcc --offload-arch=gfx950 -O3 handoff_probe.hip -o handoff_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kRounds = 1000;

template <int MODE>
__global__ void __launch_bounds__(128) k_pingpong(long long* clk, int* bad) {
    __shared__ unsigned word[2];
    __shared__ unsigned long long wide[64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 2) word[threadIdx.x] = 0;
    if (threadIdx.x < 64) wide[threadIdx.x] = 0;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    long long spins = 0;
    for (int r = 0; r < kRounds; ++r) {
        const unsigned tok = 2u * r + 1u + (unsigned)w;  // wave 0 writes odd tokens, wave 1 even
        const unsigned want = tok - 1u;
        if (!(w == 0 && r == 0)) {  // wait for the other wave's previous token
            if (MODE == 3) {
                for (;;) {
                    const unsigned long long h =
                        __hip_atomic_load(&wide[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (__all((unsigned)(h >> 32) == want)) break;
                    ++spins;
                }
            } else {
                for (;;) {
                    const unsigned v = __hip_atomic_load(&word[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (__builtin_amdgcn_readfirstlane(v) == want) break;
                    ++spins;
                    if (MODE == 1) __builtin_amdgcn_s_sleep(1);
                    if (MODE == 2) __builtin_amdgcn_s_sleep(8);
                }
            }
        }
        if (MODE == 3) {
            __hip_atomic_store(&wide[lane], ((unsigned long long)tok << 32) | lane, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            if (lane == 0) __hip_atomic_store(&word[0], tok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (MODE == 2) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                asm volatile("s_wakeup" ::: "memory");
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        clk[w] = t1 - t0;
        clk[2 + w] = spins;
    }
    if (lane == 0 && w == 1 && word[0] != 2u * kRounds && MODE != 3) *bad = 1;
}

int main() {
    long long* clk;
    int* bad;
    (void)hipMalloc(&clk, 4 * 8);
    (void)hipMalloc(&bad, 4);
    (void)hipMemset(bad, 0, 4);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const char* names[] = {"poll", "poll_sleep1", "sleep_wakeup", "poll64_all"};
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            switch (mode) {
                case 0: hipLaunchKernelGGL(k_pingpong<0>, dim3(1), dim3(128), 0, 0, clk, bad); break;
                case 1: hipLaunchKernelGGL(k_pingpong<1>, dim3(1), dim3(128), 0, 0, clk, bad); break;
                case 2: hipLaunchKernelGGL(k_pingpong<2>, dim3(1), dim3(128), 0, 0, clk, bad); break;
                default: hipLaunchKernelGGL(k_pingpong<3>, dim3(1), dim3(128), 0, 0, clk, bad); break;
            }
        }
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        long long h[4];
        int hb = 0;
        (void)hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
        printf("{\"form\": \"%s\", \"clk_per_handoff\": %.1f, \"spins_per_wait\": %.1f, \"bad\": %d}\n", names[mode],
               h[0] / (2.0 * kRounds), h[1] / (double)kRounds, hb);
    }
    return 0;
}
