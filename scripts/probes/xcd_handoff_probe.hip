// Probe: one-way latency of an 8-byte {tag, value} granule between two
// workgroups, by store flavour and by placement (same XCD: blocks 0 and 8;
// other XCD: blocks 0 and 1 under the observed round-robin placement, each
// block's XCC id read and reported).  The question it answers: does keeping
// configs[2]'s y exchange inside one XCD's L2 (plain or sc0 stores, which keep
// the line in L2, read back with sc1 loads, which bypass only L1) beat the
// agent-coherent sc1 / sc1 granules k_split_persist uses (sc1 stores drop the
// line from L2, so even a same-XCD reader goes to the fabric)?
// One lane per block ping-pongs kReps times; s_memtime (shader clock) and
// s_memrealtime (100 MHz) around the loop; every wait is bounded by a spin
// count, and a wait that ran out is counted (a flavour whose store is never
// seen by the reader reports failures instead of hanging).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 xcd_handoff_probe.hip -o xcd_handoff_probe
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

typedef unsigned long long u64;
constexpr int kReps = 4000;
constexpr unsigned kSpins = 1u << 16;  // ~65 ms per wait at ~1 us per poll

template <int SK>
__device__ __forceinline__ void put(u64* p, u64 v) {
    if constexpr (SK == 0) asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SK == 1) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SK == 2) asm volatile("global_store_dwordx2 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ u64 get(const u64* p) {
    u64 v;
    asm volatile("global_load_dwordx2 %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// true when the wanted tag arrived within the spin bound
__device__ __forceinline__ bool wait_tag(const u64* p, unsigned want) {
    for (unsigned s = 0; s < kSpins; ++s)
        if ((unsigned)(get(p) >> 32) == want) return true;
    return false;
}

template <int SK>
__global__ void __launch_bounds__(64) k_pp(u64* slots, int peer, u64* out) {
    const int b = blockIdx.x;
    if ((b != 0 && b != peer) || threadIdx.x != 0) return;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    u64* mine = slots + (b == 0 ? 0 : 16);  // 128-byte lines of their own
    u64* theirs = slots + (b == 0 ? 16 : 0);
    unsigned miss = 0;
    const u64 t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < kReps; ++r) {
        const unsigned a = 2 * r + 1, c = 2 * r + 2;
        if (b == 0) {
            put<SK>(mine, ((u64)a << 32) | (unsigned)r);
            if (!wait_tag(theirs, c)) { ++miss; break; }  // the first expired wait ends this side
        } else {
            if (!wait_tag(theirs, a)) { ++miss; break; }
            put<SK>(mine, ((u64)c << 32) | (unsigned)r);
        }
    }
    const u64 t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    u64* o = out + (b == 0 ? 0 : 4);
    o[0] = t1 - t0;
    o[1] = r1 - r0;
    o[2] = xcc & 0xf;
    o[3] = miss;
}

template <int SK>
void run(const char* name, int peer, u64* slots, u64* out, bool comma) {
    u64 h[8];
    for (int rep = 0; rep < 2; ++rep) {  // the first launch warms up
        CK(hipMemset(slots, 0, 256));
        CK(hipMemset(out, 0, 64));
        hipLaunchKernelGGL(k_pp<SK>, dim3(16), dim3(64), 0, 0, slots, peer, out);
        CK(hipDeviceSynchronize());
    }
    CK(hipMemcpy(h, out, 64, hipMemcpyDeviceToHost));
    // one way = a round trip / 2
    printf("%s{\"store\": \"%s\", \"peer\": %d, \"xcc\": [%llu, %llu], \"one_way_clk\": %.1f, "
           "\"one_way_ns\": %.1f, \"expired_waits\": [%llu, %llu]}\n",
           comma ? "," : "", name, peer, h[2], h[6], (double)h[0] / (2.0 * kReps), (double)h[1] * 10.0 / (2.0 * kReps),
           h[3], h[7]);
    fflush(stdout);
}

int main() {
    u64 *slots, *out;
    CK(hipMalloc(&slots, 256));
    CK(hipMalloc(&out, 64));
    printf("[\n");
    bool c = false;
    for (int peer : {8, 1}) {
        run<0>("sc1", peer, slots, out, c), c = true;
        run<1>("plain", peer, slots, out, c);
        run<2>("sc0", peer, slots, out, c);
        run<3>("sc0 sc1", peer, slots, out, c);
    }
    printf("]\n");
    return 0;
}
