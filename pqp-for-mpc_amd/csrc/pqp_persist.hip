// pqp_persist.hip -- fixed-iteration mode of ONE problem of n_dual <= 1024
// (BASELINE configs[2]) as ONE persistent launch: every update of the solve
// runs inside the kernel, the split matrices stay in LDS for the whole solve,
// and the iterate moves between workgroups through tagged 8-byte granules in
// global memory instead of through a kernel boundary per update.
//
// What one update is (PQP_CPU.c:603-618, updateY2 over the stored split
// matrices Qdn_theta / Qdp_theta, :524-537):
//   acc_p = sum_{k=0..N-1} S_p[k] * y[k]  (sequential, from +0.0f)
//   num_i = acc_{2i} + 1.0f * Fdn_i ; den_i = acc_{2i+1} + 1.0f * Fdp_i
//   y_next[i] = num_i / den_i * y[i]                             (updY :594)
// with lane p = 2i + side owning row side p (the k_split_relay layout, 32
// row sides per workgroup).  Only the adds form the sequential chain; the
// products are rounded one by one exactly as in the reference (q * y, no FMA).
//
// Geometry: workgroup b owns row sides [32b, 32b + 32) = rows [16b, 16b + 16);
// its W waves split the k range into slices of PW packets (4 PW values of k).
// Per update:
//   1. wave w fetches y[k] of its slice: the initial iterate from Y0, later
//      the granules {tag = update, bits(y)} published by the producing
//      workgroups (agent-scope relaxed 8-byte loads, `global_load_dwordx2 sc1`,
//      repeated until every tag matches -- the data is its own flag);
//   2. forms its slice's products q * y in registers (q from LDS);
//   3. waits for wave w-1's running sums (one 64-bit LDS word per lane:
//      tag and sum), adds its products in k order, hands the sums on;
//   4. the last wave adds Fdn/Fdp, divides, multiplies by y_i and publishes
//      y_next[i] as a granule (`global_store_dwordx2 sc1`); the last update
//      also writes Yout.
// Granules, LDS hand-off words and y slices are double-buffered by update
// parity; the tags make every wait exact (see the hazard notes in
// k_split_persist).  Every wait is bounded in time: a workgroup that never
// gets a slot ends the launch with an error word instead of a hang.
//
// Requirement: all G = ceil(2N / 32) workgroups resident at once (one per CU
// by their LDS; G <= 64 of the 256 CUs).
#include "pqp_device.h"
#include "pqp_launch.h"

namespace pqp {

namespace {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int kPLanes = 32;  // row sides per workgroup
constexpr int kPW = 48;      // packets (4 values of k) per wave: the products live in 4 * kPW VGPRs
constexpr int kPMaxWaves = 6;
constexpr long long kPTimeoutTicks = 200000000LL;  // s_memrealtime runs at 100 MHz: 2 s

__device__ __forceinline__ u64 rt_now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void fail(int* err, int code) {
    __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

int g_persist_off = 0;

int persist_waves(int N) { return (split_kblocks(N) + kPW - 1) / kPW; }
int persist_max_n() { return 4 * kPW * kPMaxWaves > 1024 ? 1024 : 4 * kPW * kPMaxWaves; }
// LDS: the workgroup's packets zero-padded to W * kPW (so every wave runs the
// same unguarded loops: a +0 packet times y = +0 adds exactly nothing to a sum
// that is never -0), two y slices per wave, two hand-off words per lane and wave
size_t persist_lds_bytes(int N) {
    const int W = persist_waves(N);
    return sizeof(float) * ((size_t)W * kPW * kPLanes * 4 + (size_t)2 * W * kPW * 4) + sizeof(u64) * 2 * W * 64;
}

// SP: the k_build_split layout with lw = 32 (workgroup-major packets).
// gran: 2 * N granules, zeroed before the launch.  err: zeroed before the launch.
__global__ void __launch_bounds__(64 * kPMaxWaves, 1)
    k_split_persist(const float* __restrict__ SP, const float* __restrict__ fdpn, int N, int updates,
                    const float* __restrict__ Y0, float* __restrict__ Yout, u64* gran_, int* err) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    gu64* gran = (gu64*)gran_;
    const int KB = split_kblocks(N);
    const int W = (KB + kPW - 1) / kPW;
    const int KP = W * kPW;                       // packets incl. the zero padding
    f4v* qs = reinterpret_cast<f4v*>(lds);        // [KP][32] packets of this workgroup
    float* ysb = lds + (size_t)KP * kPLanes * 4;  // [2][W * 4 kPW] y slices by update parity
    u64* slot = reinterpret_cast<u64*>(ysb + 2 * W * kPW * 4);  // [2][W][64] hand-off words
    const int ny = W * kPW * 4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ll = lane & (kPLanes - 1);  // lanes 32..63 repeat lanes 0..31 (discarded)
    const int p = blockIdx.x * kPLanes + ll;
    const bool live = lane < kPLanes && p < 2 * N;
    const int row = p >> 1;

    // this workgroup's packets -> LDS (read-only input: plain loads)
    {
        const f4v* src = reinterpret_cast<const f4v*>(SP) + (size_t)blockIdx.x * KB * kPLanes;
        for (int e = tid; e < KP * kPLanes; e += blockDim.x)
            qs[e] = (e < KB * kPLanes) ? src[e] : f4v{0.0f, 0.0f, 0.0f, 0.0f};
        for (int e = tid; e < 2 * W * 64; e += blockDim.x) slot[e] = 0ull;
    }
    const float fd = live ? fdpn[p] : 0.0f;
    __syncthreads();

    const int pk0 = w * kPW;                                   // first packet of this wave's slice
    const int k0 = 4 * pk0, k1 = (4 * (pk0 + kPW)) < N ? 4 * (pk0 + kPW) : N;  // y[k0, k1) of the slice
    const bool last = (w == W - 1);
    for (int u = 0; u < updates; ++u) {
        const int par = u & 1;
        float* ys = ysb + par * ny;
        // ---- 1. y of this slice (k in [k0, k1)), staged in LDS ----
        if (u == 0) {
            for (int k = k0 + lane; k < k1; k += 64) ys[k] = Y0 ? Y0[k] : 1000.0f;  // initMat(Y, 1000) :710
        } else {
            const gu64* g = gran + (size_t)par * N;
            const unsigned tag = (unsigned)u;
            for (int kb = k0; kb < k1; kb += 256) {  // up to 4 granules per lane per sweep
                float v[4];
                const u64 t0 = rt_now();
                for (unsigned spins = 0;; ++spins) {
                    bool ok = true;
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const int k = kb + 64 * m + lane;
                        if (k < k1) {
                            const u64 x = __hip_atomic_load(g + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            v[m] = __uint_as_float((unsigned)x);
                            ok &= (unsigned)(x >> 32) == tag;
                        }
                    }
                    if (__all(ok)) break;
                    if ((spins & 63) == 63 && (long long)(rt_now() - t0) > kPTimeoutTicks) {
                        fail(err, 1);
                        return;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int k = kb + 64 * m + lane;
                    if (k < k1) ys[k] = v[m];
                }
            }
        }
        // zero y past N up to the slice end (read by the last packet's products)
        for (int k = (k1 > k0 ? k1 : k0) + lane; k < 4 * (pk0 + kPW); k += 64) ys[k] = 0.0f;
        // ---- 2. products of the slice, off the add chain ----
        f4v prod[kPW];
        // one base address per operand, the packet index as an immediate offset
        const f4v* qw = qs + (size_t)pk0 * kPLanes + ll;
        const f4v* yw = reinterpret_cast<const f4v*>(ys) + pk0;
#pragma unroll
        for (int j0 = 0; j0 < kPW; j0 += 4) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int j = j0 + jj;
                const f4v q = qw[j * kPLanes];
                const f4v y = yw[j];
                const f2v lo = f2v{q.x, q.y} * f2v{y.x, y.y};
                const f2v hi = f2v{q.z, q.w} * f2v{y.z, y.w};
                prod[j] = f4v{lo.x, lo.y, hi.x, hi.y};
            }
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) asm volatile("" : "+v"(prod[j0 + jj]));
        }
        // ---- 3. the running sums of the previous slice, then this slice's adds ----
        float acc = 0.0f;
        u64* sl = slot + (size_t)par * W * 64;
        const unsigned want = (unsigned)(u + 1);
        if (w > 0) {
            const u64 t0 = rt_now();
            u64 h;
            for (unsigned spins = 0;; ++spins) {
                h = __hip_atomic_load(sl + (w - 1) * 64 + lane, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (__all((unsigned)(h >> 32) == want)) break;
                if ((spins & 255) == 255 && (long long)(rt_now() - t0) > kPTimeoutTicks) {
                    fail(err, 2);
                    return;
                }
            }
            acc = __uint_as_float((unsigned)h);
        }
        __builtin_amdgcn_s_setprio(3);
#pragma unroll
        for (int j = 0; j < kPW; ++j) {
            acc += prod[j].x;  // :608-609, k in order
            acc += prod[j].y;
            acc += prod[j].z;
            acc += prod[j].w;
        }
        if (!last) {
            __hip_atomic_store(sl + w * 64 + lane, ((u64)want << 32) | __float_as_uint(acc), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
            __builtin_amdgcn_s_setprio(0);
            continue;
        }
        __builtin_amdgcn_s_setprio(0);
        // ---- 4. the last slice's wave finishes the rows ----
        const float v = acc + 1.0f * fd;     // even lane: num (:611), odd lane: den (:612)
        const float den = __shfl_xor(v, 1);  // whole wave active
        if (!(p & 1) && live) {
            const float yn = v / den * ys[row];  // :594; ys[row] was staged by its slice's wave (hand-off order)
            __hip_atomic_store(gran + (size_t)(par ^ 1) * N + row, ((u64)want << 32) | __float_as_uint(yn),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (u == updates - 1) Yout[row] = yn;
        }
    }
}

hipError_t launch_split_persist(const float* SP, const float* fdpn, int N, int updates, const float* Y0, float* Yout,
                                unsigned long long* gran, int* err, hipStream_t s) {
    if (updates <= 0) return hipSuccess;
    const int W = persist_waves(N);
    const int G = (2 * N + kPLanes - 1) / kPLanes;
    hipError_t e = hipMemsetAsync(gran, 0, sizeof(u64) * 2 * N, s);
    if (e == hipSuccess) e = hipMemsetAsync(err, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_split_persist, dim3(G), dim3(64 * W), persist_lds_bytes(N), s, SP, fdpn, N, updates, Y0,
                       Yout, gran, err);
    return hipGetLastError();
}

}  // namespace pqp
