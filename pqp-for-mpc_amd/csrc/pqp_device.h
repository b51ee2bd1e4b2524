// pqp_device.h -- device-side arithmetic shared by every PQP kernel (gfx950).
//
// Float rules: the whole library is compiled with
// -ffp-contract=off, so `a * b + c` is a rounded product followed by a rounded
// add, exactly like PQP_CPU.c built without FMA.  Division uses the default
// correctly rounded fp32 divide (never __fdividef / fast-math).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace pqp {

// The reference's max(): `a > b ? a : b` on floats (PQP_CPU.c:32-36).  Not
// fmaxf: max(0,-0.0f) is -0.0f and a NaN second operand propagates.
__host__ __device__ __forceinline__ float max_ref(float a, float b) { return (a > b) ? a : b; }

// Tolerances erc = eac = eaj = erj (PQP_CPU.c:19-22).
constexpr double kTol = 1e-6;

// terminate()'s gap tests (PQP_CPU.c:683-685) in the reference's own order,
// each returning early: the double division (about ten dependent f64
// operations) only once the first two tests pass -- Jp > -Jd alone decides
// almost every iterate short of the stop.  True: terminate() returns 1.
__host__ __device__ __forceinline__ bool gap_stop(float Jp, float Jd) {
    if (Jp > -Jd) return false;
    const double gap = (double)(Jp + Jd);
    if (gap > kTol) return false;
    return !(gap / fabs((double)Jd) > kTol);
}

// ---------------------------------------------------------------------------
// Relay hand-off wait (k_split_relay, k_lean_relay, k_gemv_relay): spin until
// every lane's 64-bit LDS word {sequence, bits(running sum)} carries sequence
// g.  Bounded, so a broken hand-off cannot hang the GPU; an expired wait sets
// `stale` (a register), and the kernel ORs it into the caller's sticky error
// word once, at exit -- the host turns that into PQP_ERR_HIP instead of
// returning wrong sums.  spin_max < 0 expires every wait (tests of the error
// path only); the default budget is kRelaySpinMax (pqp_launch.h).
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long relay_wait(unsigned long long* slot, int lane, int g, int spin_max,
                                                         bool& stale) {
    // the loop keeps the one-compare exit of a plain bounded spin (a second
    // exit branch per poll measured 6-9 % slower on chain-bound blocks); the
    // expiry is derived from the counter after the loop
    unsigned long long h;
    int spin = 0;
    for (;; ++spin) {
        h = __hip_atomic_load(slot + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__all((int)(h >> 32) == g) || spin > spin_max) break;
    }
    stale |= spin > spin_max;
    return h;
}
// once per wave, at kernel exit (vector atomic; no store in the wait loop)
__device__ __forceinline__ void relay_report(bool stale, int* err, int lane) {
    if (stale && err && lane == 0) atomicOr(err, 1);
}

// ---------------------------------------------------------------------------
// Counter-based synthetic generator.  MUST stay identical to
// oracle/pqp_oracle.c (orc_hash32 / orc_synth_key / orc_synth_bits / orc_u01).
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__host__ __device__ __forceinline__ uint32_t synth_key(uint32_t seed, uint32_t inst, uint32_t tag) {
    uint32_t k = hash32(seed * 0x9E3779B9U + 0x632BE5ABU);
    k = hash32(k ^ (inst * 0x85EBCA6BU + 0x27D4EB2FU));
    return hash32(k + tag * 0xC2B2AE35U);
}
__host__ __device__ __forceinline__ uint32_t synth_bits(uint32_t key, uint32_t idx) {
    return hash32(key ^ hash32(idx + 0x165667B1U));
}
__host__ __device__ __forceinline__ float u01(uint32_t bits) {
    return (float)(bits >> 8) * (1.0f / 16777216.0f);
}
enum SynthTag : uint32_t { kTagQinv = 1, kTagGp = 2, kTagKp = 3, kTagFp = 4 };

struct SynthKeys {
    uint32_t q, g, k, f;
};
__host__ __device__ __forceinline__ SynthKeys synth_keys(uint32_t seed, uint32_t inst) {
    return SynthKeys{synth_key(seed, inst, kTagQinv), synth_key(seed, inst, kTagGp),
                     synth_key(seed, inst, kTagKp), synth_key(seed, inst, kTagFp)};
}
// Qp_inv diagonal entry q_j = 0.1 + u
__host__ __device__ __forceinline__ float synth_qinv(const SynthKeys& K, int j) {
    return 0.1f + u01(synth_bits(K.q, (uint32_t)j));
}
// Gp[i][j] in {-1, 0, +1}
__host__ __device__ __forceinline__ float synth_gp(const SynthKeys& K, int i, int j, int M) {
    uint32_t idx = (uint32_t)i * (uint32_t)M + (uint32_t)j;
    return (float)((int)(synth_bits(K.g, idx) % 3U) - 1);
}
__host__ __device__ __forceinline__ float synth_kp(const SynthKeys& K, int i) {
    return 10.0f * u01(synth_bits(K.k, (uint32_t)i));
}
__host__ __device__ __forceinline__ float synth_fp(const SynthKeys& K, int j) {
    float s = 20.0f * u01(synth_bits(K.f, (uint32_t)j));
    return s - 10.0f;
}

}  // namespace pqp
