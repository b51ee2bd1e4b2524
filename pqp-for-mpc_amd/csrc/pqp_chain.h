// pqp_chain.h -- device helpers shared by the two persistent launches
// (pqp_persist.hip: k_split_persist, fixed mode; pqp_converge.hip:
// k_converge_persist, converge mode): the realtime deadline of their waits and
// the products / add chain of one slice of split-matrix packets.  Every
// product and every add is rounded as the reference's (updateY2 /
// matrixMultiply, PQP_CPU.c:88-100, :608-609: q * y rounded, then summed with
// k in order); the read-ahead only changes when the LDS reads are issued.
#pragma once
#include "pqp_device.h"

namespace pqp {
namespace {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int kSliceLanes = 32;                   // row sides (output columns) per workgroup: packet row stride
constexpr long long kTimeoutTicks = 200000000LL;  // s_memrealtime runs at 100 MHz: 2 s

__device__ __forceinline__ u64 rt_now() { return __builtin_amdgcn_s_memrealtime(); }

// A wait's time limit, started at its first check.
struct Deadline {
    u64 t0 = 0;
    __device__ __forceinline__ bool expired() {
        const u64 now = rt_now();
        if (t0 == 0) {
            t0 = now;
            return false;
        }
        return (long long)(now - t0) > kTimeoutTicks;
    }
};

// Wave 0's slice with its q already in registers (read while it waited for
// y): one LDS read (y) per packet, D packets ahead, each packet's products
// added as soon as they are formed, so the chain starts with the first packet
// instead of after the whole slice.
template <int NP>
__device__ __forceinline__ float chain_qreg(float acc, const f4v (&q)[NP], const f4v* yw) {
    constexpr int D = NP < 12 ? NP : 12;
    f4v yr[D + 1];
#pragma unroll
    for (int j = 0; j < D; ++j) yr[j] = yw[j];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        if (j + D < NP) yr[(j + D) % (D + 1)] = yw[j + D];
        const f4v y = yr[j % (D + 1)];
        const f2v lo = f2v{q[j].x, q[j].y} * f2v{y.x, y.y};
        const f2v hi = f2v{q[j].z, q[j].w} * f2v{y.z, y.w};
        acc += lo.x;  // matrixMultiply :88-100 / updateY2 :608-609, k in order
        acc += lo.y;
        acc += hi.x;
        acc += hi.y;
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}

// prod[j] = prod[j] * y[j] with the slice's q already in prod (read ahead,
// while the wave waited for y): only y is read, D packets ahead.
template <int NP>
__device__ __forceinline__ void slice_products_inplace(f4v (&prod)[NP], const f4v* yw) {
    constexpr int D = NP < 6 ? NP : 6;
    f4v yr[D + 1];
#pragma unroll
    for (int j = 0; j < D; ++j) yr[j] = yw[j];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        if (j + D < NP) yr[(j + D) % (D + 1)] = yw[j + D];
        const f4v q = prod[j], y = yr[j % (D + 1)];
        const f2v lo = f2v{q.x, q.y} * f2v{y.x, y.y};
        const f2v hi = f2v{q.z, q.w} * f2v{y.z, y.w};
        prod[j] = f4v{lo.x, lo.y, hi.x, hi.y};
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Products of one slice, prod[j] = q[j] * y[j] (each product rounded as the
// reference's q * y), with the reads of packet j + D issued before packet j
// is multiplied (q straight into prod[j + D], y into a ring of D + 1): the
// LDS latency is paid about once per slice instead of once per packet (the
// compiler's own schedule kept two packets in flight, ~48 clocks each).
template <int NP>
__device__ __forceinline__ void slice_products(f4v (&prod)[NP], const f4v* qw, const f4v* yw) {
    constexpr int D = NP < 6 ? NP : 6;
    f4v yr[D + 1];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        prod[j] = qw[j * kSliceLanes];
        yr[j] = yw[j];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        if (j + D < NP) {
            prod[j + D] = qw[(j + D) * kSliceLanes];
            yr[(j + D) % (D + 1)] = yw[j + D];
        }
        const f4v q = prod[j], y = yr[j % (D + 1)];
        const f2v lo = f2v{q.x, q.y} * f2v{y.x, y.y};
        const f2v hi = f2v{q.z, q.w} * f2v{y.z, y.w};
        prod[j] = f4v{lo.x, lo.y, hi.x, hi.y};
        __builtin_amdgcn_sched_barrier(0);  // keep the reads D packets ahead of their use
    }
}

}  // namespace
}  // namespace pqp
