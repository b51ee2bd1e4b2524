// Probe: clocks per packet (4 terms q * y, 32 row sides) of the product
// formation in k_split_persist's slices, by where q and y come from:
//   0 lds_q_lds_y: q b128 per lane (distinct) + y b128 (one address, broadcast) + 2 v_pk_mul
//   1 reg_q_lds_y: q held in VGPRs, y b128 broadcast from LDS
//   2 lds_q_sgpr_y: q b128 from LDS, y as an SGPR pair operand of v_pk_mul
//   3 reg_q_sgpr_y: no LDS reads
//   4 lds_q_lds_y_half: as 0, lanes 32..63 inactive
// 48 packets per wave, one workgroup of 1 or 6 waves all forming products at once.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off products_probe.hip -o products_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int NP = 48;

template <int MODE>
__global__ void __launch_bounds__(384) k_products(const float* __restrict__ in, float* out, long long* clk, float ys0,
                                                  float ys1) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    f4v* qs = reinterpret_cast<f4v*>(lds);               // [NP][32]
    f4v* yv = reinterpret_cast<f4v*>(lds) + NP * 32;     // [NP]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, ll = lane & 31;
    for (int e = threadIdx.x; e < NP * 32 + NP; e += blockDim.x) {
        const int i = e * 4;
        qs[e] = f4v{in[i & 4095], in[(i + 1) & 4095], in[(i + 2) & 4095], in[(i + 3) & 4095]};
    }
    f4v qr[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) qr[j] = f4v{in[(j * 64 + lane) & 4095], 1.0f, 2.0f, in[(j * 7 + lane) & 4095]};
#pragma unroll
    for (int j = 0; j < NP; ++j) asm volatile("" : "+v"(qr[j]));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const f4v* qw = qs + ll;
    f4v prod[NP];
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 4 && lane >= 32) {
    } else {
        constexpr int D = 6;
        f4v ringq[D + 1], ringy[D + 1];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if (MODE == 0 || MODE == 2 || MODE == 4) ringq[j] = qw[j * 32];
            if (MODE == 0 || MODE == 1 || MODE == 4) ringy[j] = yv[j];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            if (j + D < NP) {
                if (MODE == 0 || MODE == 2 || MODE == 4) ringq[(j + D) % (D + 1)] = qw[(j + D) * 32];
                if (MODE == 0 || MODE == 1 || MODE == 4) ringy[(j + D) % (D + 1)] = yv[j + D];
            }
            const f4v q = (MODE == 1 || MODE == 3) ? qr[j] : ringq[j % (D + 1)];
            const f4v y = (MODE == 2 || MODE == 3) ? f4v{ys0, ys1, ys0, ys1} : ringy[j % (D + 1)];
            const f2v lo = f2v{q.x, q.y} * f2v{y.x, y.y};
            const f2v hi = f2v{q.z, q.w} * f2v{y.z, y.w};
            prod[j] = f4v{lo.x, lo.y, hi.x, hi.y};
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) asm volatile("" : "+v"(prod[j]));
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < NP; ++j) s += prod[j].x + prod[j].y + prod[j].z + prod[j].w;
    out[threadIdx.x] = s;
    if (lane == 0) clk[w] = t1 - t0;
}

template <int MODE>
static void run(const char* name, const float* in, float* out, long long* clk, int waves) {
    long long h[6] = {};
    for (int rep = 0; rep < 3; ++rep)
        hipLaunchKernelGGL(k_products<MODE>, dim3(1), dim3(64 * waves), (NP * 32 + NP) * 16, 0, in, out, clk, 1.5f,
                           2.5f);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, clk, sizeof(long long) * waves, hipMemcpyDeviceToHost);
    printf("{\"form\": \"%s\", \"waves\": %d, \"clk_per_packet\": [", name, waves);
    for (int w = 0; w < waves; ++w) printf("%s%.1f", w ? ", " : "", h[w] / (double)NP);
    printf("]}\n");
}

int main() {
    float *in, *out;
    long long* clk;
    (void)hipMalloc(&in, 4096 * 4);
    (void)hipMalloc(&out, 384 * 4);
    (void)hipMalloc(&clk, 6 * 8);
    float h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = 1.0f + (i % 97) * 0.01f;
    (void)hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    for (int waves : {1, 6}) {
        run<0>("lds_q_lds_y", in, out, clk, waves);
        run<1>("reg_q_lds_y", in, out, clk, waves);
        run<2>("lds_q_sgpr_y", in, out, clk, waves);
        run<3>("reg_q_sgpr_y", in, out, clk, waves);
        run<4>("lds_q_lds_y_half", in, out, clk, waves);
    }
    return 0;
}
