#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float sf2 __attribute__((ext_vector_type(2)));
typedef float sf4 __attribute__((ext_vector_type(4)));

// V: 0 scalar add chain over LDS values; 1 mul+add chain (dot); 2 pk_mul+pk_add chain (pairs);
//    3 max,max,pk_mul,pk_add (row, no diag); 4 like 3 with diag select; 5 register-only add chain
//    6: two interleaved rows of V3 per lane; 12-15: lane pairs (one side of a row per lane,
//    v_med3_f32 against +-inf gives max(q,0) / min(q,0), odd lanes multiply by -y): plain,
//    with the fused Y'Qd term, two rows per lane, with the diagonal select
template <int V>
__global__ void __launch_bounds__(1024) mb(const float* g, float* out, unsigned long long* cyc, int n, int reps) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x;
    const int ld = n + 4;
    for (int e = tid; e < 64 * ld + 2 * (n + 8); e += blockDim.x) lds[e] = g[e % 1000] * 1e-3f;
    __syncthreads();
    const float* row = lds + (tid & 63) * ld;
    const float* y = lds + 64 * ld;
    // V >= 12 (lane pairs): odd lanes read the negated copy of y
    const float* ys = (V >= 12 && (tid & 1)) ? y + n + 8 : y;
    const float lim = (tid & 1) ? -__builtin_inff() : __builtin_inff();
    float s2 = 0.0f;
    float s = 0.0f;
    sf2 acc = {0.0f, 0.0f}, acc2 = {0.f, 0.f};
    const int i = tid & 63;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        for (int k = 0; k < n; k += 8) {
            const sf4 q0 = *reinterpret_cast<const sf4*>(row + k), q1 = *reinterpret_cast<const sf4*>(row + k + 4);
            const sf4 y0 = *reinterpret_cast<const sf4*>(ys + k), y1 = *reinterpret_cast<const sf4*>(ys + k + 4);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float q = j < 4 ? q0[j] : q1[j - 4];
                const float yk = j < 4 ? y0[j] : y1[j - 4];
                if constexpr (V == 0) s += q;
                else if constexpr (V == 1) s += q * yk;
                else if constexpr (V == 2) acc += sf2{q, yk} * sf2{yk, yk};
                else if constexpr (V == 3 || V == 4 || V == 6) {
                    float qp, qn;
                    asm("v_max_f32 %0, %1, 0" : "=v"(qp) : "v"(q));
                    asm("v_max_f32_e64 %0, -%1, 0" : "=v"(qn) : "v"(q));
                    if constexpr (V == 4) {
                        const bool d = (k + j == i);
                        qp = d ? 3.0f : qp;
                        qn = d ? 2.0f : qn;
                    }
                    acc += sf2{qp, qn} * sf2{yk, yk};
                    if constexpr (V == 6) acc2 += sf2{qn, qp} * sf2{yk, yk};
                }
                else if constexpr (V == 5) s += yk;
                else if constexpr (V == 7 || V == 8) {
                    float qp, qn;
                    asm("v_max_f32 %0, %1, 0" : "=v"(qp) : "v"(q));
                    asm("v_max_f32_e64 %0, -%1, 0" : "=v"(qn) : "v"(q));
                    if constexpr (V == 8) {
                        const bool d = (k + j == i);
                        qp = d ? 3.0f : qp;
                        qn = d ? 2.0f : qn;
                    }
                    const float tp = qp * yk, tn = qn * yk;
                    asm volatile("" :: "v"(tp), "v"(tn));
                    acc.x += tp;
                    acc.y += tn;
                }
                else if constexpr (V == 9) {  // split storage: (qp, qn) = (q, yk-ish) pairs
                    const float tp = q * yk, tn = yk * yk;
                    acc.x += tp;
                    acc.y += tn;
                }
                else if constexpr (V == 10) {  // t = q*y; max forms after the product
                    const float t = q * yk;
                    float tp, tn;
                    asm("v_max_f32 %0, %1, 0" : "=v"(tp) : "v"(t));
                    asm("v_max_f32_e64 %0, -%1, 0" : "=v"(tn) : "v"(t));
                    acc.x += tp;
                    acc.y += tn;
                }
                else if constexpr (V >= 12 && V <= 15) {  // lane pairs: one side per lane, med3 split
                    float t;
                    asm("v_med3_f32 %0, %1, 0, %2" : "=v"(t) : "v"(q), "v"(lim));
                    if constexpr (V == 15) t = (k + j == i) ? 3.0f : t;
                    s += t * yk;
                    if constexpr (V == 13) s2 += yk * q;
                    if constexpr (V == 14) {
                        float t2;
                        asm("v_med3_f32 %0, %1, 0, %2" : "=v"(t2) : "v"(-q), "v"(lim));
                        s2 += t2 * yk;
                    }
                }
                else if constexpr (V == 11) {  // row scalar + fused aq chain
                    float qp, qn;
                    asm("v_max_f32 %0, %1, 0" : "=v"(qp) : "v"(q));
                    asm("v_max_f32_e64 %0, -%1, 0" : "=v"(qn) : "v"(q));
                    const float tp = qp * yk, tn = qn * yk;
                    asm volatile("" :: "v"(tp), "v"(tn));
                    acc.x += tp;
                    acc.y += tn;
                    s += yk * q;
                }
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + tid] = s + s2 + acc.x + acc.y + acc2.x + acc2.y;
    if ((tid & 63) == 0) cyc[blockIdx.x * 16 + (tid >> 6)] = t1 - t0;
}

template <int V>
void run(const float* g, float* out, unsigned long long* cyc, int n, int threads, const char* name) {
    const int reps = 50;
    size_t lds = sizeof(float) * (64 * (n + 4) + 2 * (n + 8));
    hipLaunchKernelGGL(mb<V>, dim3(1), dim3(threads), lds, 0, g, out, cyc, n, reps);
    hipLaunchKernelGGL(mb<V>, dim3(1), dim3(threads), lds, 0, g, out, cyc, n, reps);
    hipDeviceSynchronize();
    unsigned long long h[16];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    const int w = threads / 64;
    double mx = 0, mn = 1e30;
    for (int i = 0; i < w; ++i) { mx = h[i] > mx ? h[i] : mx; mn = h[i] < mn ? h[i] : mn; }
    printf("%-28s threads %4d: %.1f cycles per k (slowest wave), %.1f (fastest)\n", name, threads,
           mx / (reps * (double)n), mn / (reps * (double)n));
}

int main() {
    float *g, *out;
    unsigned long long* cyc;
    hipMalloc(&g, 4000 * 4);
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cyc, 1024);
    std::vector<float> hg(4000);
    for (int i = 0; i < 4000; ++i) hg[i] = (float)((i * 7919) % 1000) - 500.0f;
    hipMemcpy(g, hg.data(), 16000, hipMemcpyHostToDevice);
    const int n = 144;
    for (int t : {64, 256, 512, 1024}) {
        run<5>(g, out, cyc, n, t, "reg add chain (y bcast)");
        run<0>(g, out, cyc, n, t, "add chain (row ld)");
        run<1>(g, out, cyc, n, t, "mul+add chain");
        run<2>(g, out, cyc, n, t, "pk_mul+pk_add chain");
        run<3>(g, out, cyc, n, t, "row: max,max,pk_mul,pk_add");
        run<4>(g, out, cyc, n, t, "row + diag select");
        run<6>(g, out, cyc, n, t, "two rows interleaved");
        run<7>(g, out, cyc, n, t, "row scalar");
        run<8>(g, out, cyc, n, t, "row scalar + diag");
        run<9>(g, out, cyc, n, t, "split pairs scalar");
        run<10>(g, out, cyc, n, t, "product then max");
        run<11>(g, out, cyc, n, t, "row scalar + fused aq");
        run<12>(g, out, cyc, n, t, "lane pair med3");
        run<13>(g, out, cyc, n, t, "lane pair med3 + fused aq");
        run<14>(g, out, cyc, n, t, "lane pair med3, 2 rows");
        run<15>(g, out, cyc, n, t, "lane pair med3 + diag");
    }
    return 0;
}
