// Probe: forms of the bundled example's fixed-iteration solve (configs[1]:
// N = 28, 999 updates of updateY2, PQP_CPU.c:603-618, no terminate) on ONE
// wave.  Each form is checked bit for bit against the reference's Y after 999
// updates (tests/golden/bundled.npz: Y_fixed999) and timed in shader clocks
// (s_memtime around the update loop) and with HIP events.
//   0 rl      the library's k_fixed_tiny<28, RL>: y_k on lane 2k, 28 v_readlane
//             broadcasts feeding packed products, then the 28-add chain
//   1 rl_u2   the same, two updates per loop trip on a 32-bit counter
//   2 hyb     y_0..y_{R-1} by v_readlane, the rest by one ds_write and
//             ds_read_b128 broadcasts (issued first, landing under the chain)
//   3 sparse  each lane's nonzero split entries only, in k order (the skipped
//             entries are +-0: with every y finite they add exactly nothing to a
//             sum that is never -0), y gathered by ds_bpermute; a finiteness
//             ballot per update (a real solver would fall back to the dense form)
// Input: a binary file written by bundled_probe_data.py (N, Qd, Fd, Y_fixed999).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off bundled_probe.hip -o bundled_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#pragma clang fp contract(off)

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NMAX = 28;
constexpr int PMAX = 4;  // nonzero split entries per lane in the sparse form
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float max_ref(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float rdl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }

template <int V, int R>
__global__ void __launch_bounds__(64) k_fx(const float* __restrict__ Qd, const float* __restrict__ Fd, int N, int nup,
                                           float* __restrict__ Y, long long* __restrict__ clk) {
    __shared__ __attribute__((aligned(16))) float ybuf[32];
    const int lane = threadIdx.x, i = lane >> 1, side = lane & 1;
    const bool row = i < N;
    float mat[NMAX];
#pragma unroll
    for (int k = 0; k < NMAX; ++k) mat[k] = 0.0f;
    float fd_own = 0.0f;
    float th = 0.0f;
    if (row) {
        for (int k = 0; k < N; ++k) th += max_ref(0.0f, -Qd[i * N + k]) * 1.0f;  // :503-519
        th = max_ref(th, 5.0f);
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
            if (k < N) {
                const float q = Qd[i * N + k];
                const float t = (i == k) ? th : 0.0f;
                mat[k] = (side ? max_ref(0.0f, q) : max_ref(0.0f, -q)) + 1.0f * t;  // :524-537
            }
        }
        const float f = Fd[i];
        fd_own = side ? max_ref(0.0f, f) : max_ref(0.0f, -f);
    }
    // sparse form: this lane's nonzero entries in k order, y's source lane 2k
    float sc[PMAX];
    int sa[PMAX];
    int nnz = 0;
#pragma unroll
    for (int s = 0; s < PMAX; ++s) { sc[s] = 0.0f; sa[s] = (row ? 2 * i : 0) * 4; }
    for (int k = 0; k < NMAX; ++k) {
        if (row && mat[k] != 0.0f) {
            if (nnz < PMAX) {
#pragma unroll
                for (int s = 0; s < PMAX; ++s)
                    if (s == nnz) { sc[s] = mat[k]; sa[s] = 2 * k * 4; }
            }
            ++nnz;
        }
    }
    // (a lane with more than PMAX entries would need the dense form: flagged)
    const bool sparse_ok = !__any(nnz > PMAX);
    float yk = (!side && row) ? 1000.0f : 0.0f;  // initMat(Y, 1000) :710
    for (int k = lane; k < 32; k += 64) ybuf[k] = (k < N) ? 1000.0f : 0.0f;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) {
        for (int h = 0; h < nup; ++h) {
            const float yi = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(yk), 0xA0, 0xF, 0xF, true));
            float p[NMAX];
#pragma unroll
            for (int k = 0; k < NMAX; k += 2) {
                const f2v pr = f2v{mat[k], mat[k + 1]} * f2v{rdl(yk, 2 * k), rdl(yk, 2 * k + 2)};
                p[k] = pr.x;
                p[k + 1] = pr.y;
            }
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < NMAX; ++k) acc += p[k];
            const float v = acc + 1.0f * fd_own;
            const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
            const float yn = v / den * yi;
            yk = (!side && row) ? yn : 0.0f;
        }
    } else if constexpr (V == 1) {
        auto step = [&]() {
            const float yi = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(yk), 0xA0, 0xF, 0xF, true));
            float p[NMAX];
#pragma unroll
            for (int k = 0; k < NMAX; k += 2) {
                const f2v pr = f2v{mat[k], mat[k + 1]} * f2v{rdl(yk, 2 * k), rdl(yk, 2 * k + 2)};
                p[k] = pr.x;
                p[k + 1] = pr.y;
            }
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < NMAX; ++k) acc += p[k];
            const float v = acc + 1.0f * fd_own;
            const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
            const float yn = v / den * yi;
            yk = (!side && row) ? yn : 0.0f;
        };
        int h = 0;
        for (; h + 2 <= nup; h += 2) { step(); step(); }
        for (; h < nup; ++h) step();
    } else if constexpr (V == 2) {
        for (int h = 0; h < nup; ++h) {
            // the LDS copy first: its reads land while the readlane part is summed
            if (!side && lane < 64) ybuf[i & 31] = yk;  // lanes >= 2N write +0 pads
            f4v yl[(NMAX - R) / 4];
#pragma unroll
            for (int g = 0; g < (NMAX - R) / 4; ++g) yl[g] = *reinterpret_cast<const f4v*>(ybuf + R + 4 * g);
            const float yi = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(yk), 0xA0, 0xF, 0xF, true));
            float p[NMAX];
#pragma unroll
            for (int k = 0; k < R; k += 2) {
                const f2v pr = f2v{mat[k], mat[k + 1]} * f2v{rdl(yk, 2 * k), rdl(yk, 2 * k + 2)};
                p[k] = pr.x;
                p[k + 1] = pr.y;
            }
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < R; ++k) acc += p[k];
#pragma unroll
            for (int g = 0; g < (NMAX - R) / 4; ++g) {
                const int k = R + 4 * g;
                const f2v lo = f2v{mat[k], mat[k + 1]} * f2v{yl[g].x, yl[g].y};
                const f2v hi = f2v{mat[k + 2], mat[k + 3]} * f2v{yl[g].z, yl[g].w};
                acc += lo.x;
                acc += lo.y;
                acc += hi.x;
                acc += hi.y;
            }
            const float v = acc + 1.0f * fd_own;
            const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
            const float yn = v / den * yi;
            yk = (!side && row) ? yn : 0.0f;
        }
    } else if constexpr (V == 3) {
        if (!sparse_ok) return;
        for (int h = 0; h < nup; ++h) {
            const float yi = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(yk), 0xA0, 0xF, 0xF, true));
            float acc = 0.0f;
#pragma unroll
            for (int s = 0; s < R; ++s)  // R = the batch's largest nnz per lane
                acc += sc[s] * __int_as_float(__builtin_amdgcn_ds_bpermute(sa[s], __float_as_int(yk)));
            const float v = acc + 1.0f * fd_own;
            const float den = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
            const float yn = v / den * yi;
            yk = (!side && row) ? yn : 0.0f;
            // every y must stay finite for the skipped +-0 terms to be exact
            if (__any(!__builtin_isfinite(yk))) break;
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (!side && row) Y[i] = yk;
    if (V == 2 || V == 0 || V == 1 || V == 3) {}
    if (lane == 0) clk[0] = t1 - t0;
}

static std::vector<char> slurp(const char* p) {
    FILE* f = fopen(p, "rb");
    if (!f) { printf("cannot open %s\n", p); exit(1); }
    std::vector<char> b;
    char tmp[65536];
    size_t n;
    while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + n);
    fclose(f);
    return b;
}

int main(int argc, char** argv) {
    const char* path = argc > 1 ? argv[1] : "gpurun_out/bundled.bin";
    const int reps = argc > 2 ? atoi(argv[2]) : 200;
    std::vector<char> b = slurp(path);
    int N;
    memcpy(&N, b.data(), 4);
    const float* Qd = reinterpret_cast<const float*>(b.data() + 4);
    const float* Fd = Qd + N * N;
    const float* Yref = Fd + N;
    float *dQ, *dF, *dY;
    long long* dclk;
    CK(hipMalloc(&dQ, N * N * 4));
    CK(hipMalloc(&dF, N * 4));
    CK(hipMalloc(&dY, 64 * 4));
    CK(hipMalloc(&dclk, 8));
    CK(hipMemcpy(dQ, Qd, N * N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dF, Fd, N * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto kern) {
        std::vector<float> y(N);
        // warm
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, dQ, dF, N, 999, dY, dclk);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(y.data(), dY, N * 4, hipMemcpyDeviceToHost));
        const bool same = memcmp(y.data(), Yref, N * 4) == 0;
        long long clk = 0;
        CK(hipMemcpy(&clk, dclk, 8, hipMemcpyDeviceToHost));
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, dQ, dF, N, 999, dY, dclk);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"form\": \"%s\", \"bit_exact_fixed999\": %s, \"clk_per_update\": %.1f, \"us_per_launch_b2b\": %.2f}\n", name,
               same ? "true" : "false", clk / 999.0, ms * 1e3 / reps);
    };
    run("rl", k_fx<0, 0>);
    run("rl_u2", k_fx<1, 0>);
    run("hyb8", k_fx<2, 8>);
    run("hyb12", k_fx<2, 12>);
    run("hyb16", k_fx<2, 16>);
    run("sparse2", k_fx<3, 2>);
    run("sparse3", k_fx<3, 3>);
    return 0;
}
