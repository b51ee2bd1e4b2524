// read_ceiling: how fast can one MI355X stream 16 GiB out of HBM, by access shape?
// Tuning probe only (not part of libpqp).  The hot kernel (k_batch_iterate) reads each
// problem's 4 MiB of QdT front to back, one workgroup per problem; this compares that
// shape with flat grid-stride and chunked reads, workgroup sizes and load policies.
// Build: hipcc --offload-arch=gfx950 -O3 -o read_ceiling read_ceiling.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <bool NT>
__device__ __forceinline__ float4 ld4(const float4* p) {
    if constexpr (NT) {
        float4 v;
        v.x = __builtin_nontemporal_load(&p->x);
        v.y = __builtin_nontemporal_load(&p->y);
        v.z = __builtin_nontemporal_load(&p->z);
        v.w = __builtin_nontemporal_load(&p->w);
        return v;
    } else {
        return *p;
    }
}

// (a) the hot kernel's shape: workgroup b streams problem b (n4 float4 = 4 MiB), T threads,
// each thread one float4 column slot, U loads in flight.
template <int T, int U, bool NT>
__global__ void __launch_bounds__(T) k_problem(const float4* __restrict__ src, long long n4, float* out) {
    const float4* p = src + (size_t)blockIdx.x * n4 + threadIdx.x;
    float acc = 0.f;
    for (long long i = threadIdx.x; i + (long long)(U - 1) * T < n4; i += (long long)U * T, p += U * T) {
        float4 q[U];
#pragma unroll
        for (int j = 0; j < U; ++j) q[j] = ld4<NT>(p + j * T);
#pragma unroll
        for (int j = 0; j < U; ++j) acc += q[j].x + q[j].y + q[j].z + q[j].w;
    }
    if (acc == 123.f) out[blockIdx.x * T + threadIdx.x] = acc;
}

// (b) flat grid-stride over the whole buffer, G workgroups.
template <int T, int U, bool NT>
__global__ void __launch_bounds__(T) k_flat(const float4* __restrict__ src, long long total4, float* out) {
    const long long stride = (long long)gridDim.x * T;
    float acc = 0.f;
    long long i = (long long)blockIdx.x * T + threadIdx.x;
    for (; i + (U - 1) * stride < total4; i += U * stride) {
        float4 q[U];
#pragma unroll
        for (int j = 0; j < U; ++j) q[j] = ld4<NT>(src + i + j * stride);
#pragma unroll
        for (int j = 0; j < U; ++j) acc += q[j].x + q[j].y + q[j].z + q[j].w;
    }
    if (acc == 123.f) out[blockIdx.x * T + threadIdx.x] = acc;
}

// (c) persistent chunked: G workgroups take contiguous chunks of C float4 round-robin.
template <int T, int U, bool NT>
__global__ void __launch_bounds__(T) k_chunk(const float4* __restrict__ src, long long total4, long long C, float* out) {
    float acc = 0.f;
    for (long long c0 = (long long)blockIdx.x * C; c0 < total4; c0 += (long long)gridDim.x * C) {
        const float4* p = src + c0 + threadIdx.x;
        for (long long i = 0; i + (long long)(U - 1) * T < C; i += (long long)U * T, p += U * T) {
            float4 q[U];
#pragma unroll
            for (int j = 0; j < U; ++j) q[j] = ld4<NT>(p + j * T);
#pragma unroll
            for (int j = 0; j < U; ++j) acc += q[j].x + q[j].y + q[j].z + q[j].w;
        }
    }
    if (acc == 123.f) out[blockIdx.x * T + threadIdx.x] = acc;
}

template <typename F>
static double time_ms(F launch, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a));
        launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float t;
        CHECK(hipEventElapsedTime(&t, a, b));
        ts.push_back(t);
    }
    std::sort(ts.begin(), ts.end());
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ts[ts.size() / 2];
}

int main() {
    const int B = 4096;
    const long long n4 = 1024LL * 1024 / 4;  // float4 per 4 MiB problem
    const long long total4 = n4 * B;
    const double bytes = (double)total4 * 16.0;
    float4* src;
    float* out;
    CHECK(hipMalloc(&src, (size_t)total4 * 16));
    CHECK(hipMalloc(&out, (size_t)B * 1024 * 4));
    CHECK(hipMemset(src, 0, (size_t)total4 * 16));
    CHECK(hipDeviceSynchronize());
    const int reps = 9;
    auto report = [&](const char* name, double ms) {
        printf("%-40s %8.4f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 80.0);
        fflush(stdout);
    };
#define PROB(T, U, NT) \
    report("problem T=" #T " U=" #U " nt=" #NT, \
           time_ms([&] { hipLaunchKernelGGL((k_problem<T, U, NT>), dim3(B), dim3(T), 0, 0, src, n4, out); }, reps))
    PROB(256, 8, true);
    PROB(256, 16, true);
    PROB(512, 8, true);
    PROB(1024, 4, true);
    PROB(256, 8, false);
#define FLAT(T, U, NT, G) \
    report("flat T=" #T " U=" #U " nt=" #NT " G=" #G, \
           time_ms([&] { hipLaunchKernelGGL((k_flat<T, U, NT>), dim3(G), dim3(T), 0, 0, src, total4, out); }, reps))
    FLAT(256, 8, true, 1024);
    FLAT(256, 8, true, 2048);
    FLAT(512, 8, true, 1024);
    FLAT(256, 4, true, 4096);
    FLAT(256, 8, false, 2048);
#define CHUNK(T, U, NT, G, C) \
    report("chunk T=" #T " U=" #U " nt=" #NT " G=" #G " C=" #C, \
           time_ms([&] { hipLaunchKernelGGL((k_chunk<T, U, NT>), dim3(G), dim3(T), 0, 0, src, total4, (long long)C, out); }, reps))
    CHUNK(256, 8, true, 1024, 16384);
    CHUNK(256, 8, true, 2048, 16384);
    CHUNK(512, 8, true, 1024, 65536);
    CHUNK(256, 16, true, 768, 65536);
    // the hot kernel's shape again, last, to check drift over the run
    PROB(256, 8, true);
    CHECK(hipFree(src));
    CHECK(hipFree(out));
    return 0;
}
