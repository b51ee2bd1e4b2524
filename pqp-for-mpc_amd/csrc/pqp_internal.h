// pqp_internal.h -- host-side internals shared by the libpqp translation units.
#pragma once
// No HIP here: pqp_io.cpp and pqp_host.cpp build without it (tests/asan/).
// PQP_HIP expands only where pqp_launch.h (hip_runtime.h) is included.
#include <cstddef>
#include <string>
#include <vector>

#include "../../include/pqp.h"

namespace pqp {

// Record an error for pqp_last_error() and return `code`.
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void restore_error(const std::string& text);  // put back a saved pqp_last_error() text

#define PQP_HIP(expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return ::pqp::set_error(PQP_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                                    __LINE__);                                                         \
    } while (0)

#define PQP_TRY(expr)                \
    do {                             \
        int rc_ = (expr);            \
        if (rc_ != PQP_OK) return rc_; \
    } while (0)

// The bundled example (PQP_CPU.c:757-930) as read from disk.
struct ExampleData {
    int m = 0, nd = 0, ns = 0;  // nInput*pHorizon, nDis*pHorizon, nState
    std::vector<float> Qp_inv, Fp1, Fp2, Fp3, Mp1, Mp2, Mp3, Mp4, Mp5, Mp6, Gp, Kp, x, D;
};
int read_example(const char* dir, int m, int nd, int ns, ExampleData& e);
int read_unused_example(const char* dir, int ns, int no, int nd, float* Z, float* theta7);

// testing/ sample-test file (see pqp_io.cpp).
struct TestfileData {
    int M = 0, N = 0;
    std::vector<float> Qp_inv, Fp, Mp, Kp, Gp;
};
int read_testfile(const char* path, bool glibc_kp, TestfileData& t);
int glibc_rand_sequence(int n, int* out);

// Reference compile-time dimensions (PQP_CPU.c:13-17).
constexpr int kRefPHorizon = 1, kRefNState = 29, kRefNInput = 7, kRefNOutput = 7, kRefNDis = 1;

}  // namespace pqp
