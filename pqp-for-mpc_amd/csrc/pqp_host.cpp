// pqp_host.cpp -- the host-only part of the C ABI: the thread-local error
// text (pqp_last_error) and the two file readers (pqp_read_example,
// pqp_read_testfile).  No HIP: this file and pqp_io.cpp also build on their
// own into the CPU AddressSanitizer harness (tests/asan/).
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "pqp_internal.h"

namespace pqp {

static thread_local std::string t_err;

int set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}

void restore_error(const std::string& text) { t_err = text; }

}  // namespace pqp

using namespace pqp;

extern "C" {

const char* pqp_last_error(void) { return t_err.c_str(); }

int pqp_read_example(const char* dir, int m, int nd, int ns, float* Qp_inv, float* Fp1, float* Fp2, float* Fp3,
                     float* Mp1, float* Mp2, float* Mp3, float* Mp4, float* Mp5, float* Mp6, float* Gp, float* Kp,
                     float* x, float* D) {
    ExampleData e;
    try {
        PQP_TRY(read_example(dir, m, nd, ns, e));
    } catch (const std::bad_alloc&) {
        return set_error(PQP_ERR_ALLOC, "pqp_read_example: no host memory (m=%d nd=%d ns=%d)", m, nd, ns);
    }
    auto put = [](float* dst, const std::vector<float>& v) {
        if (dst) std::memcpy(dst, v.data(), v.size() * sizeof(float));
    };
    put(Qp_inv, e.Qp_inv);
    put(Fp1, e.Fp1);
    put(Fp2, e.Fp2);
    put(Fp3, e.Fp3);
    put(Mp1, e.Mp1);
    put(Mp2, e.Mp2);
    put(Mp3, e.Mp3);
    put(Mp4, e.Mp4);
    put(Mp5, e.Mp5);
    put(Mp6, e.Mp6);
    put(Gp, e.Gp);
    put(Kp, e.Kp);
    put(x, e.x);
    put(D, e.D);
    return PQP_OK;
}

int pqp_read_testfile(const char* path, int glibc_kp, int* M_out, int* N_out, float* Qp_inv, float* Fp, float* Mp,
                      float* Gp, float* Kp) {
    if (!path) return set_error(PQP_ERR_ARG, "pqp_read_testfile: null path");
    const bool fill = Qp_inv || Fp || Mp || Gp || Kp;
    // filling call: the caller passes the (M, N) its arrays were sized for
    if (fill && (!M_out || !N_out))
        return set_error(PQP_ERR_ARG, "pqp_read_testfile: pass the expected M and N along with the arrays");
    TestfileData t;
    PQP_TRY(read_testfile(path, glibc_kp != 0, t));
    if (fill && (t.M != *M_out || t.N != *N_out))
        return set_error(PQP_ERR_IO, "pqp_read_testfile: %s holds M=%d N=%d, the arrays were sized for M=%d N=%d",
                         path, t.M, t.N, *M_out, *N_out);
    if (M_out) *M_out = t.M;
    if (N_out) *N_out = t.N;
    auto put = [](float* dst, const std::vector<float>& v) {
        if (dst) std::memcpy(dst, v.data(), v.size() * sizeof(float));
    };
    put(Qp_inv, t.Qp_inv);
    put(Fp, t.Fp);
    put(Mp, t.Mp);
    put(Gp, t.Gp);
    put(Kp, t.Kp);
    return PQP_OK;
}

}  // extern "C"
