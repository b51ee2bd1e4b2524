// pqp_io.cpp -- host-side readers for the reference's input formats.
//
// example/*.txt (PQP_CPU.c:757-930): each file is one line of `%f` tokens;
// matrices are listed transposed, i.e. the file's (outer, inner) listing puts
// token o*inner + in at element [in][o] of the row-major matrix.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pqp_internal.h"

namespace pqp {

static int read_tokens(const std::string& path, float* dst, int count) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return set_error(PQP_ERR_IO, "cannot open %s", path.c_str());
    for (int i = 0; i < count; ++i) {
        if (std::fscanf(f, "%f", dst + i) != 1) {  // same conversion as the reference's fscanf
            std::fclose(f);
            return set_error(PQP_ERR_IO, "%s: expected %d values, found %d", path.c_str(), count, i);
        }
    }
    std::fclose(f);
    return PQP_OK;
}

static int read_transposed(const std::string& path, float* out, int outer, int inner) {
    std::vector<float> tmp((size_t)outer * inner);
    int rc = read_tokens(path, tmp.data(), outer * inner);
    if (rc != PQP_OK) return rc;
    for (int o = 0; o < outer; ++o)
        for (int in = 0; in < inner; ++in) out[(size_t)in * outer + o] = tmp[(size_t)o * inner + in];
    return PQP_OK;
}

int read_example(const char* dir, int m, int nd, int ns, ExampleData& e) {
    if (!dir || m <= 0 || nd <= 0 || ns <= 0) return set_error(PQP_ERR_ARG, "read_example: bad arguments");
    const int N = 4 * m;
    e.m = m;
    e.nd = nd;
    e.ns = ns;
    e.Qp_inv.assign((size_t)m * m, 0.f);
    e.Fp1.assign((size_t)m * nd, 0.f);
    e.Fp2.assign((size_t)m * ns, 0.f);
    e.Fp3.assign(m, 0.f);
    e.Mp1.assign((size_t)ns * ns, 0.f);
    e.Mp2.assign((size_t)nd * ns, 0.f);
    e.Mp3.assign((size_t)nd * nd, 0.f);
    e.Mp4.assign(ns, 0.f);
    e.Mp5.assign(nd, 0.f);
    e.Mp6.assign(1, 0.f);
    e.Gp.assign((size_t)N * m, 0.f);
    e.Kp.assign(N, 0.f);
    e.x.assign(ns, 0.f);
    e.D.assign(nd, 0.f);
    const std::string d(dir);
    int rc;
    if ((rc = read_transposed(d + "/Qp_inv.txt", e.Qp_inv.data(), m, m))) return rc;  // :764-773
    if ((rc = read_transposed(d + "/Fp1.txt", e.Fp1.data(), nd, m))) return rc;      // :776-785
    if ((rc = read_transposed(d + "/Fp2.txt", e.Fp2.data(), ns, m))) return rc;      // :788-797
    if ((rc = read_tokens(d + "/Fp3.txt", e.Fp3.data(), m))) return rc;              // :800-806
    if ((rc = read_transposed(d + "/Mp1.txt", e.Mp1.data(), ns, ns))) return rc;     // :809-818
    if ((rc = read_transposed(d + "/Mp2.txt", e.Mp2.data(), ns, nd))) return rc;     // :821-830
    if ((rc = read_transposed(d + "/Mp3.txt", e.Mp3.data(), nd, nd))) return rc;     // :833-842
    if ((rc = read_tokens(d + "/Mp4.txt", e.Mp4.data(), ns))) return rc;             // :845-851
    if ((rc = read_tokens(d + "/Mp5.txt", e.Mp5.data(), nd))) return rc;             // :854-860
    if ((rc = read_tokens(d + "/Mp6.txt", e.Mp6.data(), 1))) return rc;              // :863-866
    if ((rc = read_transposed(d + "/Gp.txt", e.Gp.data(), m, N))) return rc;         // :869-878
    if ((rc = read_tokens(d + "/Kp.txt", e.Kp.data(), N))) return rc;                // :881-887
    if ((rc = read_tokens(d + "/D.txt", e.D.data(), nd))) return rc;                 // :914-920
    if ((rc = read_tokens(d + "/x.txt", e.x.data(), ns))) return rc;                 // :923-929
    return PQP_OK;
}

// Z.txt and Theta.txt are read by the reference but never used (PQP_CPU.c:889-911).
int read_unused_example(const char* dir, int ns, int no, int nd, float* Z, float* theta7) {
    const std::string d(dir);
    int rc;
    if (Z && (rc = read_transposed(d + "/Z.txt", Z, ns, no))) return rc;
    if (theta7 && (rc = read_transposed(d + "/Theta.txt", theta7, nd, no))) return rc;
    return PQP_OK;
}

}  // namespace pqp
