// pqp_io.cpp -- host-side readers for the reference's input formats.
//
// example/*.txt (PQP_CPU.c:757-930): each file is one line of `%f` tokens;
// matrices are listed transposed, i.e. the file's (outer, inner) listing puts
// token o*inner + in at element [in][o] of the row-major matrix.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
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
    if (m > (1 << 14) || nd > (1 << 14) || ns > (1 << 14))
        return set_error(PQP_ERR_ARG, "read_example: dimensions out of range (m=%d nd=%d ns=%d)", m, nd, ns);
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

// glibc rand() from its default seed (srand(1)): the TYPE_3 additive-feedback
// generator, r[i] = r[i-3] + r[i-31] (mod 2^32), output r[i] >> 1, with the
// first 310 outputs discarded.  The testing/ harness overwrites Kp with
// fabs(10.0*rand()/RAND_MAX) (testing/GPU unoptimized version/
// PQP_GPU_unoptimized.cu:775) without seeding, i.e. this sequence.
class GlibcRand {
   public:
    explicit GlibcRand(uint32_t seed = 1) {
        int32_t r[34];
        r[0] = (int32_t)(seed ? seed : 1);
        for (int i = 1; i < 31; ++i) {
            const int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
            int64_t w = 16807 * lo - 2836 * hi;
            if (w < 0) w += 2147483647;
            r[i] = (int32_t)w;
        }
        for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
        for (int i = 0; i < 34; ++i) ring_[i] = (uint32_t)r[i];
        n_ = 34;
        for (int i = 0; i < 310; ++i) next();
    }
    int next() {
        const uint32_t v = ring_[(n_ - 31) % 34] + ring_[(n_ - 3) % 34];
        ring_[n_ % 34] = v;
        ++n_;
        return (int)(v >> 1);
    }

   private:
    uint32_t ring_[34];
    uint64_t n_;
};

// testing/ sample-test file (written by testing/test_generator.c:936-987, read
// by testing/GPU unoptimized version/PQP_GPU_unoptimized.cu:751-794 and
// testing/CPU version/PQP_CPU_test.c:936-978): "M N", M diagonal entries of
// Qp_inv, M of Fp, Mp, N of Kp, then N x M integers for Gp.
// Largest header the reader accepts: M, N <= 65536 and Gp (N x M) plus the
// dense Qp_inv (M x M) within 2^30 floats (4 GiB of host memory).  The
// reference's own sample files are (100, 400), (500, 1500), (800, 1200).
constexpr long long kTestfileMaxDim = 1 << 16, kTestfileMaxFloats = 1LL << 30;

int read_testfile(const char* path, bool glibc_kp, TestfileData& t) {
    FILE* f = std::fopen(path, "r");
    if (!f) return set_error(PQP_ERR_IO, "cannot open %s", path);
    auto fail = [&](const char* what) {
        std::fclose(f);
        return set_error(PQP_ERR_IO, "%s: short or malformed file (%s)", path, what);
    };
    int M = 0, N = 0;
    if (std::fscanf(f, "%d%d", &M, &N) != 2 || M <= 0 || N <= 0) return fail("header");
    if (M > kTestfileMaxDim || N > kTestfileMaxDim ||
        (long long)N * M + (long long)M * M > kTestfileMaxFloats) {
        std::fclose(f);
        return set_error(PQP_ERR_IO, "%s: header M=%d N=%d exceeds the reader's bounds (M, N <= %lld)", path, M, N,
                         kTestfileMaxDim);
    }
    t.M = M;
    t.N = N;
    try {
        t.Qp_inv.assign((size_t)M * M, 0.0f);
        t.Fp.assign(M, 0.0f);
        t.Mp.assign(1, 0.0f);
        t.Kp.assign(N, 0.0f);
        t.Gp.assign((size_t)N * M, 0.0f);
    } catch (const std::bad_alloc&) {
        std::fclose(f);
        return set_error(PQP_ERR_ALLOC, "%s: no host memory for M=%d N=%d", path, M, N);
    }
    for (int i = 0; i < M; ++i)
        if (std::fscanf(f, "%f", &t.Qp_inv[(size_t)i * M + i]) != 1) return fail("Qp_inv");
    for (int i = 0; i < M; ++i)
        if (std::fscanf(f, "%f", &t.Fp[i]) != 1) return fail("Fp");
    if (std::fscanf(f, "%f", &t.Mp[0]) != 1) return fail("Mp");
    for (int i = 0; i < N; ++i)
        if (std::fscanf(f, "%f", &t.Kp[i]) != 1) return fail("Kp");
    GlibcRand rng(1);
    for (int i = 0; i < N; ++i) {
        if (glibc_kp) t.Kp[i] = (float)std::fabs(10.0 * rng.next() / 2147483647.0);  // RAND_MAX
        for (int j = 0; j < M; ++j) {
            int v = 0;
            if (std::fscanf(f, "%d", &v) != 1) return fail("Gp");
            // C remainder: -1 % 3 == -1, so a file value of -1 maps to +1 (the quirk)
            t.Gp[(size_t)i * M + j] = (v % 3 == 0) ? 0.0f : ((v % 3 == 2) ? -1.0f : 1.0f);
        }
    }
    std::fclose(f);
    return PQP_OK;
}

int glibc_rand_sequence(int n, int* out) {
    GlibcRand rng(1);
    for (int i = 0; i < n; ++i) out[i] = rng.next();
    return PQP_OK;
}

}  // namespace pqp
