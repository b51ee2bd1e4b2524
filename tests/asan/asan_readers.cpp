// CPU AddressSanitizer / UBSan harness of the host readers (no GPU, no HIP):
// pqp_read_example (PQP_CPU.c:757-930's input()) and pqp_read_testfile
// (testing/ sample files, PQP_CPU_test.c:936-978) on missing, short,
// malformed, oversized and changed-between-calls files.  Built by
// tests/asan/Makefile from pqp_io.cpp + pqp_host.cpp; run by
// tests/test_asan.py.  Exit 0 = every case returned the expected status and
// the sanitizers stayed quiet.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pqp.h"

static int g_fail = 0;
#define EXPECT(cond, ...)                                   \
    do {                                                    \
        if (!(cond)) {                                      \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);              \
            std::fprintf(stderr, " (%s)\n", pqp_last_error()); \
            ++g_fail;                                       \
        }                                                   \
    } while (0)

static void write_file(const std::string& path, const std::string& text) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) {
        std::perror(path.c_str());
        std::exit(2);
    }
    std::fputs(text.c_str(), f);
    std::fclose(f);
}

// bundled example sizes (PQP_CPU.c:13-17): m = 7, nd = 1, ns = 29
struct Ex {
    std::vector<float> Qp_inv = std::vector<float>(49), Fp1 = std::vector<float>(7), Fp2 = std::vector<float>(203),
                       Fp3 = std::vector<float>(7), Mp1 = std::vector<float>(841), Mp2 = std::vector<float>(29),
                       Mp3 = std::vector<float>(1), Mp4 = std::vector<float>(29), Mp5 = std::vector<float>(1),
                       Mp6 = std::vector<float>(1), Gp = std::vector<float>(196), Kp = std::vector<float>(28),
                       x = std::vector<float>(29), D = std::vector<float>(1);
    int read(const std::string& dir) {
        return pqp_read_example(dir.c_str(), 7, 1, 29, Qp_inv.data(), Fp1.data(), Fp2.data(), Fp3.data(), Mp1.data(),
                                Mp2.data(), Mp3.data(), Mp4.data(), Mp5.data(), Mp6.data(), Gp.data(), Kp.data(),
                                x.data(), D.data());
    }
};

static std::string tokens(int n, float v = 0.5f) {
    std::string s;
    char b[32];
    for (int i = 0; i < n; ++i) {
        std::snprintf(b, sizeof b, "%f ", v);
        s += b;
    }
    return s + "#";
}

static void write_example(const std::string& dir, int short_qp_inv) {
    const struct {
        const char* name;
        int n;
    } files[] = {{"Qp_inv", 49}, {"Fp1", 7}, {"Fp2", 203}, {"Fp3", 7}, {"Mp1", 841}, {"Mp2", 29}, {"Mp3", 1},
                 {"Mp4", 29},    {"Mp5", 1}, {"Mp6", 1},   {"Gp", 196}, {"Kp", 28},  {"D", 1},    {"x", 29}};
    for (const auto& f : files) {
        const int n = (short_qp_inv && !std::strcmp(f.name, "Qp_inv")) ? short_qp_inv : f.n;
        write_file(dir + "/" + f.name + ".txt", tokens(n));
    }
}

static int read_tf(const std::string& path, int* M, int* N, std::vector<float>* a = nullptr) {
    if (!a) return pqp_read_testfile(path.c_str(), 1, M, N, nullptr, nullptr, nullptr, nullptr, nullptr);
    return pqp_read_testfile(path.c_str(), 1, M, N, a[0].data(), a[1].data(), a[2].data(), a[3].data(), a[4].data());
}

static std::string testfile(int M, int N, int drop_gp = 0) {
    std::string s = std::to_string(M) + " " + std::to_string(N) + "\n";
    for (int i = 0; i < M; ++i) s += "0.5 ";
    for (int i = 0; i < M; ++i) s += "1.0 ";
    s += "1.0 ";
    for (int i = 0; i < N; ++i) s += "2.0 ";
    for (long i = 0; i < (long)N * M - drop_gp; ++i) s += (i % 3 == 0) ? "-1 " : "2 ";
    return s;
}

int main(int argc, char** argv) {
    const std::string tmp = argc > 1 ? argv[1] : "/tmp";
    // ---- example/ reader ----
    {
        Ex e;
        EXPECT(e.read(tmp + "/does_not_exist") == PQP_ERR_IO, "missing directory");
        EXPECT(pqp_read_example(nullptr, 7, 1, 29, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == PQP_ERR_ARG,
               "null dir");
        EXPECT(pqp_read_example(tmp.c_str(), 1 << 20, 1, 29, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == PQP_ERR_ARG,
               "oversized m");
        const std::string good = tmp + "/ex_good", shrt = tmp + "/ex_short";
        (void)!std::system(("mkdir -p '" + good + "' '" + shrt + "'").c_str());
        write_example(good, 0);
        write_example(shrt, 48);  // one token short
        EXPECT(e.read(good) == PQP_OK, "complete example");
        EXPECT(e.Qp_inv[0] == 0.5f && e.Gp[195] == 0.5f && e.D[0] == 0.5f, "example values");
        EXPECT(e.read(shrt) == PQP_ERR_IO, "short Qp_inv.txt");
        // NULL outputs are skipped, not written
        EXPECT(pqp_read_example(good.c_str(), 7, 1, 29, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == PQP_OK,
               "NULL outputs");
    }
    // ---- testing/ reader ----
    {
        int M = 0, N = 0;
        EXPECT(read_tf(tmp + "/nope.txt", &M, &N) == PQP_ERR_IO, "missing file");
        EXPECT(pqp_read_testfile(nullptr, 1, &M, &N, nullptr, nullptr, nullptr, nullptr, nullptr) == PQP_ERR_ARG,
               "null path");
        const std::string p = tmp + "/tf.txt";
        write_file(p, "");
        EXPECT(read_tf(p, &M, &N) == PQP_ERR_IO, "empty file");
        write_file(p, "3 -4\n");
        EXPECT(read_tf(p, &M, &N) == PQP_ERR_IO, "negative N");
        write_file(p, "abc def\n");
        EXPECT(read_tf(p, &M, &N) == PQP_ERR_IO, "non-numeric header");
        write_file(p, "2000000000 2000000000\n");
        EXPECT(read_tf(p, &M, &N) == PQP_ERR_IO, "oversized header");
        write_file(p, "60000 60000\n");  // within the per-dimension bound, N*M + M*M is not
        EXPECT(read_tf(p, &M, &N) == PQP_ERR_IO, "oversized product");
        write_file(p, testfile(3, 5, 1));
        EXPECT(read_tf(p, &M, &N) == PQP_ERR_IO, "short Gp");
        write_file(p, testfile(3, 5));
        EXPECT(read_tf(p, &M, &N) == PQP_OK && M == 3 && N == 5, "header of a good file");
        std::vector<float> a[5] = {std::vector<float>(9), std::vector<float>(3), std::vector<float>(1),
                                   std::vector<float>(15), std::vector<float>(5)};
        EXPECT(read_tf(p, &M, &N, a) == PQP_OK, "good file");
        EXPECT(a[0][0] == 0.5f && a[0][1] == 0.0f && a[3][0] == 1.0f && a[3][1] == -1.0f, "values / Gp quirk");
        EXPECT(pqp_read_testfile(p.c_str(), 1, nullptr, nullptr, a[0].data(), a[1].data(), a[2].data(), a[3].data(),
                                 a[4].data()) == PQP_ERR_ARG,
               "fill without expected dims");
        // the file grows between the sizing call and the filling call: refused, nothing written
        write_file(p, testfile(4, 7));
        std::vector<float> before = a[3];
        EXPECT(read_tf(p, &M, &N, a) == PQP_ERR_IO, "file changed between the calls");
        EXPECT(a[3] == before, "no write after a refused fill");
    }
    if (g_fail) {
        std::fprintf(stderr, "%d case(s) failed\n", g_fail);
        return 1;
    }
    std::printf("asan_readers: all cases passed\n");
    return 0;
}
