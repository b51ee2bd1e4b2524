// CPU AddressSanitizer harness of the C ABI's argument and handle paths
// (pqp_problem_*, pqp_rowblock_*, the drop-ins' argument checks) in a host
// build of libpqp's shim: no GPU is visible here, so every call must fail
// cleanly -- PQP_ERR_ARG for bad arguments (checked before any HIP call),
// PQP_ERR_NO_DEVICE once the arguments are fine -- with no sanitizer report.
#include <cstdio>
#include <vector>

#include "../../include/pqp.h"

static int g_fail = 0;
#define EXPECT_RC(call, want)                                                                           \
    do {                                                                                                \
        const int rc_ = (call);                                                                         \
        if (rc_ != (want)) {                                                                            \
            std::fprintf(stderr, "FAIL line %d: %s -> %d, want %d (%s)\n", __LINE__, #call, rc_, want, \
                         pqp_last_error());                                                             \
            ++g_fail;                                                                                   \
        }                                                                                               \
    } while (0)

int main() {
    const int N = 28, M = 7;
    std::vector<float> Qd(N * N, 1.0f), Fd(N), Md(1), Qp(M * M), Qi(M * M), Fp(M), Mp(1), Gp(N * M), Kp(N), Y(N),
        U(M);
    pqp_problem* P = reinterpret_cast<pqp_problem*>(0x1);
    EXPECT_RC(pqp_problem_create(Qd.data(), Fd.data(), Md.data(), Qp.data(), Qi.data(), Fp.data(), Mp.data(),
                                 Gp.data(), Kp.data(), N, M, nullptr),
              PQP_ERR_ARG);
    EXPECT_RC(pqp_problem_create(nullptr, Fd.data(), Md.data(), Qp.data(), Qi.data(), Fp.data(), Mp.data(),
                                 Gp.data(), Kp.data(), N, M, &P),
              PQP_ERR_ARG);
    if (P != nullptr) {
        std::fprintf(stderr, "FAIL: *out not cleared on error\n");
        ++g_fail;
    }
    EXPECT_RC(pqp_problem_create(Qd.data(), Fd.data(), Md.data(), Qp.data(), Qi.data(), Fp.data(), Mp.data(),
                                 Gp.data(), Kp.data(), 0, M, &P),
              PQP_ERR_ARG);
    EXPECT_RC(pqp_problem_create(Qd.data(), Fd.data(), Md.data(), Qp.data(), Qi.data(), Fp.data(), Mp.data(),
                                 Gp.data(), Kp.data(), N, M, &P),
              PQP_ERR_NO_DEVICE);
    EXPECT_RC(pqp_problem_solve(nullptr, PQP_MODE_FIXED, 10, 0, Y.data(), U.data(), nullptr, nullptr, nullptr),
              PQP_ERR_ARG);
    EXPECT_RC(pqp_problem_destroy(nullptr), PQP_OK);
    EXPECT_RC(pqp_solve_dual(Qd.data(), Fd.data(), Md.data(), Qp.data(), Qi.data(), Fp.data(), Mp.data(), Gp.data(),
                             Kp.data(), N, M, 7, 10, 0, Y.data(), U.data(), nullptr, nullptr, nullptr),
              PQP_ERR_ARG);
    EXPECT_RC(pqp_solve_dual(Qd.data(), Fd.data(), Md.data(), Qp.data(), Qi.data(), Fp.data(), Mp.data(), Gp.data(),
                             Kp.data(), N, M, PQP_MODE_FIXED, 10, 0, nullptr, U.data(), nullptr, nullptr, nullptr),
              PQP_ERR_ARG);
    EXPECT_RC(pqp_solve_dual(Qd.data(), Fd.data(), Md.data(), Qp.data(), Qi.data(), Fp.data(), Mp.data(), Gp.data(),
                             Kp.data(), N, M, PQP_MODE_FIXED, 10, 0, Y.data(), U.data(), nullptr, nullptr, nullptr),
              PQP_ERR_NO_DEVICE);
    pqp_rowblock* b = reinterpret_cast<pqp_rowblock*>(0x1);
    EXPECT_RC(pqp_rowblock_create(Qd.data(), N, Fd.data(), N, 0, N, nullptr, nullptr), PQP_ERR_ARG);
    EXPECT_RC(pqp_rowblock_create(Qd.data(), N - 1, Fd.data(), N, 0, N, nullptr, &b), PQP_ERR_ARG);
    EXPECT_RC(pqp_rowblock_create(Qd.data(), N, Fd.data(), N, 5, N, nullptr, &b), PQP_ERR_ARG);
    EXPECT_RC(pqp_rowblock_update(nullptr, Y.data(), Y.data(), nullptr), PQP_ERR_ARG);
    EXPECT_RC(pqp_rowblock_check(nullptr, nullptr), PQP_ERR_ARG);
    EXPECT_RC(pqp_rowblock_destroy(nullptr), PQP_OK);
    EXPECT_RC(pqp_batch_update(0, N, Qd.data(), N, (long long)N * N, Fd.data(), Fd.data(), N, Y.data(), U.data(),
                               nullptr),
              PQP_ERR_ARG);
    EXPECT_RC(pqp_update_host(Qd.data(), Fd.data(), Fd.data(), Y.data(), Y.data(), 0), PQP_ERR_ARG);
    if (g_fail) {
        std::fprintf(stderr, "%d case(s) failed\n", g_fail);
        return 1;
    }
    std::printf("asan_capi: all cases passed\n");
    return 0;
}
