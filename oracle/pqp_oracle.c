/*
 * oracle/pqp_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A from-scratch CPU restatement of the reference solver's arithmetic
 * (yashsoni501/PQP-for-MPC, PQP_CPU.c).  It exists so that tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() have a checker.  Nothing in the
 * product (pqp-for-mpc_amd/, include/) links, loads or calls this file: the
 * product path is HIP-only and fails loudly without its extension.
 *
 * Parity is PINNED: tests/test_oracle.py compares every function below with
 * the reference itself (oracle/_ref/libpqp_ref.so, compiled from
 * /root/reference/PQP_CPU.c by oracle/Makefile) and with the committed golden
 * fixtures under tests/golden/ that were generated from that build.
 *
 * Float rules followed:
 *   - every product is rounded before it is added (build with
 *     -ffp-contract=off; no -ffast-math);
 *   - every dot product runs k = 0..b-1 in order from +0.0f;
 *   - max() is the reference's `a > b ? a : b` on floats (PQP_CPU.c:32-36),
 *     never fmaxf;
 *   - the few double-promoted expressions of the reference are reproduced
 *     literally (computeCost's 0.5*t, compare's erc*Kp, terminate's gap tests).
 */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define ORC_TOL 1e-6 /* erc = eac = eaj = erj, PQP_CPU.c:19-22 */

/* PQP_CPU.c:32-36 */
static float orc_fmax_ref(float a, float b) { return (a > b) ? a : b; }

/* Element (i,k) of an a-by-b operand that is stored either as is (row-major
 * a x b) or transposed (row-major b x a).  Mirrors the index forms at
 * PQP_CPU.c:96,110,124,138. */
static inline float orc_lhs(const float *A, int tA, int a, int b, int i, int k)
{
    return tA ? A[(size_t)k * a + i] : A[(size_t)i * b + k];
}
static inline float orc_rhs(const float *B, int tB, int b, int c, int k, int j)
{
    return tB ? B[(size_t)j * b + k] : B[(size_t)k * c + j];
}

/* matrixMultiply (PQP_CPU.c:84-147): out[a x c] = op(A)[a x b] * op(B)[b x c].
 * Results are staged so the output may alias an input (PQP_CPU.c:86,144). */
void orc_matmul(float *out, const float *A, int tA, const float *B, int tB, int a, int b, int c)
{
    float *stage = (float *)malloc(sizeof(float) * (size_t)a * c + 4);
    for (int i = 0; i < a; ++i)
        for (int j = 0; j < c; ++j) {
            float s = 0.0f;
            for (int k = 0; k < b; ++k)
                s += orc_lhs(A, tA, a, b, i, k) * orc_rhs(B, tB, b, c, k, j);
            stage[(size_t)i * c + j] = s;
        }
    memcpy(out, stage, sizeof(float) * (size_t)a * c);
    free(stage);
}

/* Gauss_Jordan (PQP_CPU.c:251-326): no pivoting, one bubble pass on column 0. */
void orc_gauss_jordan(const float *A, float *inv, int n)
{
    const int w = 2 * n;
    float *aug = (float *)calloc((size_t)n * w + 1, sizeof(float));
    for (int r = 0; r < n; ++r) {
        for (int c = 0; c < n; ++c) aug[(size_t)r * w + c] = A[(size_t)r * n + c];
        aug[(size_t)r * w + n + r] = 1.0f;
    }
    for (int r = n - 1; r > 0; --r) {
        float *lo = aug + (size_t)r * w, *hi = aug + (size_t)(r - 1) * w;
        if (hi[0] < lo[0])
            for (int c = 0; c < w; ++c) { float t = lo[c]; lo[c] = hi[c]; hi[c] = t; }
    }
    for (int p = 0; p < n; ++p) {
        const float *prow = aug + (size_t)p * w;
        for (int r = 0; r < n; ++r) {
            if (r == p) continue;
            float *row = aug + (size_t)r * w;
            float f = row[p] / prow[p];
            for (int c = 0; c < w; ++c) row[c] -= prow[c] * f;
        }
    }
    for (int r = 0; r < n; ++r) {
        float *row = aug + (size_t)r * w;
        float d = row[r];
        for (int c = 0; c < w; ++c) row[c] = row[c] / d;
    }
    for (int r = 0; r < n; ++r)
        memcpy(inv + (size_t)r * n, aug + (size_t)r * w + n, sizeof(float) * n);
    free(aug);
}

/* computeFp (PQP_CPU.c:373-382): Fp = Fp1*D + Fp2*x - Fp3.
 * m = nInput*pHorizon, nd = nDis*pHorizon, ns = nState. */
void orc_compute_fp(float *Fp, const float *Fp1, const float *Fp2, const float *Fp3,
                    const float *D, const float *x, int m, int nd, int ns)
{
    float *t = (float *)malloc(sizeof(float) * m);
    orc_matmul(Fp, Fp1, 0, D, 0, m, nd, 1);
    orc_matmul(t, Fp2, 0, x, 0, m, ns, 1);
    for (int i = 0; i < m; ++i) Fp[i] += 1.0f * t[i];
    for (int i = 0; i < m; ++i) Fp[i] += -1.0f * Fp3[i];
    free(t);
}

/* computeMp (PQP_CPU.c:395-428): every term is added halved, in this order. */
void orc_compute_mp(float *Mp, const float *Mp1, const float *Mp2, const float *Mp3,
                    const float *Mp4, const float *Mp5, const float *Mp6,
                    const float *D, const float *x, int nd, int ns)
{
    int big = ns > nd ? ns : nd;
    float *row = (float *)malloc(sizeof(float) * (size_t)big);
    float acc = 0.0f;
    orc_matmul(row, x, 1, Mp1, 0, 1, ns, ns);     /* x' Mp1    */
    orc_matmul(row, row, 0, x, 0, 1, ns, 1);      /* (x' Mp1) x */
    acc += row[0] / 2;
    orc_matmul(row, D, 1, Mp2, 0, 1, nd, ns);     /* D' Mp2    */
    orc_matmul(row, row, 0, x, 0, 1, ns, 1);
    acc += row[0] / 2;
    orc_matmul(row, Mp4, 1, x, 0, 1, ns, 1);      /* Mp4' x    */
    acc += row[0] / 2;
    orc_matmul(row, D, 1, Mp3, 0, 1, nd, nd);     /* D' Mp3    */
    orc_matmul(row, row, 0, D, 0, 1, nd, 1);
    acc += row[0] / 2;
    orc_matmul(row, Mp5, 1, D, 0, 1, nd, 1);      /* Mp5' D    */
    acc += row[0] / 2;
    acc += Mp6[0] / 2;
    Mp[0] = acc;
    free(row);
}

/* convertToDual + computeQd/Fd/Md (PQP_CPU.c:440-498). */
void orc_convert_to_dual(float *Qd, float *Fd, float *Md, const float *Qp_inv,
                         const float *Gp, const float *Kp, const float *Fp,
                         const float *Mp, int N, int M)
{
    float *GQ = (float *)malloc(sizeof(float) * (size_t)N * M + 4);
    float *fq = (float *)malloc(sizeof(float) * (size_t)M + 4);
    orc_matmul(GQ, Gp, 0, Qp_inv, 0, N, M, M);     /* Gp Qp^-1           */
    orc_matmul(Qd, GQ, 0, Gp, 1, N, M, N);         /* (Gp Qp^-1) Gp'     */
    orc_matmul(Fd, GQ, 0, Fp, 0, N, M, 1);         /* (Gp Qp^-1) Fp      */
    for (int i = 0; i < N; ++i) Fd[i] += 1.0f * Kp[i];
    orc_matmul(fq, Fp, 1, Qp_inv, 0, 1, M, M);     /* Fp' Qp^-1          */
    orc_matmul(Md, fq, 0, Fp, 0, 1, M, 1);
    Md[0] -= Mp[0];
    free(GQ);
    free(fq);
}

/* computeTheta + diagonalAdd (PQP_CPU.c:503-519, 235-242): returns the
 * diagonal only; the reference's theta matrix is zero elsewhere. */
void orc_theta_diag(float *theta, const float *Qd, int N)
{
    for (int i = 0; i < N; ++i) {
        float s = 0.0f;
        for (int k = 0; k < N; ++k) s += orc_fmax_ref(0.0f, -Qd[(size_t)i * N + k]) * 1.0f;
        theta[i] = orc_fmax_ref(s, 5.0f);
    }
}

/* The reference's stored split matrices max(0,+-Qd) + Theta
 * (computeQdp_theta / computeQdn_theta, PQP_CPU.c:524-537). */
void orc_split_theta(float *Qdp_theta, float *Qdn_theta, const float *Qd, const float *theta, int N)
{
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < N; ++k) {
            size_t e = (size_t)i * N + k;
            float t = (i == k) ? theta[i] : 0.0f;
            Qdp_theta[e] = orc_fmax_ref(0.0f, Qd[e]) + 1.0f * t;
            Qdn_theta[e] = orc_fmax_ref(0.0f, -Qd[e]) + 1.0f * t;
        }
}

/* updateY2 + updY (PQP_CPU.c:603-618, 590-596) on the stored split matrices. */
void orc_update_split(float *Y_next, const float *Y, const float *Qdp_theta, const float *Qdn_theta,
                      const float *Fdp, const float *Fdn, int N)
{
    float *nd = (float *)malloc(sizeof(float) * 2 * (size_t)N + 4);
    for (int i = 0; i < N; ++i) {
        float num = 0.0f, den = 0.0f;
        const float *rn = Qdn_theta + (size_t)i * N, *rp = Qdp_theta + (size_t)i * N;
        for (int k = 0; k < N; ++k) num += rn[k] * Y[k];
        for (int k = 0; k < N; ++k) den += rp[k] * Y[k];
        nd[2 * i] = num + 1.0f * Fdn[i];
        nd[2 * i + 1] = den + 1.0f * Fdp[i];
    }
    for (int i = 0; i < N; ++i) Y_next[i] = nd[2 * i] / nd[2 * i + 1] * Y[i];
    free(nd);
}

/* Same update, with the split matrices and Fd+- derived from Qd/theta/Fd on
 * the fly (bit-identical to storing them). */
void orc_update(float *Y_next, const float *Y, const float *Qd, const float *theta,
                const float *Fd, int N)
{
    float *nd = (float *)malloc(sizeof(float) * 2 * (size_t)N + 4);
    for (int i = 0; i < N; ++i) {
        float num = 0.0f, den = 0.0f;
        const float *row = Qd + (size_t)i * N;
        for (int k = 0; k < N; ++k) {
            float t = (i == k) ? theta[i] : 0.0f;
            num += (orc_fmax_ref(0.0f, -row[k]) + 1.0f * t) * Y[k];
        }
        for (int k = 0; k < N; ++k) {
            float t = (i == k) ? theta[i] : 0.0f;
            den += (orc_fmax_ref(0.0f, row[k]) + 1.0f * t) * Y[k];
        }
        nd[2 * i] = num + 1.0f * orc_fmax_ref(0.0f, -Fd[i]);
        nd[2 * i + 1] = den + 1.0f * orc_fmax_ref(0.0f, Fd[i]);
    }
    for (int i = 0; i < N; ++i) Y_next[i] = nd[2 * i] / nd[2 * i + 1] * Y[i];
    free(nd);
}

/* computeUfromY (PQP_CPU.c:352-360): U = -Qp_inv (Gp'Y + Fp). */
void orc_u_from_y(float *U, const float *Y, const float *Fp, const float *Gp,
                  const float *Qp_inv, int N, int M)
{
    float *t = (float *)malloc(sizeof(float) * (size_t)M + 4);
    orc_matmul(t, Gp, 1, Y, 0, M, N, 1);
    for (int j = 0; j < M; ++j) t[j] += 1.0f * Fp[j];
    orc_matmul(U, Qp_inv, 0, t, 0, M, M, 1);
    for (int j = 0; j < M; ++j) U[j] = -U[j];
    free(t);
}

/* checkFeas + compare (PQP_CPU.c:632-641, 334-343). */
int orc_feasible(const float *U, const float *Gp, const float *Kp, int N, int M)
{
    float *gu = (float *)malloc(sizeof(float) * (size_t)N + 4);
    int ok = 1;
    orc_matmul(gu, Gp, 0, U, 0, N, M, 1);
    for (int i = 0; i < N; ++i)
        if (gu[i] > Kp[i] + orc_fmax_ref((float)(ORC_TOL * Kp[i]), (float)ORC_TOL)) ok = 0;
    free(gu);
    return ok;
}

/* computeCost (PQP_CPU.c:648-666): J = 0.5*(Z'Q)Z + F'Z + M/2. */
float orc_cost(const float *Z, const float *Q, const float *F, const float *Mc, int n)
{
    float J = 0.0f;
    float *row = (float *)malloc(sizeof(float) * (size_t)n + 4);
    orc_matmul(row, Z, 1, Q, 0, 1, n, n);
    orc_matmul(row, row, 0, Z, 0, 1, n, 1);
    J += 0.5 * row[0];
    orc_matmul(row, F, 1, Z, 0, 1, n, 1);
    J += row[0];
    J += Mc[0] / 2;
    free(row);
    return J;
}

/* terminate (PQP_CPU.c:673-687).  Writes U (as the reference does) and the
 * two costs when they were evaluated (jp/jd may be NULL). */
int orc_terminate(const float *Y, const float *Qd, const float *Fd, const float *Md, float *U,
                  const float *Qp, const float *Qp_inv, const float *Fp, const float *Mp,
                  const float *Gp, const float *Kp, int N, int M, float *jp, float *jd)
{
    orc_u_from_y(U, Y, Fp, Gp, Qp_inv, N, M);
    if (!orc_feasible(U, Gp, Kp, N, M)) return 0;
    float Jd = orc_cost(Y, Qd, Fd, Md, N);
    float Jp = orc_cost(U, Qp, Fp, Mp, M);
    if (jp) *jp = Jp;
    if (jd) *jd = Jd;
    if (Jp > -Jd) return 0;
    if (Jp + Jd > ORC_TOL) return 0;
    if ((Jp + Jd) / fabs(Jd) > ORC_TOL) return 0;
    return 1;
}

/* solveQuadraticDual (PQP_CPU.c:694-750) without the printf.
 *   mode 0 (converge): while(!terminate) update; h counts terminate calls
 *          (= updates + 1, the number the reference prints).  Stops early at
 *          max_updates updates and then returns -h.
 *   mode 1 (fixed):    while(h < num_iter) update  -> num_iter-1 updates, no
 *          terminate (the testing/ harness loop).
 * Returns h. */
long orc_solve(float *Y, const float *Qd, const float *Fd, const float *Md, float *U,
               const float *Qp, const float *Qp_inv, const float *Fp, const float *Mp,
               const float *Gp, const float *Kp, int N, int M, int mode, long num_iter,
               long max_updates)
{
    float *theta = (float *)malloc(sizeof(float) * (size_t)N + 4);
    float *nxt = (float *)malloc(sizeof(float) * (size_t)N + 4);
    orc_theta_diag(theta, Qd, N);
    for (int i = 0; i < N; ++i) Y[i] = 1000.0f;
    long h = 1;
    if (mode == 1) {
        while (h < num_iter) {
            orc_update(nxt, Y, Qd, theta, Fd, N);
            memcpy(Y, nxt, sizeof(float) * N);
            ++h;
        }
    } else {
        while (!orc_terminate(Y, Qd, Fd, Md, U, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M, NULL, NULL)) {
            if (h - 1 >= max_updates) { h = -h; break; }
            orc_update(nxt, Y, Qd, theta, Fd, N);
            memcpy(Y, nxt, sizeof(float) * N);
            ++h;
        }
    }
    free(theta);
    free(nxt);
    return h;
}

/* ------------------------------------------------------------------------
 * example-directory .txt reader (PQP_CPU.c:757-930).  Each file is one line of
 * `%f` tokens; matrices are written transposed (file index i*cols_f + j goes
 * to element [j][i]).  Returns 0 on success, -1 on a missing/short file.
 * ---------------------------------------------------------------------- */
static int orc_read_tokens(const char *dir, const char *name, float *dst, int count)
{
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    for (int i = 0; i < count; ++i)
        if (fscanf(f, "%f", dst + i) != 1) { fclose(f); return -1; }
    fclose(f);
    return 0;
}

/* file holds an (outer x inner) listing; element (o, in) lands at out[in*outer + o] */
static int orc_read_transposed(const char *dir, const char *name, float *out, int outer, int inner)
{
    float *tmp = (float *)malloc(sizeof(float) * (size_t)outer * inner + 4);
    int rc = orc_read_tokens(dir, name, tmp, outer * inner);
    if (rc == 0)
        for (int o = 0; o < outer; ++o)
            for (int in = 0; in < inner; ++in) out[(size_t)in * outer + o] = tmp[(size_t)o * inner + in];
    free(tmp);
    return rc;
}

/* dims: m = nInput*pHorizon, N = 4m, nd = nDis*pHorizon, ns = nState */
int orc_load_example(const char *dir, int m, int nd, int ns, float *Qp_inv, float *Fp1,
                     float *Fp2, float *Fp3, float *Mp1, float *Mp2, float *Mp3, float *Mp4,
                     float *Mp5, float *Mp6, float *Gp, float *Kp, float *x, float *D)
{
    int N = 4 * m, rc = 0;
    rc |= orc_read_transposed(dir, "Qp_inv.txt", Qp_inv, m, m);
    rc |= orc_read_transposed(dir, "Fp1.txt", Fp1, nd, m);
    rc |= orc_read_transposed(dir, "Fp2.txt", Fp2, ns, m);
    rc |= orc_read_tokens(dir, "Fp3.txt", Fp3, m);
    rc |= orc_read_transposed(dir, "Mp1.txt", Mp1, ns, ns);
    rc |= orc_read_transposed(dir, "Mp2.txt", Mp2, ns, nd);
    rc |= orc_read_transposed(dir, "Mp3.txt", Mp3, nd, nd);
    rc |= orc_read_tokens(dir, "Mp4.txt", Mp4, ns);
    rc |= orc_read_tokens(dir, "Mp5.txt", Mp5, nd);
    rc |= orc_read_tokens(dir, "Mp6.txt", Mp6, 1);
    rc |= orc_read_transposed(dir, "Gp.txt", Gp, m, N);
    rc |= orc_read_tokens(dir, "Kp.txt", Kp, N);
    rc |= orc_read_tokens(dir, "D.txt", D, nd);
    rc |= orc_read_tokens(dir, "x.txt", x, ns);
    return rc ? -1 : 0;
}

/* ------------------------------------------------------------------------
 * Synthetic primal generator (not in the reference).
 * Counter-based: every value is a pure function of (seed, instance, tag,
 * index), so the device generator reproduces it bit for bit.
 *   Qp_inv = diag(0.1 + u), Gp in {-1,0,+1}, Kp = 10u, Fp = 20u - 10, Mp = 1.
 * Must stay identical to pqp-for-mpc_amd/csrc/pqp_synth.h.
 * ---------------------------------------------------------------------- */
static inline uint32_t orc_hash32(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
uint32_t orc_synth_key(uint32_t seed, uint32_t inst, uint32_t tag)
{
    uint32_t k = orc_hash32(seed * 0x9E3779B9U + 0x632BE5ABU);
    k = orc_hash32(k ^ (inst * 0x85EBCA6BU + 0x27D4EB2FU));
    return orc_hash32(k + tag * 0xC2B2AE35U);
}
static inline uint32_t orc_synth_bits(uint32_t key, uint32_t idx) { return orc_hash32(key ^ orc_hash32(idx + 0x165667B1U)); }
static inline float orc_u01(uint32_t bits) { return (float)(bits >> 8) * (1.0f / 16777216.0f); }

void orc_synth_primal(uint32_t seed, uint32_t inst, int N, int M, float *Qp_inv, float *Gp,
                      float *Kp, float *Fp, float *Mp)
{
    uint32_t kq = orc_synth_key(seed, inst, 1), kg = orc_synth_key(seed, inst, 2);
    uint32_t kk = orc_synth_key(seed, inst, 3), kf = orc_synth_key(seed, inst, 4);
    memset(Qp_inv, 0, sizeof(float) * (size_t)M * M);
    for (int j = 0; j < M; ++j) Qp_inv[(size_t)j * M + j] = 0.1f + orc_u01(orc_synth_bits(kq, (uint32_t)j));
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < M; ++j) {
            uint32_t idx = (uint32_t)i * (uint32_t)M + (uint32_t)j;
            Gp[(size_t)i * M + j] = (float)((int)(orc_synth_bits(kg, idx) % 3U) - 1);
        }
    for (int i = 0; i < N; ++i) Kp[i] = 10.0f * orc_u01(orc_synth_bits(kk, (uint32_t)i));
    for (int j = 0; j < M; ++j) {
        float u = orc_u01(orc_synth_bits(kf, (uint32_t)j));
        float s = 20.0f * u;
        Fp[j] = s - 10.0f;
    }
    Mp[0] = 1.0f;
}

/* Fixed-iteration batch used by bench.py's cpu_baseline leg: `updates`
 * updateY2 calls on one dual problem from Y = 1000.  Returns seconds spent
 * in the update loop only (setup excluded). */

double orc_time_updates(float *Y, const float *Qd, const float *Fd, int N, long updates)
{
    float *theta = (float *)malloc(sizeof(float) * (size_t)N + 4);
    float *Qp = (float *)malloc(sizeof(float) * (size_t)N * N + 4);
    float *Qn = (float *)malloc(sizeof(float) * (size_t)N * N + 4);
    float *Fp = (float *)malloc(sizeof(float) * (size_t)N + 4);
    float *Fn = (float *)malloc(sizeof(float) * (size_t)N + 4);
    float *nxt = (float *)malloc(sizeof(float) * (size_t)N + 4);
    orc_theta_diag(theta, Qd, N);
    orc_split_theta(Qp, Qn, Qd, theta, N);
    for (int i = 0; i < N; ++i) {
        Fp[i] = orc_fmax_ref(0.0f, Fd[i]);
        Fn[i] = orc_fmax_ref(0.0f, -Fd[i]);
        Y[i] = 1000.0f;
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (long u = 0; u < updates; ++u) {
        orc_update_split(nxt, Y, Qp, Qn, Fp, Fn, N);
        memcpy(Y, nxt, sizeof(float) * N);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(theta); free(Qp); free(Qn); free(Fp); free(Fn); free(nxt);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* All-core comparison row of bench.py's cpu_baseline (labelled "not
 * reference"): `rounds` fixed-mode updates of each of B independent problems
 * whose stored split matrices lie back to back (Qp/Qn: B x N x N, Fp/Fn/Y:
 * B x N), the problems spread over `threads` OpenMP threads, each update the
 * bit-exact orc_update_split (PQP_CPU.c:603-618).  Returns seconds. */
double orc_time_updates_batch(int B, float *Y, const float *Qp, const float *Qn, const float *Fp, const float *Fn,
                              int N, long rounds, int threads)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(threads)
#endif
    for (int b = 0; b < B; ++b) {
        float *nxt = (float *)malloc(sizeof(float) * (size_t)N + 4);
        float *y = Y + (size_t)b * N;
        const size_t o = (size_t)b * N * N;
        for (long r = 0; r < rounds; ++r) {
            orc_update_split(nxt, y, Qp + o, Qn + o, Fp + (size_t)b * N, Fn + (size_t)b * N, N);
            memcpy(y, nxt, sizeof(float) * N);
        }
        free(nxt);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    (void)threads;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
