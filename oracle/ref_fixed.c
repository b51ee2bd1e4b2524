/* oracle/ref_fixed.c -- TEST / BASELINE INFRASTRUCTURE (never linked by the
 * product).  The reference's fixed-iteration solve, driven through the
 * reference's OWN functions from _ref/libpqp_ref.so (PQP_CPU.c compiled
 * unmodified): the setup of solveQuadraticDual (PQP_CPU.c:696-710) and the
 * testing harness's loop `while (h < NUM_ITER) { updateY2; copyMatrix; h++ }`
 * (testing/CPU version/PQP_CPU_test.c:714-744; 999 updates for NUM_ITER 1000),
 * timed with clock_gettime like the survey asks.  Only the
 * control loop is restated here; every floating-point operation is the
 * reference's. */
#include <stdlib.h>
#include <time.h>

float *newMatrix(int n, int m);
void initMat(float *mat, float val, int N);
void copyMatrix(float *output, float *mat, int a, int b);
void matrixPos(float *out, float *mat, int a, int b);
void matrixNeg(float *out, float *mat, int a, int b);
void computeTheta(float *theta, float *Qd, int N);
void computeQdp_theta(float *out, float *Qd, float *theta, int N);
void computeQdn_theta(float *out, float *Qd, float *theta, int N);
void updateY2(float *Y_next, float *Y, float *Qdp_theta, float *Qdn_theta, float *Fd, float *Fdp, float *Fdn, int N);

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* Y (N, out) after num_iter - 1 updates from Y = 1000.  Returns the seconds of
 * the whole call (setup + loop, what the harness's `time` measured); *loop_s
 * gets the update loop alone. */
double ref_fixed_solve(float *Y, float *Qd, float *Fd, int N, long num_iter, double *loop_s)
{
    const double t0 = now();
    float *theta = newMatrix(N, N), *Qdp_theta = newMatrix(N, N), *Qdn_theta = newMatrix(N, N);
    float *Y_next = newMatrix(N, 1), *Fdn = newMatrix(N, 1), *Fdp = newMatrix(N, 1);
    matrixPos(Fdp, Fd, N, 1);
    matrixNeg(Fdn, Fd, N, 1);
    computeTheta(theta, Qd, N);
    computeQdp_theta(Qdp_theta, Qd, theta, N);
    computeQdn_theta(Qdn_theta, Qd, theta, N);
    initMat(Y, 1000.0f, N);
    const double t1 = now();
    for (long h = 1; h < num_iter; ++h) {
        updateY2(Y_next, Y, Qdp_theta, Qdn_theta, Fd, Fdp, Fdn, N);
        copyMatrix(Y, Y_next, N, 1);
    }
    const double t2 = now();
    free(theta); free(Qdp_theta); free(Qdn_theta); free(Y_next); free(Fdn); free(Fdp);
    if (loop_s) *loop_s = t2 - t1;
    return t2 - t0;
}
