/* oracle/ref_converge.c -- TEST INFRASTRUCTURE (never linked by the product).
 * The reference's converge-mode solve with an update cap, driven through the
 * reference's OWN functions from _ref/libpqp_ref.so (PQP_CPU.c compiled
 * unmodified): solveQuadraticDual's setup (PQP_CPU.c:696-710) and its loop
 * `while (!terminate(...)) { updateY2; copyMatrix; h++ }` (:718-740), plus one
 * test before each update: after `cap` updates the solve stops and returns -h
 * (the bench's horizon leg caps at 999 updates; one perturbed H = 2 problem
 * never meets the reference's gap test, so the uncapped solveQuadraticDual
 * would not return).  For a problem that stops within the cap the calls, their
 * order and every floating-point operation are the reference's, so Y, U and h
 * equal what solveQuadraticDual gives.  Only the control loop is restated. */
#include <stdlib.h>

float *newMatrix(int n, int m);
void initMat(float *mat, float val, int N);
void copyMatrix(float *output, float *mat, int a, int b);
void matrixPos(float *out, float *mat, int a, int b);
void matrixNeg(float *out, float *mat, int a, int b);
void computeTheta(float *theta, float *Qd, int N);
void computeQdp_theta(float *out, float *Qd, float *theta, int N);
void computeQdn_theta(float *out, float *Qd, float *theta, int N);
void updateY2(float *Y_next, float *Y, float *Qdp_theta, float *Qdn_theta, float *Fd, float *Fdp, float *Fdn, int N);
int terminate(float *Y, float *Qd, float *Fd, float *Md, float *U, float *Qp, float *Qp_inv, float *Fp, float *Mp,
              float *Gp, float *Kp, int N, int M);

long ref_converge_solve(float *Y, float *Qd, float *Fd, float *Md, float *U, float *Qp, float *Qp_inv, float *Fp,
                        float *Mp, float *Gp, float *Kp, int N, int M, long cap)
{
    float *theta = newMatrix(N, N), *Qdp_theta = newMatrix(N, N), *Qdn_theta = newMatrix(N, N);
    float *Y_next = newMatrix(N, 1), *Fdn = newMatrix(N, 1), *Fdp = newMatrix(N, 1);
    matrixPos(Fdp, Fd, N, 1);
    matrixNeg(Fdn, Fd, N, 1);
    computeTheta(theta, Qd, N);
    computeQdp_theta(Qdp_theta, Qd, theta, N);
    computeQdn_theta(Qdn_theta, Qd, theta, N);
    initMat(Y, 1000.0, N);
    long h = 1;
    while (!terminate(Y, Qd, Fd, Md, U, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M)) {
        if (h - 1 >= cap) {
            h = -h;
            break;
        }
        updateY2(Y_next, Y, Qdp_theta, Qdn_theta, Fd, Fdp, Fdn, N);
        copyMatrix(Y, Y_next, N, 1);
        h++;
    }
    free(theta); free(Qdp_theta); free(Qdn_theta); free(Y_next); free(Fdn); free(Fdp);
    return h;
}
