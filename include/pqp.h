/*
 * include/pqp.h -- C ABI of libpqp (pqp-for-mpc_amd), the MI355X-native
 * drop-in for the PQP dual-update hot path of yashsoni501/PQP-for-MPC.
 *
 * Two layers:
 *
 *  1. Drop-in entry points.  Same names, argument order and meaning as the
 *     reference's C functions (PQP_CPU.c), on caller-owned HOST buffers of
 *     row-major fp32.  They run on the GPU (HIP, gfx950) and return results
 *     identical to PQP_CPU.c.  Like the reference they have no status return;
 *     on a HIP/allocation failure they print a message and exit(EXIT_FAILURE)
 *     (the reference's own failure behaviour, PQP_GPU_optimized.cu:83-89).
 *
 *  2. pqp_* entry points.  Status-returning (PQP_OK or a negative PQP_ERR_*;
 *     pqp_last_error() explains), explicit sizes, and the batched device API
 *     that works on DEVICE pointers on the caller's hipStream_t (passed as
 *     void*).  Nothing here takes framework types.
 *
 * Device layout of a batch of B dual problems of size N:
 *   QdT   [B][N][ldq]  Qd stored column-major per instance: element (i,k)
 *                      of Qd is QdT[b*qstride + k*ldq + i]; ldq >= N, ldq % 4 == 0
 *   theta, Fd, Y       [B][ldv] fp32 vectors, ldv >= N
 */
#ifndef PQP_H
#define PQP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PQP_OK 0
#define PQP_ERR_ARG (-1)           /* bad size / pointer / layout                 */
#define PQP_ERR_HIP (-2)           /* a HIP runtime call or kernel launch failed  */
#define PQP_ERR_ALLOC (-3)         /* device allocation failed                    */
#define PQP_ERR_IO (-4)            /* input file missing or short                 */
#define PQP_ERR_NOT_CONVERGED (-5) /* converge mode hit its update cap            */
#define PQP_ERR_NO_DEVICE (-6)     /* no gfx950 device visible                    */
#define PQP_ERR_NEEDS_QDT (-7)     /* pqp_batch_prepare: pass d_QdT (see there)   */

/* Solve modes of pqp_solve_dual. */
#define PQP_MODE_CONVERGE 0 /* while(!terminate(Y)) update  (PQP_CPU.c:718)            */
#define PQP_MODE_FIXED 1    /* while(h < num_iter) update   (testing/ harness, no terminate) */

const char *pqp_last_error(void);
int pqp_version(void);

/* ======================================================================
 * 1. Drop-in entry points (reference signatures, host pointers)
 * ==================================================================== */

/* PQP_CPU.c:694-750.  Runs the whole solve on the GPU in one persistent
 * workgroup (setup, terminate() before every update, updateY2) and prints
 * "Printing number of iterations = %ld\n" exactly as the reference does.
 * Y (N) and U (M) are outputs; the rest are inputs. */
void solveQuadraticDual(float *Y, float *Qd, float *Fd, float *Md, float *U, float *Qp, float *Qp_inv,
                        float *Fp, float *Mp, float *Gp, float *Kp, int N, int M);

/* PQP_CPU.c:603-618.  One multiplicative update from the stored split
 * matrices Qdp_theta = max(0,Qd)+Theta, Qdn_theta = max(0,-Qd)+Theta and
 * Fdp = max(0,Fd), Fdn = max(0,-Fd).  Fd is accepted and unused, as in the
 * reference. */
void updateY2(float *Y_next, float *Y, float *Qdp_theta, float *Qdn_theta, float *Fd, float *Fdp,
              float *Fdn, int N);

/* PQP_CPU.c:673-687.  Writes U = -Qp_inv(Gp'Y + Fp) and returns 1 when the
 * feasibility and duality-gap tests all pass. */
int terminate(float *Y, float *Qd, float *Fd, float *Md, float *U, float *Qp, float *Qp_inv, float *Fp,
              float *Mp, float *Gp, float *Kp, int N, int M);

/* PQP_CPU.c:489-498: Qd = (Gp Qp_inv) Gp', Fd = (Gp Qp_inv) Fp + Kp,
 * Md = (Fp' Qp_inv) Fp - Mp.
 * NaN operands: where an operand is NaN, the output is NaN wherever the
 * reference's is, but the NaN's sign and payload may differ (the host's and the
 * GPU's multiply carry a NaN operand's bits differently); every non-NaN output
 * is bit-identical.  DESIGN.md section 2. */
void convertToDual(float *Qd, float *Fd, float *Md, float *Qp_inv, float *Gp, float *Kp, float *Fp,
                   float *Mp, int N, int M);

/* PQP_CPU.c:352-360: U = -Qp_inv (Gp'Y + Fp). */
void computeUfromY(float *U, float *Y, float *Fp, float *Gp, float *Qp_inv, int N, int M);

/* PQP_CPU.c:648-666: J = 0.5 (Z'Q) Z + F'Z + M[0]/2. */
float computeCost(float *Z, float *Q, float *F, float *M, int N);

/* PQP_CPU.c:632-641: 1 iff Gp U <= Kp + max(1e-6 Kp, 1e-6) element-wise. */
int checkFeas(float *U, float *Gp, float *Kp, int N, int M);

/* PQP_CPU.c:503-519: theta (N x N, caller-zeroed as in the reference) gets
 * theta[i][i] = max(sum_j max(0,-Qd[i][j]), 5); other entries untouched. */
void computeTheta(float *theta, float *Qd, int N);

/* PQP_CPU.c:84-147: output[a x c] = op(mat1)[a x b] * op(mat2)[b x c];
 * output may alias an input.
 * NaN operands: where an operand is NaN, the output is NaN wherever the
 * reference's is, but the NaN's sign and payload may differ (the host's and the
 * GPU's multiply carry a NaN operand's bits differently); every non-NaN output
 * is bit-identical.  DESIGN.md section 2. */
void matrixMultiply(float *output, float *mat1, int transpose1, float *mat2, int transpose2, int a, int b,
                    int c);

/* PQP_CPU.c:251-326: res = inverse(A) by the reference's Gauss-Jordan
 * (one bubble pass on column 0, no pivoting). */
void Gauss_Jordan(float *A, float *res, int N);

/* PQP_CPU.c:373-382 / 395-428, with the reference's compile-time problem
 * dimensions (pHorizon=1, nState=29, nInput=7, nDis=1; PQP_CPU.c:13-17). */
void computeFp(float *Fp, float *Fp1, float *Fp2, float *Fp3, float *D, float *x);
void computeMp(float *Mp, float *Mp1, float *Mp2, float *Mp3, float *Mp4, float *Mp5, float *Mp6, float *D,
               float *x);

/* PQP_CPU.c:757-930: reads ./example/{Qp_inv,Fp1,Fp2,Fp3,Mp1..Mp6,Gp,Kp,Z,Theta,D,x}.txt
 * relative to the current directory, with the reference's transposed
 * layout and compile-time dimensions.  (Host I/O; no GPU work.) */
void input(float *qp_inv, float *Fp1, float *Fp2, float *Fp3, float *Mp1, float *Mp2, float *Mp3, float *Mp4,
           float *Mp5, float *Mp6, float *Gp, float *Kp, float *x, float *D, float *theta, float *Z);

/* ======================================================================
 * 2a. Status-returning host-pointer API
 * ==================================================================== */

/* solveQuadraticDual without the printf and with explicit control:
 *   mode PQP_MODE_CONVERGE: iterate until terminate() passes; gives up with
 *     PQP_ERR_NOT_CONVERGED after max_updates updates (<= 0: no cap).
 *   mode PQP_MODE_FIXED: num_iter-1 updates, no terminate (testing/ harness).
 * On return *h_out is the reference's printed h (updates + 1), Y and U hold
 * the final iterate, Jp_out and Jd_out get the costs of the last terminate() that
 * got past the feasibility test (NaN if none).  Any of the out pointers
 * except Y may be NULL. */
int pqp_solve_dual(const float *Qd, const float *Fd, const float *Md, const float *Qp, const float *Qp_inv,
                   const float *Fp, const float *Mp, const float *Gp, const float *Kp, int N, int M, int mode,
                   long long num_iter, long long max_updates, float *Y, float *U, long long *h_out,
                   float *Jp_out, float *Jd_out);

/* A dual problem resident in HBM: upload and prepare once, then solve any
 * number of times (each solve restarts from Y = 1000).  Same semantics and
 * outputs as pqp_solve_dual, which is create + solve + destroy.  Problems
 * that fit LDS run in one persistent workgroup; larger ones (N up to 38016)
 * run over many workgroups, each solve replaying a captured hipGraph.  The
 * terminate() drop-in also needs the one-workgroup solver, which limits it
 * to 12N + 12M bytes <= 150 KiB. */
typedef struct pqp_problem pqp_problem;
int pqp_problem_create(const float *Qd, const float *Fd, const float *Md, const float *Qp, const float *Qp_inv,
                       const float *Fp, const float *Mp, const float *Gp, const float *Kp, int N, int M,
                       pqp_problem **out);
/* The same on an explicit device (-1: the calling thread's current one) and
 * stream (a hipStream_t of that device; NULL: the handle creates and owns
 * one).  A handle is bound to its device and stream: every call on it runs
 * there, whatever device the calling thread has current, and restores the
 * caller's device before returning.  Calls on one handle are serialized by a
 * lock of that handle; different handles (one host thread per GPU, or several
 * per GPU) run concurrently -- the reference's solver keeps no globals
 * (PQP_CPU.c:694) and neither does this one. */
int pqp_problem_create_on(int device, void *stream, const float *Qd, const float *Fd, const float *Md,
                          const float *Qp, const float *Qp_inv, const float *Fp, const float *Mp, const float *Gp,
                          const float *Kp, int N, int M, pqp_problem **out);
/* The device a handle is bound to. */
int pqp_problem_device(const pqp_problem *p);
int pqp_problem_solve(pqp_problem *p, int mode, long long num_iter, long long max_updates, float *Y, float *U,
                      long long *h_out, float *Jp_out, float *Jd_out);
int pqp_problem_destroy(pqp_problem *p);

/* One update on host buffers from Qd/theta-diag/Fd (the fused form used by
 * the solver: Qd+-, Theta and Fd+- derived on the fly). */
int pqp_update_host(const float *Qd, const float *theta_diag, const float *Fd, const float *Y, float *Y_next,
                    int N);

/* Bundled-example reader with explicit dimensions: m = nInput*pHorizon,
 * nd = nDis*pHorizon, ns = nState, N = 4m.  Files are read from `dir`. */
int pqp_read_example(const char *dir, int m, int nd, int ns, float *Qp_inv, float *Fp1, float *Fp2,
                     float *Fp3, float *Mp1, float *Mp2, float *Mp3, float *Mp4, float *Mp5, float *Mp6,
                     float *Gp, float *Kp, float *x, float *D);

/* The testing/ sample-test format ("testing/sample test/test*.txt"; reader at
 * testing/GPU unoptimized version/PQP_GPU_unoptimized.cu:751-794 and
 * testing/CPU version/PQP_CPU_test.c:936-978): header "M N", M diagonal
 * entries of Qp_inv, M of Fp, Mp, N of Kp, N x M integers for Gp mapped by C's
 * `v % 3` (0 -> 0, 2 -> -1, otherwise +1, so a file -1 becomes +1).  With
 * glibc_kp != 0 the file's Kp is replaced, as the harness does, by
 * fabs(10.0*rand()/RAND_MAX) from glibc's unseeded rand() sequence.
 * Call with NULL arrays to get (*M_out, *N_out) first; then call again with the
 * arrays (Qp_inv is M x M dense) and *M_out / *N_out still holding those
 * dimensions: a file whose header no longer matches them gives PQP_ERR_IO and
 * nothing is written.  Headers beyond M, N <= 65536 (or N*M + M*M > 2^30) are
 * rejected with PQP_ERR_IO.  (Host I/O; no GPU work.) */
int pqp_read_testfile(const char *path, int glibc_kp, int *M_out, int *N_out, float *Qp_inv, float *Fp, float *Mp,
                      float *Gp, float *Kp);

/* main() of PQP_CPU.c:935-1013 on the GPU: read `dir`, build the dual, solve,
 * recompute U, print the reference's stdout to `out` (a FILE*; NULL = stdout). */
int pqp_run_example(const char *dir, void *out);

/* ======================================================================
 * 2b. Batched device API (device pointers, caller's stream; async)
 * ==================================================================== */

/* Synthetic dual problems: instance b of the batch is problem
 * number inst0+b of `seed`; primal Qp_inv = diag(0.1+u), Gp in {-1,0,1},
 * Kp = 10u, Fp = 20u-10, Mp = 1, converted to the dual with
 * convertToDual's exact arithmetic.  Writes QdT (column-major, padded rows
 * zeroed), Fd, Md (may be NULL) and theta. */
int pqp_batch_generate(uint32_t seed, long long inst0, int B, int N, int M, float *d_QdT, int ldq,
                       long long qstride, float *d_Fd, float *d_Md, float *d_theta, int ldv, void *stream);

/* The primal problems behind pqp_batch_generate's duals, in the layout of
 * 2c below: Qp_inv [B][M*M] (diagonal), Gp [B][N*M], Kp [B][N], Fp [B][M],
 * Mp [B] (= 1).  With pqp_batch_gauss_jordan and pqp_batch_convert_to_dual
 * this gives complete problems for converge-mode solves. */
int pqp_batch_synth_primal(uint32_t seed, long long inst0, int B, int N, int M, float *d_Qp_inv, float *d_Gp,
                           float *d_Kp, float *d_Fp, float *d_Mp, void *stream);

/* Pack B row-major N x N Qd matrices (device, contiguous) into QdT layout. */
int pqp_batch_pack(int B, int N, const float *d_Qd, float *d_QdT, int ldq, long long qstride, void *stream);

/* theta[b][i] = max(sum_j max(0,-Qd_b[i][j]), 5)  (computeTheta). */
int pqp_batch_theta(int B, int N, const float *d_QdT, int ldq, long long qstride, float *d_theta, int ldv,
                    void *stream);

/* One updateY2 for every instance: Y_next = num/den * Y. */
int pqp_batch_update(int B, int N, const float *d_QdT, int ldq, long long qstride, const float *d_theta,
                     const float *d_Fd, int ldv, const float *d_Y, float *d_Ynext, void *stream);

/* `updates` consecutive updateY2 per instance in ONE launch, the iterate
 * resident in LDS (fixed-iteration mode).  d_Y0 == NULL starts from the
 * reference's Y = 1000.  Requires 8*ldq bytes of LDS (ldq <= 20480). */
int pqp_batch_iterate(int B, int N, const float *d_QdT, int ldq, long long qstride, const float *d_theta,
                      const float *d_Fd, int ldv, const float *d_Y0, float *d_Y, int updates, void *stream);

/* ----------------------------------------------------------------------
 * 2c. Batched small problems: many independent MPC problems (batched
 * horizons / states), one workgroup each.  Every array holds B problems back
 * to back in the reference's row-major layout (e.g. Qd is [B][N*N], Kp is
 * [B][N], Md is [B]).  Synchronous: returns when every problem has finished.
 * -------------------------------------------------------------------- */

/* Gauss_Jordan (PQP_CPU.c:251-326) on B n x n matrices. */
int pqp_batch_gauss_jordan(int B, int n, const float *d_A, float *d_res, void *stream);

/* convertToDual (PQP_CPU.c:489-498) on B primal problems (NaN operands: as
 * convertToDual above). */
int pqp_batch_convert_to_dual(int B, int N, int M, const float *d_Qp_inv, const float *d_Gp, const float *d_Kp,
                              const float *d_Fp, const float *d_Mp, float *d_Qd, float *d_Fd, float *d_Md,
                              void *stream);

/* pqp_batch_convert_to_dual keeps ONE grow-only device workspace per device
 * (4*(B*N*M + B*M) bytes at its largest call: 128 MiB at B = 64, N = 1024,
 * M = 512), shared by every calling thread (calls on one device take turns
 * while they use it).  This frees every device's workspace; the next call
 * allocates again; a setup call in progress finishes first. */
int pqp_release_workspaces(void);

/* computeFp / computeMp (PQP_CPU.c:373-428) for B (D, x) pairs of one plant:
 * m = nInput*pHorizon, nd = nDis*pHorizon, ns = nState.  The plant matrices
 * (Fp1 [m*nd], Fp2 [m*ns], Fp3 [m], Mp1 [ns*ns], Mp2 [nd*ns], Mp3 [nd*nd],
 * Mp4 [ns], Mp5 [nd], Mp6 [1]) are shared; D is [B][nd], x is [B][ns]. */
int pqp_batch_compute_fp(int B, int m, int nd, int ns, const float *d_Fp1, const float *d_Fp2, const float *d_Fp3,
                         const float *d_D, const float *d_x, float *d_Fp, void *stream);
int pqp_batch_compute_mp(int B, int nd, int ns, const float *d_Mp1, const float *d_Mp2, const float *d_Mp3,
                         const float *d_Mp4, const float *d_Mp5, const float *d_Mp6, const float *d_D,
                         const float *d_x, float *d_Mp, void *stream);

/* solveQuadraticDual for B problems at once (converge or fixed mode, as
 * pqp_solve_dual).  Outputs: Y [B][N], U [B][M] (converge mode), h [B]
 * (int64, the reference's printed h) and status [B] (1 converged / done,
 * 2 hit max_updates); h and status may be NULL. */
int pqp_batch_solve(int B, int N, int M, const float *d_Qd, const float *d_Fd, const float *d_Md, const float *d_Qp,
                    const float *d_Qp_inv, const float *d_Fp, const float *d_Mp, const float *d_Gp, const float *d_Kp,
                    int mode, long long num_iter, long long max_updates, float *d_Y, float *d_U, long long *d_h,
                    int *d_status, void *stream);

/* Which batched solver pqp_batch_solve uses for (N, M): 0 one wave or one small
 * workgroup per problem (N, M <= 32), 3 one workgroup per problem with each
 * matrix held in LDS once (k_solve_mid: mid-size, about N <= 165 at M = N/4),
 * 1 the problem staged in LDS with its split copies (k_solve_small; only with
 * the mid_off knob), 2 one workgroup per problem from HBM (uses
 * pqp_batch_prepare's data: k_solve_pipe, which reads every matrix once per
 * iteration, in converge mode when d_QinvT is given, N, M are multiples of 4
 * and M >= N/3; k_solve_single otherwise), or PQP_ERR_ARG when (N, M) exceeds every
 * solver's LDS budget. */
int pqp_batch_solve_path(int N, int M);

/* Path 2's converge-mode kernel for (N, M), from the shape alone: 1 when
 * pqp_batch_solve_prepared (given d_QinvT and 16-byte-aligned arrays) runs
 * k_solve_pipe, which never reads d_GpT -- so a caller need not allocate it
 * (B*N*M floats) -- and 0 when it runs k_solve_single (d_GpT, when given, makes
 * its walks of Gp coalesced); 0 as well for the other paths.  Tuning knobs
 * (pipe_off, pipe_force) move the answer. */
int pqp_batch_solve_kernel(int N, int M);

/* pqp_batch_solve in two steps, so that what depends only on the problems is
 * computed once per batch instead of once per call (path 2 above):
 *   pqp_batch_prepare: per-problem bit-symmetry flags of Qd into d_sym [B]
 *     (int), Theta (computeTheta, PQP_CPU.c:503-519) into d_theta [B][N], and
 *     *all_sym_out = 1 when every Qd is bit-symmetric and N % 4 == 0 (Qd is
 *     then its own column-major copy).  Otherwise the column-major copy goes to
 *     d_QdT [B][N][round4(N)], which must then be given: with d_QdT NULL the
 *     call returns PQP_ERR_NEEDS_QDT with *all_sym_out = 0 (d_sym filled) --
 *     call again with it.  Optional d_GpT [B][M][N] and d_QinvT [B][M][M] (with
 *     d_Gp / d_Qp_inv) receive transposed copies: terminate()'s row walks of
 *     Gp and Qp_inv (PQP_CPU.c:357, :635) then read coalesced.  k_solve_pipe
 *     needs d_QinvT only (it walks Gp's rows from LDS tiles); d_GpT serves
 *     k_solve_single.
 *   pqp_batch_solve_prepared: pqp_batch_solve on those (d_QdT NULL when
 *     *all_sym_out was 1; d_GpT / d_QinvT NULL when not prepared).  The
 *     prepared data stay valid until Qd (or Gp, Qp_inv) change.
 * Paths 0 and 1 need none of it (NULLs are fine there). */
int pqp_batch_prepare(int B, int N, int M, const float *d_Qd, const float *d_Gp, const float *d_Qp_inv, float *d_QdT,
                      float *d_theta, int *d_sym, float *d_GpT, float *d_QinvT, int *all_sym_out, void *stream);
int pqp_batch_solve_prepared(int B, int N, int M, const float *d_Qd, const float *d_QdT, const float *d_theta,
                             const int *d_sym, const float *d_GpT, const float *d_QinvT, const float *d_Fd,
                             const float *d_Md, const float *d_Qp, const float *d_Qp_inv, const float *d_Fp,
                             const float *d_Mp, const float *d_Gp, const float *d_Kp, int mode, long long num_iter,
                             long long max_updates, float *d_Y, float *d_U, long long *d_h, int *d_status,
                             void *stream);

/* ----------------------------------------------------------------------
 * 2d. Row blocks of one large problem (a single problem
 * row-sharded across GPUs).  A pqp_rowblock holds rows [row0, row0+rows) of
 * updateY2's stored split matrices (PQP_CPU.c:524-537 Qdp_theta/Qdn_theta
 * rows, :703-704 Fdp/Fdn) on the current device.  One step reads the FULL
 * iterate Y (N, device) and writes the block's rows of Y_next
 * (PQP_CPU.c:603-618 restricted to those rows); between steps the caller
 * assembles Y_next from every block (e.g. an RCCL all-gather).  Every row's
 * sums still run over k = 0..N-1 in order, so the assembled Y_next is
 * bit-identical to updateY2's whatever the partition.  N <= 38016 (the full
 * y is staged in LDS).
 * -------------------------------------------------------------------- */
typedef struct pqp_rowblock pqp_rowblock;

/* d_Qd_rows: the block's rows of Qd, row-major with leading dimension ld >= N
 * (a pointer into a full row-major Qd works); d_Fd: the full Fd (N).  Theta_ii
 * of the block's rows is computed from them (computeTheta, PQP_CPU.c:503-519).
 * The inputs may be freed once this returns.  rows == 0 gives an empty block
 * whose update is a no-op. */
int pqp_rowblock_create(const float *d_Qd_rows, int ld, const float *d_Fd, int N, int row0, int rows, void *stream,
                        pqp_rowblock **out);
/* d_Y_rows[i] = updateY2(Y)[row0 + i] for i < rows.  d_Y must hold N floats
 * (more is allowed and ignored).  Async on `stream`. */
int pqp_rowblock_update(pqp_rowblock *b, const float *d_Y, float *d_Y_rows, void *stream);
/* Synchronizes `stream` and reports whether any pqp_rowblock_update of this
 * block since the last check hit an expired wait inside the kernel (a
 * workgroup's wave-to-wave hand-off that never arrived): PQP_ERR_HIP when one
 * did -- the rows it wrote are then not valid -- else PQP_OK.  The check clears
 * the block's error word.  No reference counterpart (the CPU loop cannot
 * fail); call it at the end of a run of updates. */
int pqp_rowblock_check(pqp_rowblock *b, void *stream);
int pqp_rowblock_destroy(pqp_rowblock *b);

/* Rows [row0, row0+rows) of synthetic problem `inst` of `seed` (the
 * generator of pqp_batch_generate), row-major with leading dimension ld >= N
 * (columns N..ld-1 zeroed), so that a rank can build its row block without
 * materialising the whole N x N matrix.  d_Fd (N) and d_Md (1) receive the
 * full Fd / Md when not NULL. */
int pqp_synth_rows(uint32_t seed, long long inst, int N, int M, int row0, int rows, float *d_Qd_rows, int ld,
                   float *d_Fd, float *d_Md, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PQP_H */
