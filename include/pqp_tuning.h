/*
 * include/pqp_tuning.h -- tuning/diagnostic entry points of libpqp.  Not part
 * of the drop-in surface; used by the tests (every variant must give the same
 * bits) and by scripts/ to A/B kernel variants and trace the persistent
 * launches on the device at hand.
 */
#ifndef PQP_TUNING_H
#define PQP_TUNING_H
#ifdef __cplusplus
extern "C" {
#endif

/* Select kernel variants (every variant is bit-identical; the tests run the
 * parity cases through each).  Bit 0x100: solve N, M <= 32 problems with the
 * LDS-staged k_solve_small instead of k_solve_tiny.  Bit 0x200: fixed-mode
 * solves of large single problems on one workgroup (k_solve_single) instead
 * of the multi-workgroup split-matrix update.  Bit 0x400: fixed mode of
 * N <= 32 problems on k_solve_tiny instead of the one-wave k_fixed_tiny.  Bits 12-13: k_split_update
 * load stage depth (0: 16 packets, 1: 8, 2: 24).  Bits 14-16: the kernel
 * behind pqp_rowblock_update and large fixed-mode solves (0: default =
 * k_split_relay with 8 waves x 16-packet segments, 1: streaming
 * k_split_update, 2: relay 4 x 64, 3: relay 8 x 32, 4: relay 16 x 16,
 * 5: relay 8 x 16).  Bits 17-19: row sides per workgroup of blocks built
 * afterwards (0: auto, about one workgroup per CU; 1: 8, 2: 16, 3: 32,
 * 4: 64).  Returns the previous value. */
int pqp_tune_set_variant(int variant);

/* Fixed mode of one problem with n_dual <= 1024 runs as ONE persistent launch
 * (pqp_persist.hip) unless off = 1, which sends it through the hipGraph-replayed
 * relay update (one launch per update).  Returns the previous setting. */
int pqp_tune_persist(int off);

/* Fixed mode of N <= 32 problems (k_fixed_tiny): launches of at most b
 * problems keep the iterate in registers (y_k on lane 2k, broadcast by
 * v_readlane), larger ones exchange it through LDS (fewer VALU instructions
 * when problems share SIMDs).  Default 1024.  Returns the previous value. */
int pqp_tune_fixed_rl_max_b(int b);

/* The relay update of one large problem (fixed mode above n_dual 1024, the
 * converge graph chain) and of a row block (pqp_rowblock_*) streams Qd itself
 * (k_lean_relay: 4 B per entry, the split terms formed in registers) instead
 * of the stored split matrices (8 B) when the block's rows x n_dual >= n^2;
 * n <= 0 never.  Default 4096.  Affects problems and row blocks built
 * afterwards.  Returns the previous value. */
int pqp_tune_lean_min_n(int n);

/* Budget, in polls, of every wave-to-wave hand-off wait in the relay kernels
 * (k_split_relay, k_lean_relay, k_gemv_relay); 0 restores the default (2^20).
 * A negative budget expires every wait, so that a test can see the error path:
 * the solve / pqp_rowblock_check then returns PQP_ERR_HIP.  Applies to launches
 * (and graphs) made afterwards.  Returns the previous value. */
int pqp_tune_relay_spin_max(int polls);


/* Setup products (convertToDual and the other matrixMultiply drop-ins) with
 * both output dimensions >= 32 run LDS-tiled (k_matmul_tiled); off != 0 sends
 * every product through the one-thread-per-output k_matmul_seq instead (A/B
 * timing; both are bit-identical to PQP_CPU.c).  Returns the previous value. */
int pqp_tune_matmul_tiled(int off);

/* Error-path tests of the persistent launches: workgroup `wg` of every
 * persistent launch (k_split_persist, k_converge_persist) returns at once, as
 * if it were never resident, so the other workgroups' waits expire (2 s) and
 * the solve falls back to the graph-replayed relay / chain path, from the
 * reference's start (pqp_tune_last_path tells which path ran and counts the
 * fallbacks).  wg < 0 turns it off.  Returns the previous value. */
int pqp_tune_persist_stall(int wg);
/* Workgroups of the persistent converge launch for (N, M) (0: not used). */
int pqp_tune_converge_grid(int N, int M);

/* Batched converge mode (pqp_batch_solve: one workgroup per problem, operands
 * from global memory).  By default, for problems whose Qd is bit-symmetric,
 * terminate()'s Y'Qd rides in the update's pass over Qd after a feasible
 * terminate() (the update runs first, speculatively); opts bit 0 turns that
 * off.  bit 1: the unprepared pqp_batch_solve makes transposed copies of Gp
 * and Qp_inv per call (pqp_batch_prepare makes them once when asked); bit 2:
 * 4-byte loads only (the 8/16-byte load forms, used by default when N and M
 * are multiples of 4 and the arrays 16-byte aligned, are turned off); bit 3:
 * the solver built for four workgroups per CU; bit 4: checkFeas sums every
 * row (by default, with the transposes, it sums the first 256 rows and stops
 * there when one is over its bound -- terminate() returns 0 either way).
 * Every setting is bit-identical.  Returns the previous value. */
int pqp_tune_batch_converge(int opts);

/* Batched Gauss_Jordan (n <= 1024): the blocked kernel (one read and write of
 * the augmented matrix per 16 or 8 pivots) by default; off != 0 takes the
 * one-pivot-per-sweep kernel (A/B timing; both bit-identical to PQP_CPU.c).
 * Returns the previous value. */
int pqp_tune_gj_blocked(int off);

/* The persistent single-problem launches (fixed mode: k_split_persist; converge
 * mode: k_converge_persist) need all their workgroups resident at once.  Before
 * launching, the library checks occupancy x CUs against the grid and otherwise
 * takes the graph-replayed relay path; a launch whose wait still expires
 * (CUs held by other work) is re-run on that path.  `cus` > 0 makes the check
 * assume that many CUs (1 forces the does-not-fit branch in tests); 0 restores
 * the device's count.  Returns the previous value. */
int pqp_tune_persist_fit_cus(int cus);

/* Which solver the last pqp_problem_solve / drop-in solve of one problem ran:
 * 1 fixed-mode persistent launch, 2 fixed-mode graph-replayed relay, 3 converge
 * persistent launch, 4 converge graph chain (pqp_wide.hip), 5 one-workgroup /
 * one-wave solvers; 0 none yet.  *fallbacks (if not NULL) receives how many
 * persistent launches fell back to the relay / graph path so far. */
int pqp_tune_last_path(long long *fallbacks);

/* Converge mode of one problem with n_dual, M <= 1024 (other than the N, M <= 32
 * problems of the one-wave solver) runs as ONE persistent pipelined launch
 * (pqp_converge.hip: terminate(Y_u) beside the update to Y_{u+1}) unless
 * off = 1, which restores the launch-per-step routing (one-workgroup solvers
 * below pqp_tune_wide_min_n, the graph-replayed chain of pqp_wide.hip above).
 * Returns the previous setting. */
int pqp_tune_converge_persist(int off);

/* Iterates one persistent converge launch decides at most before the host
 * relaunches from the iterate it left (default 65536; <= 0 restores it).
 * Returns the previous value. */
int pqp_tune_converge_chunk(int iterates);

/* Timeline of the persistent converge launch: for the first `iterates`
 * iterates of each launch, workgroup 0 of every role writes s_memrealtime
 * (100 MHz, chip-wide) marks into d_trace[iterate][29][4] (role * 6 + wave
 * for UPD, T1, T2, T3; 24 + wave for DEC, wave 0 deciding, waves 1-4 summing
 * the dots): iterate start, inputs staged, turn
 * (running sums received; DEC: sum done), done; the same marks in shader
 * clocks (s_memtime) follow at d_trace[iterates * 29 * 4] (buffer of
 * 2 * iterates * 29 * 4 words).  iterates = 0 turns it off. */
int pqp_tune_converge_trace(void* d_trace, int iterates);

/* Converge-mode solves of N, M <= 32 problems run one wave per problem
 * (k_solve_wave) when a launch holds at least b problems, else four waves per
 * problem (k_solve_tiny).  Returns the previous threshold. */
int pqp_tune_wave_min_b(int b);

/* k_solve_wave launches of at most b problems use its software-pipelined form
 * (the next iterate's pass beside this iterate's terminate()): shorter
 * iterations, more registers.  Returns the previous threshold. */
int pqp_tune_wave_pipe_max_b(int b);

/* Timeline of the persistent launch's workgroup 0 (s_memtime shader clocks):
 * for the first `updates` updates, per update u and wave w, the four words
 * d_trace[(u * waves + w) * 4 + e] = {sweep start, y staged, running sums
 * received, chain done}; then, from d_trace[updates * waves * 4], per update
 * and wave 1..waves-1, 8 words: s_memtime before each seventh of the wave's
 * add chain and after it.  The buffer holds updates * waves * 12 words.
 * updates = 0 turns the trace off. */
int pqp_tune_persist_trace(void *d_trace, int updates);

/* Converge-mode solves of problems with n_dual >= n that the persistent
 * launch above does not take (n_dual or M > 1024, or pqp_tune_converge_persist(1))
 * run over many workgroups (terminate() as multi-workgroup mat-vecs + the
 * relay update, replayed from a hipGraph) instead of one persistent workgroup;
 * n <= 0 sends every size there, LDS-sized problems included (where they fit,
 * those go on to the persistent launch).  Default 384.  Returns the previous
 * value. */
int pqp_tune_wide_min_n(int n);

/* Variants of that path: bit 0 launches the update on a forked graph branch
 * beside terminate() instead of after it; bit 1 uses 64-value k-segments in
 * the mat-vecs (default 32).  Returns the previous value. */
int pqp_tune_wide_flags(int flags);

/* The first n values of glibc's unseeded rand() as reproduced by the
 * testing/ reader (for checking the emulation against the C library). */
int pqp_tune_glibc_rand(int n, int *out);

#ifdef __cplusplus
}
#endif
#endif
