/*
 * include/pqp_tuning.h -- tuning and diagnostic entry points of libpqp.  Not
 * part of the drop-in surface: the tests use them to run every parity case
 * through each kernel variant and failure path (every variant gives the same
 * bits), and scripts/ to A/B variants and trace the persistent launches.  A
 * reference caller needs none of it: the defaults are the production settings.
 *
 * All knobs live in one process-wide struct (pqp::Tuning in the library) and
 * are reached through one keyed setter/getter, so the exported surface is four
 * functions whatever the number of knobs.
 *
 * Threading: pqp_tune and pqp_tune_trace serialize their writers, but the
 * launches read the knobs without a lock.  Call them only while no other
 * thread is inside a libpqp solve or launch (set up, then solve); a knob
 * changed during a concurrent solve may be seen by some of its launches and
 * not by others.
 */
#ifndef PQP_TUNING_H
#define PQP_TUNING_H
#ifdef __cplusplus
extern "C" {
#endif

/* Set knob `key` to `value`; the previous value goes to *old_value (may be
 * NULL).  PQP_ERR_ARG for an unknown key.  Knobs (default in brackets):
 *
 *  Kernel variants (all bit-identical):
 *   force_small [0]        N, M <= 32 converge solves on the LDS-staged
 *                          k_solve_small instead of k_solve_tiny / k_solve_wave
 *   force_single [0]       fixed mode of large single problems on one
 *                          workgroup (k_solve_single)
 *   fixed_rl_max_b [1024]  largest batch whose k_fixed_tiny keeps y in registers
 *   wave_min_b [1]         converge mode of N, M <= 32 on k_solve_wave from this
 *                          many problems on
 *   wave_pipe_max_b [4096] largest batch of the software-pipelined k_solve_wave
 *   split_lw [0]           row sides per workgroup of blocks built afterwards
 *                          (0: auto; 8, 16, 32 or 64)
 *   lean_min_n [4096]      row blocks of rows x N >= lean_min_n^2 use the lean
 *                          relay over Qd (k_lean_relay); 0 turns it off
 *   matmul_tiled_off [0]   every setup product through k_matmul_seq
 *   matmul_pk_off [0]      setup products on the 64 x 64 k_matmul_tiled instead of the packed 128 x 128 k_matmul_pk
 *   gj_blocked_off [0]     batched Gauss_Jordan through the one-pivot-per-sweep
 *                          kernel instead of the blocked one (n <= 1024)
 *   batch_opts [0]         batched converge (k_solve_single): bit 0 no fused
 *                          Y'Qd pass; bit 1 the unprepared pqp_batch_solve makes
 *                          Gp' and Qp_inv' per call; bit 4 checkFeas sums every
 *                          row (by default it stops after its first 256 rows
 *                          when one is over its bound: terminate() returns 0
 *                          either way)
 *   pipe_off [0]           batched converge of problems too large for LDS
 *                          (path 2) on k_solve_single (Gp read twice per
 *                          iteration) instead of k_solve_pipe (Gp read once;
 *                          taken when Qp_inv' is prepared, N, M are multiples
 *                          of 4 and M >= N / 3)
 *   pipe_force [0]         k_solve_pipe also where M < N / 3
 *   pipe_variant [0]       k_solve_pipe build: 0 one 128 x 96 Gp tile per
 *                          step (every wave sums a chain) and 16 update loads
 *                          per lane in flight, two workgroups per CU; 3 two
 *                          64 x 64 tiles in flight
 *   mid_off [0]            batched solves of mid-size problems through
 *                          k_solve_small / k_solve_single instead of the
 *                          LDS-resident k_solve_mid (path 3)
 *   mid_v1 [0]             1: path 3 on k_solve_mid (terminate() after each
 *                          update) instead of k_solve_mid2 (terminate(Y_h)
 *                          on other waves beside the update to Y_{h+1})
 *   mid2_pair [0]          k_solve_mid2's update rows: 0 by shape (lane sides
 *                          for 96 <= N <= 128), 1 lane sides (v_med3_f32), 2
 *                          one lane per row (max form)
 *   mid2_min_n [48]        smallest N path 3 runs on k_solve_mid2
 *   single_occ [0]         k_solve_single (16-byte loads) workgroups per CU, by
 *                          its register cap: 0 by shape and batch size (3
 *                          above n_dual 768; below, the fewest rounds of
 *                          resident problems, weighted +10 % per step); 3, 4
 *                          or 5 forces one
 *   mid2_dense [0]         k_solve_mid2 sums every k of each update row and
 *                          Y'Qd row (default: only the band of k where the
 *                          wave's rows hold a nonzero, while Y is finite)
 *   batch_chunk [0]        iterates per problem per batched-solve launch
 *                          (0: sized from N and M)
 *   single_scalar [0]      k_solve_single with 4-byte loads only
 *   wide_min_n [384]       converge mode: smallest N solved over many workgroups
 *   converge_chunk [65536] iterates decided per persistent converge launch
 *                          (<= 0 restores the default)
 *   tiny_old [0]           one problem with N, M <= 32 on the round-4 kernels
 *                          (k_fixed_tiny / k_solve_wave, state copies) instead
 *                          of k_fixed_one / k_solve_quintet (one launch, results
 *                          straight to pinned host memory)
 *   tiny_chunk [0]         iterates per launch of a one-launch tiny solve (0: about
 *                          2^26 element updates; a solve that needs more resumes
 *                          from the device state in further launches)
 *   persist_xcds [0]       k_split_persist's workgroups on this many XCDs (the grid
 *                          padded with workgroups that leave at once; 0: 4, 8:
 *                          spread over all eight)
 *   converge_xcds [0]      the same for k_converge_persist (0: 6 where the grid
 *                          fits, 8: all eight)
 *   tiny_apoll [0]         k_solve_quintet's update wave reads the decision word
 *                          every update (default: only when its ring is full)
 *   tiny_ablk [0]          k_solve_quintet's update wave publishes every update
 *                          (1) instead of every second one (0: two per pass)
 *   tiny_np [0]            k_solve_quintet's B and C roles on 2, 3 (0: default)
 *                          or 4 waves each (iterate r on B / C wave r mod np)
 *   tiny_fallback [0]      read a tiny solve's results from its device copies as
 *                          if the pinned output had missed its tag (tests)
 *   tiny_dense [0]         k_fixed_one / k_solve_quintet without the sparse
 *                          update form (every split entry summed)
 *   iterate_kind [0]       pqp_batch_iterate's kernel: 0 the default (n_dual 1024:
 *                          k_batch_resident, Qd's first blocks kept on the CU in
 *                          registers, LDS and L2 across a launch's iterations;
 *                          other multiples of 1024: k_batch_stream; else
 *                          k_batch_iterate), 1 k_batch_iterate, 2 k_batch_stream,
 *                          3 k_batch_resident without the register blocks
 *  Paths and failure tests:
 *   persist_off [0]        fixed mode of n_dual <= 1024 through the graph-replayed
 *                          relay instead of the persistent launch
 *   converge_persist_off [0]  converge mode through the graph chain instead of
 *                          the persistent launch
 *   persist_fit_cus [0]    CU count the persistent launches' residency check
 *                          assumes (0: the device's; 1 forces the fallback)
 *   persist_stall_wg [-1]  workgroup of every persistent launch that returns at
 *                          once, as if never resident: the other workgroups'
 *                          waits expire (2 s) and the solve restarts on the relay
 *                          / graph chain (< 0: off)
 *   relay_spin_max [2^20]  relay hand-off wait budget in polls; 0 restores the
 *                          default, < 0 makes every wait expire (error path),
 *                          clamped to 2^30
 *   tiny_stall [0]         k_solve_quintet's deciding waves return at once, so
 *                          every wait of the launch expires (error path)
 * Settings apply to launches and graphs made afterwards. */
int pqp_tune(const char *key, long long value, long long *old_value);

/* Read a knob, or a diagnostic:
 *   last_path          solver path of the calling thread's last single-problem
 *                      solve (1 persistent fixed, 2 relay fixed, 3 persistent
 *                      converge, 4 converge graph chain, 5 one workgroup)
 *   last_batch_kernel  the calling thread's last path-2 / path-3 batched
 *                      launch: 0 k_solve_single, 1 k_solve_pipe, 2 k_solve_mid,
 *                      3 k_solve_mid2
 *   persist_fallbacks  persistent launches that fell back (process total)
 *   converge_grid      in: *value = N << 32 | M; out: workgroups of the
 *                      persistent converge launch for (N, M) (0: not used)
 *   batch_chunk_for    in: *value = N << 32 | M; out: iterates per problem per
 *                      pqp_batch_solve launch (the batch_chunk knob if set) */
int pqp_tune_get(const char *key, long long *value);

/* Record an on-device timeline (s_memrealtime / s_memtime marks) of the
 * persistent launches into the device buffer d_buf ("persist": 12 * waves * n
 * words for n updates of k_split_persist; "converge": 2 * n * 35 * 4 words for
 * n iterates of k_converge_persist; "mid": 16 words per problem for the first
 * n problems of a batched k_solve_mid solve -- phase A/B/C/D+E clock totals,
 * iterations, then each wave's phase-A busy clocks, added to what the buffer
 * holds; a k_solve_pipe solve writes phase X / Y / cost clock totals to words
 * 0-2 and iterations to word 4; "tiny": k_solve_quintet's per-wave clocks at
 * N = 28, M <= 8, which needs n >= 24 words, else PQP_ERR_ARG).  n = 0 turns it
 * off.  Timing only. */
int pqp_tune_trace(const char *what, void *d_buf, int n);

/* Test hook: fill the LDS of every CU of the current device with `value`
 * (64 KB per workgroup, 8 workgroups per CU, on the library stream, then
 * synchronise).  A later kernel that reads LDS it never wrote -- padding of a
 * vector -- then reads `value` (e.g. a NaN) instead of whatever was there. */
int pqp_tune_poison_lds(float value);

/* The first n values of glibc's unseeded rand() sequence (the testing/
 * reader's Kp overwrite), for the tests. */
int pqp_tune_glibc_rand(int n, int *out);

#ifdef __cplusplus
}
#endif
#endif
