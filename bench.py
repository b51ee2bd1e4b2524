"""bench.py -- PQP dual-update throughput on MI355X (BASELINE.json configs).

Workload (one line of JSON on rank 0): BASELINE configs[3] at N=1 and
configs[4] across N GPUs -- synthetic dense dual problems of n_dual = 1024
(M = 512 primal), 4096 independent problems per GPU (weak scaling), each
with its own Qd (16 GiB of fp32 Qd per GPU, generated on device), run in the
reference's fixed-iteration mode (testing/ harness: updateY2 only).

A *step* is one updateY2 of every problem of the batch (one PQP iteration of
the whole job).  `value` = problems x steps over all ranks / max-over-ranks
wall time of exactly K steps (inputs already resident in HBM), in
instance-iterations per second.

Extra keys:
  roofline      the fused update kernel vs the 8 TB/s HBM peak, algorithmic
                bytes ALG(N) = 4N^2 + 16N per problem-iteration,
                duration from HIP events on the launch stream; `traffic` is
                the PMC-measured HBM bytes per launch (profiles/pmc_traffic.json)
  cpu_baseline  PQP_CPU.c's own updateY2 (oracle/_ref, compiled from the
                reference) -- or the bit-exact restatement if that build is
                absent -- single thread on this host, bounded sample
  bundled       the bundled example (configs[0]/[1]) on 1 GPU through the
                C ABI: fixed 1000-iteration mode and converge mode (h = 313)
  mpc_batch     16384 MPC problems (bundled plant at perturbed states), one
                workgroup each, converge mode with device-side terminate()
  single_n1024  configs[2]: one n_dual=1024 problem, 1000 fixed iterations
  single_converge  the same problem size in the reference's converge mode
                (terminate() before every update), capped at 2000 updates
  rowshard      one large problem (n_dual = 32768; rowshard_16384 beside it)
                row-sharded over the job's ranks: per update,
                every rank updates its rows and an RCCL all-gather assembles y
                (all ranks take part)
  gather_ms     RCCL gather of every rank's Y* to rank 0 (outside the timed
                region)
  iters_to_tol  converge mode on the problems the reference converges on (the
                bundled example, testing/ test1 and test2): h and time per
                solve, with the reference's own h (cpu_baseline) beside it

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       N > 1 either way:
         python bench.py --gpus N      (this process spawns N ranks itself, one
                                        per GPU, before it touches HIP; it
                                        relays rank 0's line and exits with the
                                        worst rank's status)
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
KERNEL = "k_batch_resident<16,2,2>"


def hot_kernel_hash() -> str:
    """SHA-256 (16 hex) of the hot kernel's source -- the text between the
    <hot-kernel> markers of pqp_kernels.hip, plus the library's compile flags.
    profiles/pmc_traffic.json records carry the hash they were measured with;
    a record whose hash differs is stale and is not reported as `traffic`."""
    return kernel_src_hash("hot-kernel")


# headers every kernel of pqp_kernels.hip includes (the float rules, gap_stop,
# SolveArgs / SolveState, the tuning knobs): a change there changes what the
# measured kernels compute or how they are launched, so it invalidates their
# PMC / VALU records like a change inside the marked region does
KERNEL_HEADERS = ("pqp_device.h", "pqp_launch.h")


def kernel_src_hash(*markers: str, root: Path | None = None) -> str:
    """SHA-256 (16 hex) of the text between pqp_kernels.hip's <marker> and
    </marker> comments (each marker's region, in order), the headers the
    kernels include (KERNEL_HEADERS) and the library's compile flags."""
    import hashlib
    import re

    base = (root or ROOT) / "pqp-for-mpc_amd"
    src = (base / "csrc" / "pqp_kernels.hip").read_text()
    text = ""
    for marker in markers:
        m = re.search(rf"// <{marker}>.*?// </{marker}>", src, re.S)
        text += m.group(0) if m else src
    for h in KERNEL_HEADERS:
        text += (base / "csrc" / h).read_text()
    flags = [ln for ln in (base / "Makefile").read_text().splitlines() if ln.startswith("HIPFLAGS")]
    text += "\n".join(flags)
    return hashlib.sha256(text.encode()).hexdigest()[:16]


def alg_bytes(n: int) -> int:
    """Algorithmic HBM bytes per problem-iteration: Qd read once (the split
    matrices and Theta are derived in registers) + theta, Fd, y_in, y_out."""
    return 4 * n * n + 16 * n


# VALU issue peak: a SIMD-32 issues one wave64 VALU instruction every 2
# clocks when it has several waves (MI355X_MICROARCH.md: 4 clocks is what ONE
# wave alone sustains), 256 CUs x 4 SIMDs x 2.4 GHz / 2
VALU_PEAK_GWI = 256 * 4 * 2.4e9 / 2 / 1e9  # 1228.8 G wave-instructions/s
# fp32 VALU lane-op rate, unpacked (no FMA on this path: a multiply and an add
# are two ops): 256 CUs x 4 SIMDs x 64 lanes / 2 clocks x 2.4 GHz
VALU_LANE_OPS = 256 * 4 * 64 / 2 * 2.4e9  # 78.6 T op/s


def converge_alg_flops(iterates: int, N: int, M: int, feasible: bool = True) -> float:
    """The reference's arithmetic per converge-mode iterate (terminate() +
    updateY2, PQP_CPU.c:603-618, :673-687; O(N) terms dropped): the update's
    two N x N mat-vecs 4N^2; computeUfromY Gp'Y 2NM + Qp_inv tmp 2M^2;
    checkFeas Gp U 2NM; on a feasible iterate computeCost's Y'Qd 2N^2 and
    U'Qp 2M^2.  (The last iterate runs no update: counted anyway, < 0.2 %.)"""
    per = 4.0 * N * N + 4.0 * N * M + 2.0 * M * M + ((2.0 * N * N + 2.0 * M * M) if feasible else 0.0)
    return iterates * per


def valu_roofline(key: str, marker: str, h_sum: int, dt: float, N: int, M: int) -> dict:
    """VALU roofline of a batched solve whose matrices stay in LDS (bound by
    instruction issue, not HBM): the wave-level VALU instructions of this exact
    solve (profiles/pmc_valu.json[key], rocprofv3 SQ_INSTS_VALU, keyed by the
    kernel source hash and the workload's iteration count) over the timed
    solve, against VALU_PEAK_GWI; beside it the reference's algorithmic flops
    (every iterate feasible, as on the bundled plant) against VALU_LANE_OPS."""
    flops = converge_alg_flops(h_sum, N, M)
    out = {"bound": "valu", "alg_flops": flops, "alg_TFLOPs": flops / dt / 1e12,
           "alg_frac": flops / dt / VALU_LANE_OPS,
           "alg_note": "6N^2 + 4NM + 4M^2 per iterate (PQP_CPU.c:603-618, :673-687), every iterate feasible, over "
                       "the unpacked fp32 VALU rate 78.6 T op/s"}
    vf = ROOT / "profiles" / "pmc_valu.json"
    vrec = json.loads(vf.read_text()).get(key) if vf.exists() else None
    khash = kernel_src_hash(marker)
    if vrec and vrec.get("kernel_src_sha256") == khash and vrec.get("h_sum") == h_sum:
        ach = vrec["sq_insts_valu"] / dt / 1e9
        out.update({"achieved": ach, "peak": VALU_PEAK_GWI, "unit": "G wave-instr/s", "frac": ach / VALU_PEAK_GWI,
                    "valu_insts": vrec["sq_insts_valu"], "source": f"profiles/pmc_valu.json {key}"})
    else:
        out.update({"achieved": None, "peak": VALU_PEAK_GWI, "unit": "G wave-instr/s", "frac": None,
                    "source": f"stale or missing VALU record for this kernel source / workload ({khash}); "
                              "re-run scripts/gpu_r06.sh hpmc + scripts/pmc_valu.py"})
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=1024, help="n_dual")
    ap.add_argument("--batch", type=int, default=4096, help="problems per GPU")
    ap.add_argument("--chunk", type=int, default=10,
                    help="iterations (steps) per kernel launch; the iterate stays in LDS between them")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    ap.add_argument("--cpu-instances", type=int, default=16,
                    help="distinct problems the CPU baseline cycles through (>= 8, DRAM-resident)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-bundled", action="store_true")
    ap.add_argument("--rowshard-n", default="32768,16384",
                    help="n_dual of the row-sharded legs, comma-separated (the first is `rowshard`, the others "
                         "`rowshard_<n>`; 0 or empty: skip)")
    ap.add_argument("--rowshard-updates", type=int, default=100)
    ap.add_argument("--rowshard-graph", action="store_true",
                    help="at N > 1, also time the row-sharded steps as hipGraph replays (update + RCCL all-gather)")
    ap.add_argument("--leg-timeout", type=float, default=150.0,
                    help="seconds an optional leg (gather, rowshard, ...) may run before the line is printed without it")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="process-group timeout (s); longer than --leg-timeout")
    return ap.parse_args()


def host_cpu() -> dict:
    """The host's CPU model and the CPUs this process may use."""
    model = "unknown"
    try:
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"model": model, "logical_cpus": os.cpu_count(), "usable_cpus": usable}


def cpu_baseline(n: int, seconds: float, instances: list, tol_cases: dict | None = None,
                 threads: int = 16, horizon: dict | None = None) -> dict:
    """The reference's updateY2 on `instances` (a list of (Qd, Fd) host
    arrays: distinct problems of the bench's own workload, copied from the
    GPU batch), DRAM-resident (8 MiB of split matrices each) and updated
    round-robin for about `seconds`, one thread; the rate extrapolates
    linearly to the batch (instances are independent).  Beside it, an
    all-core row (OpenMP over the host CPUs this process may use, capped at
    `threads`) of the bit-exact restatement, labelled "not reference"."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np

    from oracle import REF_SO, Oracle, Reference

    orc = Oracle()
    cpu = host_cpu()
    K = len(instances)
    mib = K * 8 * n * n / 2**20
    if REF_SO.exists():
        ref = Reference()
        S = [ref.split(Qd, Fd, n) for Qd, Fd in instances]
        Fds = [np.ascontiguousarray(Fd, np.float32) for _, Fd in instances]
        Ys = [np.full(n, 1000.0, np.float32) for _ in range(K)]
        ups, t0 = 0, time.perf_counter()
        while True:
            for j in range(K):
                Ys[j] = ref.update(Ys[j], S[j], Fds[j], n)
            ups += K
            el = time.perf_counter() - t0
            if el >= seconds:
                break
        del S
        kind = "reference"
        what = "oracle/_ref/libpqp_ref.so (PQP_CPU.c, gcc -O2 -ffp-contract=off) updateY2"
        # configs[0]: the bundled example through the reference's own input(),
        # setup and solveQuadraticDual (converge mode, C loop), median of 5
        B = ref.bundled_problem(ROOT / "tests" / "golden")
        times, h = [], 0
        for _ in range(5):
            tb = time.perf_counter()
            h, _, _ = ref.solve(B)
            times.append(time.perf_counter() - tb)
        tb = sorted(times)[len(times) // 2]
        bundled = {"converge_h": h, "converge_ms": tb * 1e3, "iter_per_s": h / tb,
                   "what": "PQP_CPU.c solveQuadraticDual on the bundled example (configs[0]), 1 thread"}
        # configs[0] as BASELINE states it, "1000 iters": the reference's
        # fixed-iteration solve (the testing/ harness loop, 999 updateY2 calls
        # from Y = 1000, PQP_CPU_test.c:714-744) over its own functions, median
        # of 5 -- the like-for-like figure of the GPU's bundled.fixed1000_ms
        runs = [ref.fixed_solve(B, 1000) for _ in range(5)]
        tot = sorted(r[1] for r in runs)[2]
        loop = sorted(r[2] for r in runs)[2]
        yf = runs[0][0]
        bundled["fixed1000"] = {"ms": tot * 1e3, "loop_ms": loop * 1e3, "iter_per_s": 999 / tot,
                                "y_star_zeros": int((yf == 0).sum()), "y_star_1000": int((yf == 1000).sum()),
                                "what": "oracle/_ref/libref_fixed.so: PQP_CPU.c's setup (:696-710) + 999 x "
                                        "(updateY2 :603, copyMatrix) as the testing/ harness runs them, 1 thread, "
                                        "median of 5; ms = setup + loop (the GPU's bundled.fixed1000_ms is one "
                                        "pqp_problem_solve call), loop_ms = the updates alone"}
        # the reference's convertToDual of ONE N = 1024, M = 512 problem with a
        # dense Qp_inv (the setup_convert leg's problems), one thread
        sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
        from pqp_amd import dense_qinv

        Pp = orc.synth_primal(3, 0, n, n // 2)
        tb = time.perf_counter()
        ref.convert_to_dual(dense_qinv(3, n // 2), Pp["Gp"], Pp["Kp"], Pp["Fp"], Pp["Mp"], n, n // 2)
        bundled_setup_s = time.perf_counter() - tb
        if tol_cases:  # iterations to tolerance of the reference on the converging problems
            ref_tol = {}
            for name, Pc in tol_cases.items():
                tb = time.perf_counter()
                h, _, _ = ref.solve(Pc)
                ref_tol[name] = {"h": h, "ms": (time.perf_counter() - tb) * 1e3}
            bundled["iters_to_tol"] = ref_tol
        # the horizon leg's problem 0 per H (copied back from its GPU batch):
        # the reference's solveQuadraticDual, 1 thread, median of 3, and
        # whether it stops at the GPU's h
        hz = {}
        for key, (P0, h_gpu) in (horizon or {}).items():
            ts = []
            for _ in range(3):
                tb = time.perf_counter()
                hr, _, _ = ref.solve(P0)
                ts.append(time.perf_counter() - tb)
            tr = sorted(ts)[1]
            hz[key] = {"h": hr, "same_h_as_gpu": bool(hr == h_gpu), "ms": tr * 1e3, "qp_solves_per_s": 1.0 / tr,
                       "what": "PQP_CPU.c solveQuadraticDual (oracle/_ref) on the horizon leg's problem 0, "
                               "1 thread, median of 3"}
        if hz:
            bundled["horizon"] = hz
    else:
        Qd, Fd = instances[0]
        per, _ = orc.time_updates(Qd, Fd, n, 3)
        ups = max(3, int(seconds / max(per / 3, 1e-6)))
        el, _ = orc.time_updates(Qd, Fd, n, ups)
        kind = "port"
        what = "oracle/pqp_oracle.c (bit-exact restatement, -O2 -ffp-contract=off) updateY2"
        K, mib = 1, 8 * n * n / 2**20
        bundled = None
    out = {"value": ups / el, "unit": "instance-iterations/s", "cores": 1, "kind": kind,
           "sample": f"{what}: {ups} fixed-mode updates round-robin over {K} distinct synthetic problems of the "
                     f"bench workload (n_dual={n}, M={n // 2}; {mib:.0f} MiB of split matrices, DRAM-resident) in "
                     f"{el:.1f} s, 1 thread, setup excluded; the rate extrapolates linearly to the batch "
                     f"(independent problems)",
           "host_cpu": cpu}
    if bundled:
        out["bundled"] = bundled
        out["setup_convert_s"] = bundled_setup_s
    # all-core row (not the reference: the bit-exact restatement over OpenMP)
    thr = max(1, min(threads, cpu["usable_cpus"] or 1))
    Kp = max(thr * 4, K)
    reps = (Kp + K - 1) // K
    qp = np.empty((Kp, n * n), np.float32)
    qn = np.empty((Kp, n * n), np.float32)
    fp = np.empty((Kp, n), np.float32)
    fn = np.empty((Kp, n), np.float32)
    for j in range(Kp):
        Qd, Fd = instances[j % K]
        th = orc.theta(Qd, n)
        qp[j], qn[j] = orc.split_theta(Qd, th, n)
        fp[j] = np.maximum(Fd, 0)  # matrixPos / matrixNeg (:703-704); Fd has no NaN / -0 here
        fn[j] = np.maximum(-Fd, 0)
    Y = np.full((Kp, n), 1000.0, np.float32)
    rounds = 1
    t1 = orc.time_updates_batch(Y, qp, qn, fp, fn, n, rounds, thr)
    rounds = max(1, int(min(seconds, 15.0) / max(t1, 1e-6)))
    t1 = orc.time_updates_batch(Y, qp, qn, fp, fn, n, rounds, thr)
    out["all_cores"] = {"value": Kp * rounds / t1, "unit": "instance-iterations/s", "cores": thr,
                        "kind": "port (OpenMP), not reference",
                        "sample": f"oracle/pqp_oracle.c orc_update_split (bit-exact with PQP_CPU.c updateY2): "
                                  f"{rounds} updates of each of {Kp} problems ({K} distinct, repeated {reps}x; "
                                  f"{Kp * 8 * n * n / 2**30:.2f} GiB of split matrices) over {thr} threads in "
                                  f"{t1:.1f} s"}
    return out


def bundled_bench(pqp_amd) -> dict:
    """configs[1]: the bundled example (N=28, M=7) on one GPU through the C
    ABI.  The problem is uploaded once (pqp_problem_create); each timed solve
    is one pqp_problem_solve call: kernel launch(es) + state/Y readback."""
    import numpy as np

    P = pqp_amd.example_problem(ROOT / "tests" / "golden" / "example")
    reps = 50
    with pqp_amd.Problem(P) as prob:
        prob.solve(pqp_amd.MODE_FIXED, num_iter=1000)  # warm
        t0 = time.perf_counter()
        for _ in range(reps):
            r = prob.solve(pqp_amd.MODE_FIXED, num_iter=1000)
        fixed_s = (time.perf_counter() - t0) / reps
        prob.solve(max_updates=200000)
        t0 = time.perf_counter()
        for _ in range(reps):
            c = prob.solve(max_updates=200000)
        conv_s = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(5):
        pqp_amd.solve_dual(P, mode=pqp_amd.MODE_FIXED, num_iter=1000)
    oneshot_s = (time.perf_counter() - t0) / 5
    return {"n_dual": int(P["N"]), "fixed1000_ms": fixed_s * 1e3, "fixed1000_iter_per_s": 999 / fixed_s,
            "converge_ms": conv_s * 1e3, "converge_h": c["h"], "converge_iter_per_s": c["h"] / conv_s,
            "oneshot_fixed1000_ms": oneshot_s * 1e3, "y_fixed_finite": bool(np.all(np.isfinite(r["Y"]))),
            "note": "wall time of one pqp_problem_solve call on an uploaded problem (launch + D2H of Y); "
                    "oneshot = pqp_solve_dual incl. upload/alloc/setup"}


def mpc_batch_bench(pqp_amd, B: int = 16384) -> dict:
    """Many MPC problems at once: the bundled plant (N=28, M=7) at B states x
    (x perturbed by 5 %, seed 5), per-problem setup and converge-mode solve on
    the GPU, one workgroup per problem.  Timed: the batched solve only."""
    import numpy as np
    import torch

    ex = pqp_amd.read_example(ROOT / "tests" / "golden" / "example")
    xs = pqp_amd.perturbed_states(ex["x"], B, seed=5)
    pb = pqp_amd.mpc_batch(ROOT / "tests" / "golden" / "example", xs)
    pb.solve(max_updates=200000)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pb.solve(max_updates=200000)
    dt = time.perf_counter() - t0
    h = pb.h.cpu().numpy()
    conv = float((pb.status.cpu().numpy() == 1).mean())
    t0 = time.perf_counter()
    pb.solve(pqp_amd.MODE_FIXED, num_iter=1000)
    dtf = time.perf_counter() - t0
    return {"problems": B, "n_dual": int(pb.N), "converge_ms": dt * 1e3, "qp_solves_per_s": B / dt,
            "iterations_per_s": float(h.sum()) / dt, "h_min": int(h.min()), "h_max": int(h.max()),
            "h_mean": float(h.mean()), "converged_frac": conv, "fixed1000_ms": dtf * 1e3,
            "fixed1000_instance_iter_per_s": B * 999 / dtf,
            "note": "bundled plant at B perturbed states; setup (computeFp/Mp, Gauss_Jordan, convertToDual) "
                    "on device, excluded from the timing; each solve bit-exact with PQP_CPU.c (tests)"}


def horizon_bench(pqp_amd, Hs=(2, 4, 5), B: int = 16384, keep: dict | None = None) -> dict:
    """MPC over H horizon stages: B problems of the bundled plant stacked H
    times (pqp_amd.horizon_batch -- block-diagonal primal, each stage at its
    own perturbed state (seed 7), per-stage computeFp / computeMp, Gauss_Jordan
    and convertToDual on the GPU; n_dual 28 H, M 7 H), solved at once in
    converge mode (path 3: k_solve_mid2, one workgroup per problem, every
    matrix once in LDS, terminate() beside the update).  Timed: the batched
    solve only.  With `keep`, problem 0 of each H (host copy) and its GPU h
    are left there for the cpu_baseline leg, which runs the reference's own
    solveQuadraticDual on it (cpu_baseline.horizon)."""
    import torch

    ex = ROOT / "tests" / "golden" / "example"
    E = pqp_amd.read_example(ex)
    out = {}
    for H in Hs:
        xs = pqp_amd.perturbed_states(E["x"], B * H, seed=7).reshape(B, H, -1)
        pb = pqp_amd.horizon_batch(ex, H, xs)
        # capped at the testing/ harness's 1000 iterations: a problem the
        # reference's exact-float gap test never stops (one of the 16384 at H =
        # 2, seed 7 -- the oracle runs it past 3000 updates too) costs 999
        # updates, not the whole timing
        cap = 999
        pb.solve(max_updates=cap)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pb.solve(max_updates=cap)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        h = pb.h.cpu().numpy()
        N, M = pb.N, pb.M
        row = {"n_dual": N, "m": M, "problems": B, "path": int(pqp_amd.lib().pqp_batch_solve_path(N, M)),
               "kernel": {3: "k_solve_mid2", 2: "k_solve_mid"}.get(pqp_amd.tune_get("last_batch_kernel"), "other"),
               "converge_ms": dt * 1e3, "qp_solves_per_s": B / dt, "iterations_per_s": float(h.sum()) / dt,
               "h_min": int(h.min()), "h_max": int(h.max()), "h_mean": float(h.mean()), "max_updates": cap,
               "converged_frac": float((pb.status.cpu().numpy() == 1).mean()),
               "capped": int((pb.status.cpu().numpy() == 2).sum())}
        row["roofline"] = valu_roofline(f"mid2_H{H}", "solve-mid2", int(h.sum()), dt, N, M)
        row["note"] = ("the H stages are stacked block-diagonally and decoupled (each stage its own copy of "
                       "the bundled plant at its own state): a size class of the MPC horizon (n_dual 28 H), "
                       "not a coupled horizon")
        if keep is not None:
            keep[f"H{H}"] = (pb.problem(0), int(h[0]))
        out[f"H{H}"] = row
        del pb
        torch.cuda.empty_cache()
    return out


# the dense companion of the horizon leg: n_dual of H = 4 and H = 5, M = N / 4
# as in the stacked plant, every iterate feasible, h = 313 for every problem
DENSE_SIZES = ((112, 28), (140, 35))
DENSE_UPDATES = 312


def dense_horizon_batch(pqp_amd, N: int, M: int, B: int = 16384, seed: int = 11):
    """B synthetic problems of n_dual N, M primal (the generator behind
    configs[2]-[4]: Gp in {-1, 0, +1}, so Qd = Gp Qp_inv Gp' is dense -- no
    zero band for k_solve_mid2's band sums to skip), duals built on the GPU;
    then Kp = 1e30 seen by checkFeas only (Fd keeps the generator's Kp), so
    every iterate is feasible and runs all of computeCost, as the stacked
    plant's do.  The generator's problems do not meet the exact gap test, so a
    solve capped at DENSE_UPDATES updates stops every problem at h = 313, the
    bundled plant's iteration count."""
    pb = pqp_amd.ProblemBatch.synthetic(seed, 0, B, N, M)
    pb.Kp.fill_(1e30)
    return pb


def horizon_dense_bench(pqp_amd, B: int = 16384) -> dict:
    """The horizon leg's solver on DENSE Qd of the same sizes (VERDICT r5:
    the stacked plant's Qd is block-diagonal, so its band sums skip zeros a
    coupled horizon would not have).  Converge mode, DENSE_UPDATES updates per
    problem, k_solve_mid2 (path 3); timed: the batched solve only."""
    import torch

    out = {}
    for N, M in DENSE_SIZES:
        pb = dense_horizon_batch(pqp_amd, N, M, B)
        pb.solve(max_updates=DENSE_UPDATES)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pb.solve(max_updates=DENSE_UPDATES)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        h = pb.h.cpu().numpy()
        row = {"n_dual": N, "m": M, "problems": B, "path": int(pqp_amd.lib().pqp_batch_solve_path(N, M)),
               "kernel": {3: "k_solve_mid2", 2: "k_solve_mid"}.get(pqp_amd.tune_get("last_batch_kernel"), "other"),
               "converge_ms": dt * 1e3, "qp_solves_per_s": B / dt, "iterations_per_s": float(h.sum()) / dt,
               "h_min": int(h.min()), "h_max": int(h.max()), "max_updates": DENSE_UPDATES,
               "roofline": valu_roofline(f"mid2_dense_N{N}", "solve-mid2", int(h.sum()), dt, N, M),
               "note": "synthetic dense Qd (seed 11), Kp = 1e30 for checkFeas: every iterate feasible, capped at "
                       f"{DENSE_UPDATES} updates (h = 313 as on the bundled plant)"}
        out[f"N{N}"] = row
        del pb
        torch.cuda.empty_cache()
    return out


def single_bench(pqp_amd, N: int = 1024, iters: int = 1000) -> dict:
    """configs[2]: ONE synthetic n_dual=1024 problem, 1000 fixed-mode
    iterations, through pqp_problem_solve (multi-workgroup k_split_update,
    graph-replayed).  The 8 MB of stored split matrices stay in L2/MALL, so
    this is latency- not HBM-bound (single-instance caveat)."""
    import numpy as np

    M = N // 2
    b = pqp_amd.Batch(1, N).generate(seed=1, inst0=0, M=M)
    P = dict(Qd=b.qd_rowmajor(0), Fd=b.Fd[0, :N].cpu().numpy(), Md=b.Md[:1].cpu().numpy(),
             Qp=np.zeros(M * M, np.float32), Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32),
             Mp=np.zeros(1, np.float32), Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32), N=N, M=M)
    del b
    with pqp_amd.Problem(P) as prob:
        prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
        dt = (time.perf_counter() - t0) / reps
    return {"n_dual": N, "iterations": iters, "ms_per_solve": dt * 1e3, "iter_per_s": (iters - 1) / dt,
            "alg_GBps_split_matrices": 8.0 * N * N * (iters - 1) / dt / 1e9,
            "note": "1 problem, fixed mode; per-iteration floor = one lane's N-long sequential sum"}


def setup_bench(pqp_amd, N: int = 1024, M: int = 512, B: int = 64) -> dict:
    """convertToDual (PQP_CPU.c:440-498) of B problems with a
    DENSE Qp_inv on the GPU -- the setup GEMMs (Gp Qp_inv) and (Gp Qp_inv) Gp'
    LDS-tiled, bit-identical to the reference (tests/test_gpu_setup.py)."""
    import torch

    L = pqp_amd.lib()
    pb = pqp_amd.ProblemBatch(B, N, M)
    pqp_amd._check(L.pqp_batch_synth_primal(3, 0, B, N, M, *[pb._p(getattr(pb, k)) for k in pb.PRIMAL], pb._s()))
    pb.Qp_inv.copy_(torch.from_numpy(pqp_amd.dense_qinv(3, M)).cuda().expand(B, -1))
    pb.convert_to_dual()  # warm (the grow-only workspace is allocated here)
    torch.cuda.synchronize()
    samples = []
    for _ in range(5):
        t0 = time.perf_counter()
        pb.convert_to_dual()
        torch.cuda.synchronize()
        samples.append(time.perf_counter() - t0)
    dt = sorted(samples)[len(samples) // 2]
    flops = B * (2.0 * N * M * M + 2.0 * N * N * M)
    del pb
    torch.cuda.empty_cache()
    return {"problems": B, "n_dual": N, "m": M, "ms": dt * 1e3, "ms_samples": [t * 1e3 for t in samples],
            "problems_per_s": B / dt, "gemm_TFLOPs": flops / dt / 1e12,
            "note": "pqp_batch_convert_to_dual, dense Qp_inv: k_matmul_pk (packed fp32, no FMA, k in order per "
                    "output) for the two GEMMs, k_matvec_lane for Fd, k_vecmat for Md; median of 5 calls; "
                    "the reference's one-problem setup time is cpu_baseline.setup_convert_s"}


def batch_converge_bench(pqp_amd, N: int = 1024, B: int = 4096, K: int = 4) -> dict:
    """converge mode of B synthetic problems at once
    (ProblemBatch over pqp_batch_prepare + pqp_batch_solve_prepared,
    terminate() before every update), capped at K updates (the synthetic
    problems do not meet the exact gap test at this size).  One iteration =
    terminate() + updateY2 (PQP_CPU.c:716-725).  Two cases: the generator's
    problems, whose iterates fail checkFeas (terminate() stops there: no Y'Qd,
    no U'Qp), and the same problems with Kp = 1e30 seen by checkFeas only, so
    every iterate runs all of computeCost (PQP_CPU.c:648-666)."""
    import torch

    pb = pqp_amd.ProblemBatch.synthetic(1, 0, B, N)
    M = pb.M
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pb.prepare()  # once per batch: symmetry flags, Theta, Gp' and Qp_inv'
    torch.cuda.synchronize()
    prep_ms = (time.perf_counter() - t0) * 1e3
    pb.solve(max_updates=1)  # warm

    def call(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pb.solve(max_updates=k)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    pipe = pqp_amd.tune_get("last_batch_kernel") == 1
    # iterates per launch of pqp_batch_solve_prepared, as the library sizes it
    # (2^28 / the update's and terminate()'s element count, or the batch_chunk knob)
    chunk = pqp_amd.batch_chunk_for(N, M)
    kname = "k_solve_pipe" if pipe else "k_solve_single"
    rec = {}
    tf = ROOT / "profiles" / "pmc_traffic.json"
    db = json.loads(tf.read_text()) if tf.exists() else {}
    khash = kernel_src_hash("solve-single", "solve-pipe") if pipe else kernel_src_hash("solve-single")
    # algorithmic bytes per problem-iteration: every matrix terminate() and
    # updateY2 read, once -- Qd (the update; on feasible iterates Y'Qd rides in
    # the same pass), Gp (Gp'Y and checkFeas's Gp U), Qp_inv, and on feasible
    # iterates Qp (U'Qp).  k_solve_pipe moves exactly these.  k_solve_single
    # (pipe_off) reads Gp twice: the second time, on these infeasible
    # iterates, only its first 256 rows (a row over its bound there decides
    # terminate(); tuning bit 4 reads all 4NM) -- its `design_bytes_per_iter`
    first = 4.0 * min(N, 256) * M
    for case, alg in (("infeasible", 4.0 * N * N + 4.0 * N * M + 4.0 * M * M),
                      ("feasible", 4.0 * N * N + 4.0 * N * M + 8.0 * M * M)):
        design = alg if pipe else alg + (first if case == "infeasible" else 4.0 * N * M)
        if case == "feasible":
            pb.Kp.fill_(1e30)
            pb.solve(max_updates=1)
        # warm-up: >= 2 s of these very iterations first (after 0.5 s the
        # pass still ran up to 5 % slower than a second later:
        # profiles/r04/bench_r04q.json, profiles/r04/pipe/bench_vs_standalone.json)
        tw = time.perf_counter()
        while time.perf_counter() - tw < 2.0:
            call(3 * K)
        # the same call with K and with 3K updates, both within one launch (a
        # launch runs `chunk` iterates, pqp_capi.cpp): the difference is 2K
        # iterations, no per-call or per-launch cost; the median of 3 such pairs
        assert 3 * K <= chunk, (K, chunk)
        samples, ok, dts = [], True, []
        for _ in range(3):
            dt = call(K)
            ok = ok and bool((pb.h == K + 1).all().item())
            dt3 = call(3 * K)
            ok = ok and bool((pb.h == 3 * K + 1).all().item())
            samples.append((dt3 - dt) / (2 * K))
            dts.append(dt)
        per_iter = sorted(samples)[1]
        dt = sorted(dts)[1]
        # a long solve also pays each launch's start (state, the first Gp'Y
        # pass, the host's check of the pending count): chunk vs 2 chunk
        # updates, one launch more per chunk iterations
        per_iter_solve = (call(2 * chunk) - call(chunk)) / chunk
        single = None
        if pipe:  # the same iterations on k_solve_single (Gp read twice), same process and box
            prev = pqp_amd.tune("pipe_off", 1)
            try:
                tw = time.perf_counter()
                while time.perf_counter() - tw < 0.5:
                    call(3 * K)
                single = sorted((call(3 * K) - call(K)) / (2 * K) for _ in range(3))[1]
            finally:
                pqp_amd.tune("pipe_off", prev)
        gbs = alg * B / per_iter / 1e9
        r = {"ms_per_iteration": per_iter * 1e3, "ms_per_iteration_samples": [x * 1e3 for x in samples],
             "instance_iter_per_s": B / per_iter,
             "alg_bytes_per_iter": alg, "alg_GBps": gbs, "frac_of_hbm_peak": gbs / HBM_PEAK_GBS,
             "design_bytes_per_iter": design, "design_GBps": design * B / per_iter / 1e9,
             "call_ms": dt * 1e3, "call_instance_iter_per_s": B * K / dt, "all_capped": ok,
             "ms_per_iteration_incl_launches": per_iter_solve * 1e3,
             "frac_of_hbm_peak_incl_launches": alg * B / per_iter_solve / 1e9 / HBM_PEAK_GBS}
        if single is not None:
            r["k_solve_single_ms_per_iteration"] = single * 1e3
            r["speedup_vs_k_solve_single"] = single / per_iter
        pmc = db.get(f"{kname}_{case}")
        if pmc and pmc.get("kernel_src_sha256") == khash:
            r["traffic_ratio"] = pmc["traffic_ratio"]
            r["traffic_source"] = f"profiles/pmc_traffic.json {kname}_{case}"
        else:
            r["traffic_ratio"] = None
            r["traffic_source"] = "no PMC record for this kernel source (scripts/gpu_batch_converge.sh)"
        rec[case] = r
    del pb
    torch.cuda.empty_cache()
    return {"problems": B, "n_dual": N, "m": M, "updates": K, "iterates_per_launch": chunk, "prepare_ms": prep_ms,
            **rec, "kernel": kname,
            "note": f"{kname}, one workgroup per problem; ms_per_iteration = (time of a 3K-update call - time "
                    "of a K-update call) / 2K, both within one launch: the iterations alone, median of 3 pairs; "
                    "ms_per_iteration_incl_launches = the same over calls of 1 and 2 launches (each launch's "
                    "start amortized over its iterates, as in a long solve); call_ms = one K-update call "
                    "(K + 1 terminate() + K updates, state init and readback); prepare_ms = pqp_batch_prepare, "
                    "once per batch"}


def _testing_file(name: str, tmpdir: Path) -> Path:
    """testing/sample test/<name>, committed under tests/golden/testing (the
    two large ones gzip'd)."""
    import gzip

    plain = ROOT / "tests" / "golden" / "testing" / name
    if plain.exists():
        return plain
    out = tmpdir / name
    out.write_bytes(gzip.decompress((plain.parent / (name + ".gz")).read_bytes()))
    return out


TOL_CASES = ("bundled", "test1.txt", "test2.txt")


def tol_problems(pqp_amd, tmpdir: Path) -> dict:
    """The converging reference problems: the bundled example and the two
    testing/ samples that converge (n_dual 1500 and 400)."""
    P = {"bundled": pqp_amd.example_problem(ROOT / "tests" / "golden" / "example")}
    for name in TOL_CASES[1:]:
        P[name] = pqp_amd.testfile_problem(_testing_file(name, tmpdir))
    return P


def iters_to_tol_bench(pqp_amd, problems: dict) -> dict:
    """Converge mode on the GPU: iterations to the reference's tolerance and
    wall time per solve (problem resident, launch + readback)."""
    out = {}
    for name, P in problems.items():
        with pqp_amd.Problem(P) as prob:
            r = prob.solve(max_updates=200000)
            ts = []
            for _ in range(5):  # median of 5 solves (one solve is a fraction of a millisecond)
                t0 = time.perf_counter()
                r = prob.solve(max_updates=200000)
                ts.append(time.perf_counter() - t0)
            dt = sorted(ts)[2]
        out[name] = {"n_dual": int(P["N"]), "h": r["h"], "converged": bool(r["converged"]), "ms": dt * 1e3}
    return out


def single_converge_bench(pqp_amd, N: int = 1024, updates: int = 2000) -> dict:
    """One synthetic problem (primal, Qp and duals built on the device) in
    converge mode: terminate() + updateY2 per iteration, as one persistent
    pipelined launch.  The synthetic problems do not meet the reference's exact
    gap test at this size, so the solve is capped."""
    pb = pqp_amd.ProblemBatch.synthetic(1, 0, 1, N)
    P = pb.problem(0)
    del pb
    with pqp_amd.Problem(P) as prob:
        prob.solve(max_updates=2)
        t0 = time.perf_counter()
        r = prob.solve(max_updates=updates)
        dt = time.perf_counter() - t0
    return {"n_dual": N, "m": N // 2, "iterations": r["h"], "converged": bool(r["converged"]),
            "ms_per_solve": dt * 1e3, "us_per_iter": dt / r["h"] * 1e6, "iter_per_s": r["h"] / dt,
            "note": "one persistent pipelined launch (pqp_converge.hip): the update and terminate()'s stages as "
                    "concurrent workgroup roles, terminate(Y_u) beside the update to Y_{u+1}"}


def _sync(dev):
    import torch

    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class _FaultyBlock:
    """PQP_BENCH_FAULT=rowshard:<rank>: this rank's row block raises inside
    the leg's first timed update (failure injection for the N > 1 tests)."""

    def __init__(self, blk):
        self.blk, self.row0, self.rows, self.calls = blk, blk.row0, blk.rows, 0

    def update(self, Y, Y_rows):
        self.calls += 1
        if self.calls > 5:  # past the warm-up steps, inside the timed region
            raise RuntimeError("injected row-block failure (PQP_BENCH_FAULT)")
        self.blk.update(Y, Y_rows)


def rowshard_bench(pqp_amd, dist, rank: int, world: int, dev, N: int, updates: int, graph: bool = True,
                   make_block=None) -> dict:
    """One synthetic problem of n_dual = N whose rows are spread over the
    ranks (pqp_amd.rowshard); fixed-mode updates, timed as the max over
    ranks.  Every rank ends with the whole iterate.  `make_block(N, row0,
    rows)`: another block than the GPU RowBlock (the CPU tests)."""
    import torch

    from pqp_amd.rowshard import RowShardedSolver, row_plan

    R, plan = row_plan(N, world)
    row0, rows = plan[rank]
    # every rank builds its block; the ranks agree on the outcome before any
    # collective of the leg, so a failed setup on one rank ends the leg on all
    # of them instead of leaving its peers in an all-gather
    blk, err = None, None
    try:
        blk = (make_block(N, row0, rows) if make_block else
               pqp_amd.RowBlock.synthetic(7, 0, N, row0, rows, device=dev)[0])
    except Exception as e:  # noqa: BLE001 -- reported below, on every rank
        err = f"{type(e).__name__}: {e}"
    if dist is not None:
        flag = torch.tensor([0 if err is None else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if int(flag.item()) and err is None:
            err = "row-block setup failed on another rank"
    if err is not None:
        raise RuntimeError(err)
    if os.environ.get("PQP_BENCH_FAULT") == f"rowshard:{rank}":
        blk = _FaultyBlock(blk)
    solver = RowShardedSolver(blk, N, dev, dist=dist)

    def timed(n, fn=None):
        _sync(dev)
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        (fn or solver.advance)(n)
        _sync(dev)
        if dist is not None:
            dist.barrier()
        t = torch.tensor([time.perf_counter() - t0, 0.0], dtype=torch.float64, device=dev)
        try:
            solver.check()  # no expired in-kernel wait in any update of this rank's block
        except Exception:  # noqa: BLE001 -- every rank learns of it from the all-reduce below
            t[1] = 1.0
        if dist is not None:  # the flag rides with the timing: no rank raises while a peer waits
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if float(t[1]):
            raise RuntimeError("a row block's in-kernel hand-off wait expired (pqp_rowblock_check) on some rank")
        return float(t[0]) / n

    solver.Y.fill_(1000.0)
    solver.advance(5)
    dt_eager = timed(updates)
    y_eager = solver.Y[:N].clone()
    # the same eager updates without the collective (each rank's block alone,
    # max over ranks): the difference is what the all-gather costs per update
    # (DESIGN §6 assumed 10-25 us for it; this measures it on the first N > 1 run)
    dt_block = timed(updates, solver.block_steps)
    # the same updates as hipGraph replays (block update + RCCL all-gather per
    # step, 16 steps per graph); not on gloo (rehearsal), see RowShardedSolver.capture
    G = 16
    # RowShardedSolver.capture is tested on a one-rank RCCL group only (one GPU
    # per box); at N > 1 the bench captures only when asked (--rowshard-graph)
    graphed = solver.capture(G) if graph else False
    dt_graph, same = None, None
    if graphed:
        solver.Y.fill_(1000.0)
        solver.advance(5)
        solver.advance(updates)  # reach the eager run's iterate, then time more
        same = bool(torch.equal(solver.Y[:N], y_eager))
        dt_graph = timed(max(G, updates // G * G))
    dt = min(dt_eager, dt_graph) if dt_graph else dt_eager
    y = solver.Y[:N]
    out = {"n_dual": N, "ranks": world, "rows_per_rank": R, "updates": updates, "us_per_update": dt * 1e6,
           "iter_per_s": 1.0 / dt,
           "finite_nonneg": bool(torch.isfinite(y).all().item()) and bool((y >= 0).all().item()),
           "us_per_update_eager": dt_eager * 1e6,
           "us_per_update_block_only": dt_block * 1e6,
           "allgather_us_per_update": (dt_eager - dt_block) * 1e6 if dist is not None else None,
           "us_per_update_graph": dt_graph * 1e6 if dt_graph else None,
           "graph_same_bits_as_eager": same,
           "graph_note": (f"{G} updates ({'block update + all-gather' if dist is not None else 'block update'}) "
                          "per hipGraph replay" if graphed else
                          "not captured: N > 1 without --rowshard-graph" if not graph else
                          f"not captured: {solver.capture_error or 'gloo group (rehearsal)'}"),
           "note": "us_per_update = the faster of eager launches (pqp_rowblock_update + all_gather_into_tensor per "
                   "update at N>1 ranks) and graph replays"}
    if make_block is None:
        lean_min = pqp_amd.tune_get("lean_min_n")
        lean = lean_min > 0 and rows * N >= lean_min * lean_min  # row blocks choose the lean relay by rows x N
        bpe = 4 if lean else 8  # bytes per matrix entry the update streams
        out["layout"] = "Qd packets, k_lean_relay (4 B/entry)" if lean else "stored split matrices (8 B/entry)"
        out["alg_GBps"] = bpe * N * N / dt / 1e9
    del solver, blk
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    return out


def _dig(d, *path):
    for k in path:
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return d


def summary(result: dict) -> dict:
    """Every leg's headline numbers in one small object, printed as the LAST
    key of the line (the driver's record keeps only the line's tail, so the
    legs printed early -- batch_converge first -- would otherwise be cut).
    A leg that failed or did not run shows as null."""
    def r(v, nd=4):
        return round(v, nd) if isinstance(v, float) else v

    S = {"value": r(result.get("value"), 1), "hbm_frac": r(_dig(result, "roofline", "frac")),
         "avg_launch_ms": r(_dig(result, "roofline", "avg_launch_ms"), 3),
         "traffic_ratio": (r(_dig(result, "roofline", "traffic") / _dig(result, "roofline", "alg_bytes_per_launch"))
                           if isinstance(_dig(result, "roofline", "traffic"), (int, float)) else None)}
    if result.get("n_gpus", 1) > 1:
        S["per_rank_timed_s"] = _dig(result, "per_rank", "timed_s")
        S["gather_ms"] = _dig(result, "per_rank", "gather_ms")
    for case in ("infeasible", "feasible"):
        S[f"batch_converge_{case}"] = {"ms_per_iter": r(_dig(result, "batch_converge", case, "ms_per_iteration"), 3),
                                       "hbm_frac": r(_dig(result, "batch_converge", case, "frac_of_hbm_peak"))}
    for H in ("H2", "H4", "H5"):
        S[f"horizon_{H}"] = {"ms": r(_dig(result, "horizon", H, "converge_ms"), 2),
                             "valu_frac": r(_dig(result, "horizon", H, "roofline", "frac")),
                             "alg_frac": r(_dig(result, "horizon", H, "roofline", "alg_frac"))}
    for key in ("N112", "N140"):
        S[f"horizon_dense_{key}"] = {"ms": r(_dig(result, "horizon_dense", key, "converge_ms"), 2),
                                     "valu_frac": r(_dig(result, "horizon_dense", key, "roofline", "frac")),
                                     "alg_frac": r(_dig(result, "horizon_dense", key, "roofline", "alg_frac"))}
    S["bundled_fixed1000_ms"] = r(_dig(result, "bundled", "fixed1000_ms"))
    S["bundled_converge_ms"] = r(_dig(result, "bundled", "converge_ms"))
    S["mpc_batch_ms"] = r(_dig(result, "mpc_batch", "converge_ms"), 3)
    S["single_n1024_ms_per_1000"] = r(_dig(result, "single_n1024", "ms_per_solve"))
    S["single_converge_us_per_iter"] = r(_dig(result, "single_converge", "us_per_iter"))
    S["setup_TFLOPs"] = r(_dig(result, "setup_convert", "gemm_TFLOPs"), 2)
    S["rowshard_us_per_update"] = r(_dig(result, "rowshard", "us_per_update"), 2)
    S["iters_to_tol_identical"] = result.get("iters_to_tol_identical_to_reference")
    S["cpu_baseline"] = r(_dig(result, "cpu_baseline", "value"), 1)
    errors = sorted(k for k, v in result.items() if isinstance(v, dict) and "error" in v)
    if errors:
        S["legs_with_errors"] = errors
    return S


def rank_spread(dist, dev, **vals) -> dict:
    """Min and max over the job's ranks of each named value (two all-reduces;
    every rank must call it).  At one rank min = max = the value."""
    import torch

    names = list(vals)
    lo = torch.tensor([float(vals[k]) for k in names], dtype=torch.float64, device=dev)
    hi = lo.clone()
    if dist is not None:
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return {k: {"min": float(lo[i]), "max": float(hi[i])} for i, k in enumerate(names)}


class Emitter:
    """Rank 0's one JSON line, printed exactly once.

    The headline (`result`) is measured and held before any optional leg
    runs.  Each leg then runs under :meth:`leg`: an exception becomes
    ``{"error": ...}`` under the leg's key, and a leg still running after
    `leg_timeout_s` (a collective whose peer never arrives) makes the
    watchdog print the line with that leg marked as timed out and end the
    process with status 0 -- on every rank, before the process group's own
    timeout would abort it.  So no optional leg can cost the job its line.
    `abort_on_failure` (multi-rank jobs): a leg that fails ends the process
    at once, after rank 0 has printed: a peer may still be inside one of that
    leg's collectives, and any later leg's collectives would meet it there
    out of order -- leaving, the rank unblocks gloo peers at once (the
    connection closes); RCCL peers end by their own watchdog."""

    def __init__(self, rank: int, result: dict | None, leg_timeout_s: float, abort_on_failure: bool = False):
        import threading

        self.rank, self.result, self.timeout = rank, result, float(leg_timeout_s)
        self.abort = bool(abort_on_failure)
        self._lock = threading.Lock()
        self._printed = False
        self.failed = False

    def emit(self):
        with self._lock:
            if self.rank == 0 and not self._printed and self.result is not None:
                self.result.pop("summary", None)
                self.result["summary"] = summary(self.result)  # last key: the driver keeps the line's tail
                print(json.dumps(self.result), flush=True)
            self._printed = True

    def _expire(self, name: str):
        with self._lock:
            if self._printed:
                return
            if self.result is not None:
                self.result[name] = {"error": f"timed out: no result within {self.timeout:.0f} s "
                                              "(a peer rank never reached the collective?)"}
        self.emit()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)

    def leg(self, name: str, fn):
        import threading

        print(f"bench: rank {self.rank}: {name} ...", file=sys.stderr, flush=True)  # progress (stderr)
        t = threading.Timer(self.timeout, self._expire, args=(name,))
        t.daemon = True
        t.start()
        try:
            out = fn()
        except Exception as e:  # noqa: BLE001 -- an optional leg never costs the headline
            out = {"error": f"{type(e).__name__}: {e}"}
            self.failed = True
        finally:
            t.cancel()
        with self._lock:
            if self.result is not None and not self._printed:
                self.result[name] = out
        if self.failed and self.abort:
            self.emit()
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)
        return out


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, cmd: list[str], grace_s: float = 60.0) -> int:
    """Run `cmd` as n ranks of one job on this node (one process per GPU, the
    torchrun environment contract: RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT), wait for all of them and return the worst exit
    status.  Nothing here imports torch or touches HIP: the GPUs belong to the
    children.  When a rank fails, the others get `grace_s` to finish before
    they are terminated (a rank stuck in a collective with a dead peer would
    otherwise wait forever)."""
    import signal
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    rcs: list[int | None] = [None] * n
    deadline = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if deadline is None and any(rc not in (None, 0) for rc in rcs):
            deadline = time.monotonic() + grace_s
        if deadline is not None and time.monotonic() > deadline:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    os.killpg(p.pid, signal.SIGTERM)
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        os.killpg(p.pid, signal.SIGKILL)
                        rcs[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    if not bad:
        return 0
    # a signal death (negative) reports as 128 + signal, as a shell would
    return max(128 - rc if rc < 0 else rc for rc in bad)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without a launcher: become the launcher.
        sys.exit(launch_ranks(args.gpus, [sys.executable, "-u", str(Path(__file__).resolve())] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")

    import torch

    import pqp_amd

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PQP_BENCH_REHEARSE=1: rehearse the N > 1 control flow on a one-GPU box.
    # RCCL refuses two ranks on one device, so every rank takes cuda:0 and the
    # collectives go over gloo (which takes device tensors).  The numbers of
    # such a run are not throughput; the JSON line says "rehearsal".
    rehearse = os.environ.get("PQP_BENCH_REHEARSE") == "1" and world > 1
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        # an explicit timeout: a collective whose peer never arrives ends with an
        # error (after the Emitter's leg watchdog has already printed the line)
        dist.init_process_group("gloo" if rehearse else "nccl", device_id=None if rehearse else dev,
                                timeout=timedelta(seconds=args.dist_timeout))

    N, B, K, W, C = args.n, args.batch, args.steps, args.warmup, max(1, args.chunk)
    # "scatter inputs": rank 0 hands each rank its (seed, first problem, count)
    from pqp_amd.shard import gather_rows, scatter_plan

    seed, inst0, B = scatter_plan(dist, rank, world, B, args.seed, dev)

    batch = pqp_amd.Batch(B, N, device=dev)
    batch.generate(seed, inst0=inst0, M=N // 2)
    stream = torch.cuda.current_stream(dev)

    def run(steps):
        launches = 0
        done = 0
        first = True
        while done < steps:
            c = min(C, steps - done)
            batch.iterate(c, from_start=first and done == 0)
            first = False
            done += c
            launches += 1
        return launches

    run(max(W, 1))
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    launches = run(K)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1)
    # the max over ranks is the job's time; the min beside it shows a slow rank
    spread = rank_spread(dist, dev, timed_s=elapsed, kern_ms=kern_ms)
    elapsed, kern_ms = spread["timed_s"]["max"], spread["kern_ms"]["max"]

    Yh = batch.Y[:, :N]
    finite = bool(torch.isfinite(Yh).all().item()) and bool((Yh >= 0).all().item())

    # The headline line is complete here; it is held (rank 0) while the
    # optional legs run, each under the Emitter's guard.
    result = headline(args, rank, world, N, B, K, W, C, elapsed, kern_ms, launches, finite, rehearse,
                      spread=spread) if rank == 0 else None
    em = Emitter(rank, result, args.leg_timeout, abort_on_failure=world > 1)

    if dist is not None:  # gather Y* to rank 0 over RCCL (reported separately, not in `value`)
        def gather_leg():
            y = batch.Y[:, :N].contiguous()
            torch.cuda.synchronize(dev)
            g0 = time.perf_counter()
            full = gather_rows(dist, rank, world, y)
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - g0) * 1e3
            ok = None
            if rank == 0:  # rank order = problem order: rank 0's own block leads
                ok = tuple(full.shape) == (B * world, N) and bool(torch.equal(full[:B], y))
            return {"ms": ms, "ok": ok, "spread": rank_spread(dist, dev, gather_ms=ms)["gather_ms"]}

        g = em.leg("gather", gather_leg)
        if result is not None:
            result["gather_ms"], result["gather_ok"] = g.get("ms"), g.get("ok")
            result.setdefault("per_rank", {})["gather_ms"] = g.get("spread")
    # the CPU baseline's sample: distinct problems of this very workload, from
    # the GPU batch (host copies, 4 MiB of Qd each)
    inst = None
    if world == 1 and not args.no_cpu_baseline:
        inst = [(batch.qd_rowmajor(j), batch.Fd[j, :N].cpu().numpy()) for j in range(min(args.cpu_instances, B))]
    # the headline's 4096 problems (Qd alone 16 GiB per GPU) are no longer
    # needed: free them before the legs allocate their own
    batch = Yh = None
    torch.cuda.empty_cache()
    hz_keep = {}  # the horizon leg's problem 0 per H, for the cpu_baseline leg
    if world == 1 and not args.no_bundled:
        # first of the legs: run after the others (their allocations and
        # frees, compute-heavy kernels) the same pass measured 5-9 % slower
        # than in a fresh process (profiles/r04/pipe/bench_vs_standalone.json)
        em.leg("batch_converge", lambda: batch_converge_bench(pqp_amd))
    sizes = [int(v) for v in str(args.rowshard_n).split(",") if v.strip() and int(v) > 0]
    for i, n_rs in enumerate(sizes):  # every rank takes part
        em.leg("rowshard" if i == 0 else f"rowshard_{n_rs}",
               lambda n_rs=n_rs: rowshard_bench(pqp_amd, dist, rank, world, dev, n_rs, args.rowshard_updates,
                                                graph=world == 1 or args.rowshard_graph))
    if world == 1 and not args.no_bundled:
        em.leg("bundled", lambda: bundled_bench(pqp_amd))
        em.leg("mpc_batch", lambda: mpc_batch_bench(pqp_amd))
        em.leg("horizon", lambda: horizon_bench(pqp_amd, keep=None if args.no_cpu_baseline else hz_keep))
        em.leg("horizon_dense", lambda: horizon_dense_bench(pqp_amd))
        em.leg("single_n1024", lambda: single_bench(pqp_amd))
        em.leg("single_converge", lambda: single_converge_bench(pqp_amd))
        em.leg("setup_convert", lambda: setup_bench(pqp_amd))
    tol_cases = None
    if world == 1 and not args.no_bundled:
        import tempfile

        with tempfile.TemporaryDirectory() as td:
            tol_cases = tol_problems(pqp_amd, Path(td))
        em.leg("iters_to_tol", lambda: iters_to_tol_bench(pqp_amd, tol_cases))
    if world == 1 and not args.no_cpu_baseline:
        cb = em.leg("cpu_baseline", lambda: cpu_baseline(N, args.cpu_seconds, inst, tol_cases, horizon=hz_keep))
        ref_tol = cb.get("bundled", {}).get("iters_to_tol")
        if ref_tol and "iters_to_tol" in result and "error" not in result["iters_to_tol"]:
            result["iters_to_tol_identical_to_reference"] = all(
                result["iters_to_tol"][k]["h"] == ref_tol[k]["h"] for k in ref_tol)
    em.emit()
    if dist is not None:
        if em.failed:  # a peer may be stuck in the failed leg's collective: do not wait for it
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)
        dist.destroy_process_group()


def headline(args, rank, world, N, B, K, W, C, elapsed, kern_ms, launches, finite, rehearse,
             spread: dict | None = None) -> dict:
    """The headline JSON object (rank 0): throughput of exactly K steps over
    all ranks, the hot kernel's roofline, the result check."""
    per_launch_ms = kern_ms / launches
    achieved = alg_bytes(N) * B * C / (per_launch_ms * 1e-3) / 1e9 if launches else 0.0
    traffic, traffic_src = None, "no PMC record for this shape"
    khash = hot_kernel_hash()
    tf = ROOT / "profiles" / "pmc_traffic.json"
    if tf.exists():
        rec = json.loads(tf.read_text()).get(f"n{N}_b{B}_c{C}")
        if rec and rec.get("kernel_src_sha256") == khash:
            traffic = rec.get("hbm_bytes_per_launch")
            traffic_src = f"profiles/pmc_traffic.json n{N}_b{B}_c{C} ({rec.get('source', '')})"
        elif rec:
            traffic_src = (f"stale: the PMC record was measured on kernel source {rec.get('kernel_src_sha256')}, "
                           f"this tree's is {khash}; re-run scripts/gpu_profile.sh")
    result = {
        "metric": "PQP iterations/sec (and QP-instances/sec) at fixed n_dual",
        "value": B * world * K / elapsed,
        "unit": "instance-iterations/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed * 1e3 / K,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (counter-based generator, dual built on device with convertToDual's exact arithmetic)",
        "config": {"workload": "BASELINE configs[3] (N=1) / configs[4] (N=8): synthetic n_dual=1024, M=512, "
                               f"{B} independent problems per GPU, fixed-iteration updateY2",
                   "n_dual": N, "batch_per_gpu": B, "global_batch": B * world, "iters_per_launch": C,
                   "parallelism": f"problem-sharded x{world} (no data-path collective)"},
        "qp_instances_per_s_at_1000_iters": B * world * K / elapsed / 999.0,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel_src_sha256": khash, "kernel": KERNEL,
                     "alg_bytes_per_launch": alg_bytes(N) * B * C, "avg_launch_ms": per_launch_ms},
        "results_finite_nonneg": finite,
        "gather_ms": None,
        "gather_ok": None,
    }
    if world > 1 and spread is not None:
        # each rank's timed region (s) and HIP-event kernel time (ms): min and max over ranks
        result["per_rank"] = dict(spread)
    if rehearse:
        result["rehearsal"] = "all ranks on cuda:0 over gloo (PQP_BENCH_REHEARSE=1): control-flow check, not a measurement"
    return result


if __name__ == "__main__":
    main()
