"""Where the batched converge iteration's time goes:
pqp_batch_solve on B synthetic problems (n_dual N, M = N/2), steady-state
time per iteration = (time of a 3K-update call - time of a K-update call) / 2K
for: fixed mode (the update pass alone), converge mode on infeasible iterates
(terminate() stops at checkFeas) and on feasible ones (Kp = 1e30 seen by
checkFeas only: all of computeCost runs), each under the batch-converge
tuning options.  Prints one JSON line.
Usage: python scripts/batch_converge_breakdown.py [N B K [variant,...]]
(variants: fused_T unfused_T fused unfused fused_T_occ4 unfused_T_occ4 -- the
fused Y'Qd pass on / off, with / without the prepared transposes of Gp and
Qp_inv, k_solve_single built for 4 workgroups per CU; single_T: k_solve_single
instead of k_solve_pipe, which the *_T variants take by default)"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(N=1024, B=4096, K=4):
    import torch

    import pqp_amd

    pb = pqp_amd.ProblemBatch.synthetic(1, 0, B, N)
    L = pqp_amd.lib()
    M = pb.M
    kp = pb.Kp.clone()

    def per_iter(**kw):
        def call(k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if kw.get("mode") == 1:
                pb.solve(pqp_amd.MODE_FIXED, num_iter=k + 1)
            else:
                pb.solve(max_updates=k)
            torch.cuda.synchronize()
            return time.perf_counter() - t0
        call(1)
        a, b = call(K), call(3 * K)
        return {"call_ms": a * 1e3, "per_iter_ms": (b - a) / (2 * K) * 1e3, "setup_ms": (a - K * (b - a) / (2 * K)) * 1e3}

    out = {"n_dual": N, "m": M, "problems": B, "K": K}
    GB = B * 1e-9
    variants = {"fused_T": (0, True), "unfused_T": (1, True), "fused": (0, False), "unfused": (1, False),
                "fused_T_occ4": (8, True), "unfused_T_occ4": (9, True), "fused_T_fullfeas": (16, True),
                "single_T": (0, True, 1)}
    names = sys.argv[4].split(",") if len(sys.argv) > 4 else list(variants)
    for name in names:
        opts, tr, pipe_off = (variants[name] + (0,))[:3]
        pb.transposes = tr
        pb.invalidate()
        t0 = time.perf_counter()
        pb.prepare()
        torch.cuda.synchronize()
        prep_ms = (time.perf_counter() - t0) * 1e3
        prev = L.pqp_tune_batch_converge(opts)
        prev_pipe = pqp_amd.tune("pipe_off", pipe_off)
        try:
            r = {"fixed": per_iter(mode=1)}
            pb.Kp.copy_(kp)
            r["infeasible"] = per_iter()
            pb.Kp.fill_(1e30)
            r["feasible"] = per_iter()
            pb.Kp.copy_(kp)
            r["kernel"] = "k_solve_pipe" if pqp_amd.tune_get("last_batch_kernel") else "k_solve_single"
        finally:
            L.pqp_tune_batch_converge(prev)
            pqp_amd.tune("pipe_off", prev_pipe)
        r["fixed"]["TBps"] = 4.0 * N * N * GB / r["fixed"]["per_iter_ms"]
        # each matrix once per iterate (what k_solve_pipe moves)
        r["infeasible"]["TBps_min_bytes"] = (4.0 * N * N + 4.0 * N * M + 4.0 * M * M) * GB / r["infeasible"]["per_iter_ms"]
        r["feasible"]["TBps_min_bytes"] = (4.0 * N * N + 4.0 * N * M + 8.0 * M * M) * GB / r["feasible"]["per_iter_ms"]
        r["prepare_ms"] = prep_ms
        out[name] = r
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:4]])
