"""k_solve_pipe with the second resident workgroup of each CU started late
(pqp_tune "pipe_stagger", shader cycles): the bench's batch_converge shape
(4096 problems, n_dual 1024, M 512), steady state per iteration = (time of a
3K-update call - time of a K-update call) / 2K, infeasible iterates and every
iterate feasible (Kp = 1e30), arms alternating; bits compared.
Usage: python scripts/pipe_stagger_ab.py [stagger cycles, comma-separated]"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(arms):
    import torch

    import pqp_amd

    N, B, K = 1024, 4096, 8
    pb = pqp_amd.ProblemBatch.synthetic(1, 0, B, N)
    M = pb.M
    pb.prepare()

    def call(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pb.solve(max_updates=k)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    for case, alg in (("infeasible", 4.0 * N * N + 4.0 * N * M + 4.0 * M * M),
                      ("feasible", 4.0 * N * N + 4.0 * N * M + 8.0 * M * M)):
        if case == "feasible":
            pb.Kp.fill_(1e30)
        res, ys = {a: [] for a in arms}, {}
        for rep in range(2):
            for a in arms:
                old = pqp_amd.tune("pipe_stagger", a)
                try:
                    call(1)
                    per = (call(3 * K) - call(K)) / (2 * K)
                finally:
                    pqp_amd.tune("pipe_stagger", old)
                res[a].append(per)
                ys[a] = pb.Y.clone()
        out = {"case": case, "kernel": pqp_amd.tune_get("last_batch_kernel")}
        for a in arms:
            per = min(res[a])
            out[str(a)] = {"ms_per_iteration": per * 1e3, "frac_of_8TBs": alg * B / per / 8e12,
                           "same_bits": bool(torch.equal(ys[a].view(torch.int32), ys[arms[0]].view(torch.int32)))}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main([int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,300000,600000,1200000").split(",")])
