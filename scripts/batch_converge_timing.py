"""Batched converge mode at scale: pqp_batch_solve over B
synthetic problems (n_dual N, M = N/2; the bench workload's generator, primal
kept for terminate()), capped at K updates: instance-iterations/s where one
iteration is the reference loop body, terminate() + updateY2
(PQP_CPU.c:716-725).  Usage: python scripts/batch_converge_timing.py [N B K]"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(N=1024, B=4096, K=8):
    import torch

    import pqp_amd

    t0 = time.perf_counter()
    pb = pqp_amd.ProblemBatch.synthetic(1, 0, B, N)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    L = pqp_amd.lib()
    M = pb.M
    out = {"n_dual": N, "m": M, "problems": B, "updates": K, "setup_s": setup}
    ys = {}
    for name, opts in (("default", 0), ("fused", 1), ("scalar_loads", 4), ("default_again", 0), ("fused_again", 1),
                       ("transposes", 2)):
        prev = L.pqp_tune_batch_converge(opts)
        pb.solve(max_updates=1)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pb.solve(max_updates=K)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        L.pqp_tune_batch_converge(prev)
        h = pb.h.cpu()
        ys[name] = pb.Y.clone()
        # bytes per iteration: the update's Qd, Gp twice (Gp'Y, Gp U: 8NM),
        # Qp_inv -- terminate() of these (infeasible) iterates stops at checkFeas
        alg = 4.0 * N * N + 8.0 * N * M + 4.0 * M * M  # infeasible iterates: no Y'Qd, no U'Qp
        out[name] = {"ms": dt * 1e3, "instance_iter_per_s": B * K / dt, "alg_bytes_per_iter": alg,
                     "alg_GBps": alg * B * K / dt / 1e9, "h_all": int(h.min()) == int(h.max()) == K + 1}
    out["bit_identical"] = all(bool(torch.equal(ys["default"].view(torch.int32), v.view(torch.int32)))
                               for v in ys.values())
    out["speedup_vs_scalar_loads"] = out["scalar_loads"]["ms"] / out["default"]["ms"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:4]])
