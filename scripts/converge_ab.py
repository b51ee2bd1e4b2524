"""Converge-mode A/B of one library build (PQP_LIB) on the persistent
pipelined launch: one synthetic problem (n_dual 1024 by default, M = n/2),
capped at 2000 iterations, median of 5 solves; prints us/iteration and a
digest of Y*, U* so that builds can be checked bit for bit against each other.
Usage: PQP_LIB=ab/libpqp_x.so python scripts/converge_ab.py [N]"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(N: int = 1024, cap: int = 2000):
    import numpy as np

    import pqp_amd

    M = N // 2
    pb = pqp_amd.ProblemBatch.synthetic(1, 0, 1, N, M)
    P = pb.problem(0)
    del pb
    if os.environ.get("CONVERGE_AB_FEASIBLE"):
        # every iterate feasible (Kp far above any Gp U): computeCost's four
        # dots run on every iterate (the synthetic problem is infeasible)
        P["Kp"] = np.full_like(np.asarray(P["Kp"], np.float32), 1e30)
    L = pqp_amd.lib()
    ts = []
    with pqp_amd.Problem(P) as prob:
        prob.solve(max_updates=2)
        for _ in range(5):
            t0 = time.perf_counter()
            r = prob.solve(max_updates=cap)
            ts.append((time.perf_counter() - t0) / (cap + 1) * 1e6)
        assert L.pqp_tune_last_path(None) == 3, "not the persistent converge launch"
        # the launch's fixed cost: a 200-iteration solve beside the 2000 one
        t200 = []
        for _ in range(5):
            t0 = time.perf_counter()
            prob.solve(max_updates=200)
            t200.append(time.perf_counter() - t0)
        slope = (np.median(ts) * (cap + 1) * 1e-6 - np.median(t200)) / (cap - 200) * 1e6
        fixed_us = np.median(t200) * 1e6 - 201 * slope
    h = hashlib.sha256(np.asarray(r["Y"], np.float32).tobytes() + np.asarray(r["U"], np.float32).tobytes())
    print(json.dumps({"n_dual": N, "median_us_per_iter": float(np.median(ts)), "all": ts, "h": r["h"],
                      "slope_us_per_iter": float(slope), "per_solve_fixed_us": float(fixed_us),
                      "digest": h.hexdigest()[:16]}))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
