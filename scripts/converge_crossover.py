"""Converge-mode time per iteration below the wide-path threshold: the default
routing (one-wave / one-workgroup solvers) vs the persistent pipelined launch
(pqp_converge.hip), capped synthetic solves, bit-identical results checked."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main():
    import numpy as np

    import pqp_amd

    L = pqp_amd.lib()
    cap = 2000
    for N in [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "32,48,64,96,128,160,192,256,320,383").split(",")]:
        M = max(1, N // 2)
        pb = pqp_amd.ProblemBatch.synthetic(1, 0, 1, N, M)
        P = pb.problem(0)
        del pb
        out = {"n_dual": N, "m": M}
        res = {}
        with pqp_amd.Problem(P) as prob:
            for name, min_n in (("default", 384), ("persistent", 0)):
                L.pqp_tune_wide_min_n(min_n)
                prob.solve(max_updates=2)
                best = None
                for _ in range(3):
                    t0 = time.perf_counter()
                    r = prob.solve(max_updates=cap)
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                out[name + "_us_per_iter"] = best / r["h"] * 1e6
                res[name] = r
            L.pqp_tune_wide_min_n(384)
        out["h"] = res["default"]["h"]
        out["bit_identical"] = bool(np.array_equal(res["default"]["Y"].view(np.uint32),
                                                   res["persistent"]["Y"].view(np.uint32)))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
