"""Converge-mode time per iteration of ONE synthetic problem: the persistent
pipelined launch (pqp_converge.hip) vs the graph-replayed launch chain
(pqp_wide.hip).  Capped solves (the synthetic problems do not converge at
these sizes); bit-identical results checked.  Also the converging testing/
sample test2 (n_dual 400, h = 3) per solve."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "pqp-for-mpc_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))


def main():
    import numpy as np

    import pqp_amd

    sizes = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "384,512,768,1024").split(",")]
    caps = (200, 2000)
    L = pqp_amd.lib()
    for N in sizes:
        M = N // 2
        pb = pqp_amd.ProblemBatch.synthetic(1, 0, 1, N, M)
        P = pb.problem(0)
        del pb
        out = {"n_dual": N, "m": M}
        res = {}
        with pqp_amd.Problem(P) as prob:
            for name, off in (("persistent", 0), ("graph_chain", 1)):
                L.pqp_tune_converge_persist(off)
                prob.solve(max_updates=2)
                for cap in caps:
                    best = None
                    for _ in range(3):
                        t0 = time.perf_counter()
                        r = prob.solve(max_updates=cap)
                        dt = time.perf_counter() - t0
                        best = dt if best is None else min(best, dt)
                    out[f"{name}_cap{cap}"] = {"ms": best * 1e3, "us_per_iter": best / (cap + 1) * 1e6}
                    res[(name, cap)] = r
            L.pqp_tune_converge_persist(0)
        out["bit_identical"] = all(
            np.array_equal(res[("persistent", c)]["Y"].view(np.uint32), res[("graph_chain", c)]["Y"].view(np.uint32))
            and np.array_equal(res[("persistent", c)]["U"].view(np.uint32),
                               res[("graph_chain", c)]["U"].view(np.uint32)) for c in caps)
        c = caps[-1]
        out["speedup"] = out[f"graph_chain_cap{c}"]["us_per_iter"] / out[f"persistent_cap{c}"]["us_per_iter"]
        print(json.dumps(out), flush=True)
    # a converging reference problem (h = 3)
    import tempfile

    from test_gpu_wide import _testing_file

    with tempfile.TemporaryDirectory() as td:
        P = pqp_amd.testfile_problem(_testing_file("test2.txt", Path(td)))
    out = {"problem": "testing/test2.txt", "n_dual": int(P["N"]), "m": int(P["M"])}
    with pqp_amd.Problem(P) as prob:
        for name, off in (("persistent", 0), ("graph_chain", 1)):
            L.pqp_tune_converge_persist(off)
            prob.solve(max_updates=100000)
            t0 = time.perf_counter()
            for _ in range(10):
                r = prob.solve(max_updates=100000)
            out[name] = {"h": r["h"], "ms_per_solve": (time.perf_counter() - t0) / 10 * 1e3}
        L.pqp_tune_converge_persist(0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
