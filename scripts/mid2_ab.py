"""Path 3 A/B: k_solve_mid2 (terminate(Y_h) beside the update to Y_{h+1}; one
lane per row, and "pair": lane-side rows) against k_solve_mid
(pqp_tune("mid_v1", 1)), every size forced through each (mid2_min_n 0), same process,
alternating: the bundled plant as H diagonal blocks, B copies, converge mode
to the reference's h = 313 (every iterate feasible), and fixed mode (314
iterations); bits compared.  One JSON line per H.
Usage: python scripts/mid2_ab.py [H ...]   (B env, default 16384)"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
sys.path.insert(0, str(ROOT / "scripts"))


def main(Hs):
    import torch

    import pqp_amd
    from problems import block_diag_problem, bundled_problem

    base = bundled_problem()
    B = int(os.environ.get("B", "16384"))
    for H in Hs:
        P = block_diag_problem(base, H)
        pb = pqp_amd.ProblemBatch.replicate(P, B)
        out = {"H": H, "n_dual": P["N"], "m": P["M"], "problems": B}
        res = {}
        for mode in ("converge", "fixed"):
            arms = (("mid2", 0, 2), ("pair", 0, 1), ("v1", 1, 0))
            ts = {a[0]: [] for a in arms}
            for rep in range(2):
                for name, v1, pair in arms:
                    old = pqp_amd.tune("mid_v1", v1)
                    oldp = pqp_amd.tune("mid2_pair", pair)
                    oldn = pqp_amd.tune("mid2_min_n", 0)
                    try:
                        run = (lambda: pb.solve(max_updates=200000)) if mode == "converge" else \
                            (lambda: pb.solve(pqp_amd.MODE_FIXED, num_iter=314))
                        if rep == 0:
                            run()
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        run()
                        torch.cuda.synchronize()
                        ts[name].append((time.perf_counter() - t0) * 1e3)
                        kern = pqp_amd.tune_get("last_batch_kernel")
                    finally:
                        pqp_amd.tune("mid_v1", old)
                        pqp_amd.tune("mid2_pair", oldp)
                        pqp_amd.tune("mid2_min_n", oldn)
                    res[(mode, name)] = (pb.Y.clone(), pb.U.clone(), pb.h.clone(), kern)
            a, b, c = res[(mode, "mid2")], res[(mode, "v1")], res[(mode, "pair")]
            same = lambda x, y: bool(torch.equal(x[0].view(torch.int32), y[0].view(torch.int32)) and  # noqa: E731
                                     torch.equal(x[1].view(torch.int32), y[1].view(torch.int32)) and torch.equal(x[2], y[2]))
            out[mode] = {"mid2_ms": min(ts["mid2"]), "pair_ms": min(ts["pair"]), "v1_ms": min(ts["v1"]),
                         "speedup": min(ts["v1"]) / min(ts["mid2"]), "kernels": [a[3], c[3], b[3]],
                         "same_bits": same(a, b) and same(c, b),
                         "all_h_313": bool((a[2] == 313).all()) if mode == "converge" else None}
        print(json.dumps(out), flush=True)
        del pb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [2, 3, 4, 5])
