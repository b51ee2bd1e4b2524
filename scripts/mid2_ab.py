"""Path 3 A/B: k_solve_mid2 (terminate(Y_h) beside the update to Y_{h+1},
lane-pair rows) against k_solve_mid (pqp_tune("mid_v1", 1)), same process,
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
sys.path.insert(0, str(ROOT / "oracle"))


def main(Hs):
    import torch

    import pqp_amd
    from oracle import Oracle, block_diag_problem

    base = Oracle().bundled_problem(ROOT / "tests" / "golden" / "example")
    B = int(os.environ.get("B", "16384"))
    for H in Hs:
        P = block_diag_problem(base, H)
        pb = pqp_amd.ProblemBatch.replicate(P, B)
        out = {"H": H, "n_dual": P["N"], "m": P["M"], "problems": B}
        res = {}
        for mode in ("converge", "fixed"):
            ts = {"mid2": [], "v1": []}
            for rep in range(2):
                for name, v1 in (("mid2", 0), ("v1", 1)):
                    old = pqp_amd.tune("mid_v1", v1)
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
                    res[(mode, name)] = (pb.Y.clone(), pb.U.clone(), pb.h.clone(), kern)
            a, b = res[(mode, "mid2")], res[(mode, "v1")]
            out[mode] = {"mid2_ms": min(ts["mid2"]), "v1_ms": min(ts["v1"]), "speedup": min(ts["v1"]) / min(ts["mid2"]),
                         "kernels": [a[3], b[3]],
                         "same_bits": bool(torch.equal(a[0].view(torch.int32), b[0].view(torch.int32)) and
                                           torch.equal(a[1].view(torch.int32), b[1].view(torch.int32)) and
                                           torch.equal(a[2], b[2])),
                         "all_h_313": bool((a[2] == 313).all()) if mode == "converge" else None}
        print(json.dumps(out), flush=True)
        del pb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [2, 3, 4, 5])
