"""k_solve_mid2 build arms on the horizon sweep (16384 copies of the
bundled plant over H stages, converge mode to h = 313): knob sets applied in
turn, alternating, two rounds; the fastest time of each, bits compared with
k_solve_mid.  One JSON line per H.
Usage: python scripts/mid2_arms.py [H ...]"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
sys.path.insert(0, str(ROOT / "scripts"))

ARMS = {
    "def": {},
    "pair_lean": {"mid2_pair": 1},
    "row_lean": {"mid2_pair": 2},
    "v1": {"mid_v1": 1},
    "mid2": {"mid2_min_n": 0},
    "packed": {"mid2_min_n": 0, "mid2_pair": 2},
    "pair": {"mid2_min_n": 0, "mid2_pair": 1},
}


def main(Hs):
    import torch

    import pqp_amd
    from problems import block_diag_problem, bundled_problem

    base = bundled_problem()
    B = int(os.environ.get("B", "16384"))
    arms = os.environ.get("ARMS", ",".join(ARMS)).split(",")
    for H in Hs:
        P = block_diag_problem(base, H)
        pb = pqp_amd.ProblemBatch.replicate(P, B)
        ts = {a: [] for a in arms}
        res = {}
        for rep in range(2):
            for a in arms:
                old = {k: pqp_amd.tune(k, v) for k, v in ARMS[a].items()}
                try:
                    if rep == 0:
                        pb.solve(max_updates=200000)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    pb.solve(max_updates=200000)
                    torch.cuda.synchronize()
                    ts[a].append((time.perf_counter() - t0) * 1e3)
                    kern = pqp_amd.tune_get("last_batch_kernel")
                finally:
                    for k, v in old.items():
                        pqp_amd.tune(k, v)
                res[a] = (pb.Y.clone(), pb.U.clone(), pb.h.clone(), kern)
        ref = res[arms[0]]
        same = {a: bool(torch.equal(res[a][0].view(torch.int32), ref[0].view(torch.int32)) and
                        torch.equal(res[a][1].view(torch.int32), ref[1].view(torch.int32)) and
                        torch.equal(res[a][2], ref[2])) for a in arms}
        print(json.dumps({"H": H, "n_dual": P["N"], "problems": B, "ms": {a: min(ts[a]) for a in arms},
                          "kernel": {a: res[a][3] for a in arms}, "same_bits_as_" + arms[0]: same,
                          "all_h_313": bool((ref[2] == 313).all())}), flush=True)
        del pb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [2, 3, 4, 5])
