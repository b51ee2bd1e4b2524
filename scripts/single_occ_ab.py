"""k_solve_single builds (pqp_tune "single_occ" 0 / 4 / 5: 3, 4, 5 workgroups
per CU) on the horizon sweep's k_solve_single shapes (the plant stacked 8 and
16 times, whole solves) and the batch_converge shape with pipe_off,
alternating; bits compared.  One JSON line per case."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
sys.path.insert(0, str(ROOT / "scripts"))


def main():
    import torch

    import pqp_amd
    from problems import block_diag_problem, bundled_problem

    base = bundled_problem()
    cases = []
    import os
    for H in [int(h) for h in os.environ.get("HS", "8,16").split(",")]:
        P = block_diag_problem(base, H)
        B = min(16384, (1 << 31) // (4 * P["N"] * P["N"])) // 64 * 64
        cases.append((f"H{H}", pqp_amd.ProblemBatch.replicate(P, B), 200000))
    prev_off = pqp_amd.tune("pipe_off", 1)
    if not os.environ.get("HS"):
        cases.append(("bench_shape_infeasible_16", pqp_amd.ProblemBatch.synthetic(1, 0, 4096, 1024, 512), 16))
    try:
        for name, pb, cap in cases:
            ts, res = {3: [], 4: [], 5: []}, {}
            for rep in range(3):
                for occ in (3, 4, 5):
                    old = pqp_amd.tune("single_occ", occ)
                    try:
                        pb.solve(max_updates=cap)
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        pb.solve(max_updates=cap)
                        torch.cuda.synchronize()
                        ts[occ].append((time.perf_counter() - t0) * 1e3)
                    finally:
                        pqp_amd.tune("single_occ", old)
                    res[occ] = (pb.Y.clone(), pb.h.clone(), pqp_amd.tune_get("last_batch_kernel"))
            same = {o: bool(torch.equal(res[o][0].view(torch.int32), res[3][0].view(torch.int32)) and
                            torch.equal(res[o][1], res[3][1])) for o in res}
            print(json.dumps({"case": name, "ms": {str(o): min(v) for o, v in ts.items()}, "same_bits": same,
                              "kernel": res[3][2]}), flush=True)
    finally:
        pqp_amd.tune("pipe_off", prev_off)


if __name__ == "__main__":
    main()
