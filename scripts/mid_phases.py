"""Where k_solve_mid's time goes: the bundled plant as H diagonal blocks, B
copies, timed three ways -- fixed mode (the update alone), converge mode with
every iterate infeasible (Kp = -1e30: the update beside tM, U, checkFeas),
and the real solve (every iterate feasible: all of computeCost as well) --
as microseconds per iteration per workgroup (resident workgroups per CU
from the LDS footprint).  Usage: python scripts/mid_phases.py [H ...]"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
sys.path.insert(0, str(ROOT / "scripts"))


def timed(pb, torch, **kw):
    pb.solve(**kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pb.solve(**kw)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main(Hs):
    import numpy as np
    import torch

    import pqp_amd
    from problems import block_diag_problem, bundled_problem

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    base = bundled_problem()
    for H in Hs:
        P = block_diag_problem(base, H)
        N, M = P["N"], P["M"]
        B = 16384
        iters = 313
        lds = 4 * (N * (N | 1) + (N + 2 * M) * (M | 1) + 10 * N + 5 * M)
        per_cu = max(1, min(8, (160 * 1024) // lds))
        slots = cus * per_cu
        out = {"H": H, "n_dual": N, "m": M, "batch": B, "path": pqp_amd.lib().pqp_batch_solve_path(N, M),
               "wg_per_cu_est": per_cu}
        pb = pqp_amd.ProblemBatch.replicate(P, B)
        t = timed(pb, torch, mode=pqp_amd.MODE_FIXED, num_iter=iters + 1)
        out["fixed_us_per_iter_wg"] = t / (iters * B / slots) * 1e6
        t = timed(pb, torch, max_updates=200000)
        assert int(pb.h.min()) == iters
        out["feasible_us_per_iter_wg"] = t / (iters * B / slots) * 1e6
        pb.Kp.fill_(-1e30)
        t = timed(pb, torch, max_updates=iters - 1)
        out["infeasible_us_per_iter_wg"] = t / (iters * B / slots) * 1e6
        print(json.dumps(out), flush=True)
        del pb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [2, 4])
