"""Phase timeline of k_solve_mid (pqp_tune_trace "mid"): the bundled plant as
H diagonal blocks, B copies; per traced workgroup the shader cycles of each
phase (A update/tM, B U, C checkFeas, D+E costs), summed over iterations,
and each wave's busy time in phase A.  Prints one JSON line per (H, mode).
Usage: python scripts/mid_trace.py [H ...]   (MODES=fixed,infeasible,feasible)"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
sys.path.insert(0, str(ROOT / "scripts"))


def main(Hs):
    import ctypes as C

    import numpy as np
    import torch

    import pqp_amd
    from problems import block_diag_problem, bundled_problem

    base = bundled_problem()
    pqp_amd.tune("mid_v1", int(os.environ.get("MID_V1", "0")))
    pqp_amd.tune("mid2_pair", int(os.environ.get("MID2_PAIR", "0")))  # 0 by shape, 1 lane sides, 2 one lane per row
    pqp_amd.tune("mid2_min_n", 0)
    B = int(os.environ.get("B", "4096"))
    ntr = 256
    buf = torch.zeros(ntr * 16, dtype=torch.int64, device="cuda")
    for H in Hs:
        if isinstance(H, str):  # dN: bench.py's dense companion at n_dual N (feasible mode only)
            sys.path.insert(0, str(ROOT))
            from bench import DENSE_SIZES, dense_horizon_batch

            pb = dense_horizon_batch(pqp_amd, int(H[1:]), dict(DENSE_SIZES)[int(H[1:])], B)
            P = {"N": int(H[1:])}
        else:
            P = block_diag_problem(base, H)
            pb = pqp_amd.ProblemBatch.replicate(P, B)
        for mode in os.environ.get("MODES", "fixed,infeasible,feasible").split(","):
            if not isinstance(H, str):
                pb.Kp.copy_(torch.as_tensor(np.tile(P["Kp"], (B, 1)), device=pb.device))
            if mode == "infeasible":
                pb.Kp.fill_(-1e30)
            buf.zero_()
            pqp_amd._check(pqp_amd.lib().pqp_tune_trace(b"mid", C.c_void_p(buf.data_ptr()), ntr))
            try:
                if mode == "fixed":
                    pb.solve(pqp_amd.MODE_FIXED, num_iter=314)
                else:
                    pb.solve(max_updates=312 if (mode == "infeasible" or isinstance(H, str)) else 200000)
                torch.cuda.synchronize()
            finally:
                pqp_amd.lib().pqp_tune_trace(b"mid", None, 0)
            T = buf.view(ntr, 16).cpu().numpy().astype(np.float64)
            it = T[:, 4]
            ok = it > 0
            per = lambda c: float(np.median(T[ok, c] / it[ok]))  # noqa: E731
            print(json.dumps({"H": H, "n_dual": P["N"], "mode": mode, "iters": float(np.median(it[ok])),
                              "cyc_A": per(0), "cyc_B": per(1), "cyc_C": per(2), "cyc_DE": per(3),
                              # k_solve_mid2: T's Gp'Y part, C0's checkFeas part, the cost wave's U'Qp part
                              "m2_seg": {"T_gpy": per(1), "C0_checkfeas": per(2), "cost_uqp": per(3)},
                              "busyA_wave": [per(8 + w) for w in range(8)]}), flush=True)
        del pb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main([a if a.startswith("d") else int(a) for a in sys.argv[1:]] or [2, 4, 5])
