"""Phase timeline of k_solve_pipe (pqp_tune_trace "mid" buffer format): the
bench's batch_converge workload (n_dual 1024, M 512, 4096 problems), capped
at K updates; per traced workgroup the shader cycles of phase X (update,
U = -Qp_inv tM), phase Y (the pass over Gp) and the costs/decision, summed
over iterations.  Prints one JSON line per case (infeasible, feasible).
Usage: python scripts/pipe_trace.py [K]"""
from __future__ import annotations

import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(K=8):
    import numpy as np
    import torch

    import pqp_amd

    B, ntr = 4096, 256
    pb = pqp_amd.ProblemBatch.synthetic(3, 0, B, 1024, 512)
    pb.solve(max_updates=1)
    buf = torch.zeros(ntr * 16, dtype=torch.int64, device="cuda")
    for case in ("infeasible", "feasible"):
        if case == "feasible":
            pb.Kp.fill_(1e30)
        buf.zero_()
        pqp_amd._check(pqp_amd.lib().pqp_tune_trace(b"mid", C.c_void_p(buf.data_ptr()), ntr))
        try:
            pb.solve(max_updates=K)
            torch.cuda.synchronize()
        finally:
            pqp_amd.lib().pqp_tune_trace(b"mid", None, 0)
        T = buf.view(ntr, 16).cpu().numpy().astype(np.float64)
        it = T[:, 4]
        ok = it > 0
        per = lambda c: float(np.median(T[ok, c] / it[ok]))  # noqa: E731
        print(json.dumps({"case": case, "K": K, "kernel": "k_solve_pipe" if pqp_amd.tune_get("last_batch_kernel")
                          else "k_solve_single", "iters": float(np.median(it[ok])), "cyc_X": per(0),
                          "cyc_Y": per(1), "cyc_cost": per(2)}), flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:2]])
