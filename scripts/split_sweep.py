"""Per-update time of the single-problem split path vs n_dual (hipGraph
replays of pqp_problem_solve in fixed mode), to separate the fixed cost of
an update (launch, y staging, hand-offs) from the per-k cost."""
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

    sizes = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "100,128,256,512,768,1024,1536,2048").split(",")]
    iters = 400
    for N in sizes:
        M = max(1, N // 2)
        b = pqp_amd.Batch(1, N).generate(seed=1, inst0=0, M=M)
        P = dict(Qd=b.qd_rowmajor(0), Fd=b.Fd[0, :N].cpu().numpy(), Md=b.Md[:1].cpu().numpy(),
                 Qp=np.zeros(M * M, np.float32), Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32),
                 Mp=np.zeros(1, np.float32), Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32), N=N, M=M)
        with pqp_amd.Problem(P) as prob:
            prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
            t0 = time.perf_counter()
            for _ in range(3):
                prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
            dt = (time.perf_counter() - t0) / 3
        print(json.dumps({"n_dual": N, "us_per_update": dt / (iters - 1) * 1e6}), flush=True)


if __name__ == "__main__":
    main()
