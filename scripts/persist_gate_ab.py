"""A/B of a tuning word of the persistent fixed-mode launch, read from the
environment at each launch of pqp_persist.hip (variable named by
PERSIST_AB_ENV, default PQP_PERSIST_SWEEP): n_dual 1024, 1000 iterations,
variants interleaved in one process, every variant's Y checked bit for bit
against the first.  Usage: python scripts/persist_gate_ab.py [value ...]"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
AB_ENV = os.environ.get("PERSIST_AB_ENV", "PQP_PERSIST_SWEEP")
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main():
    import numpy as np

    import pqp_amd

    gates = [int(a, 0) for a in sys.argv[1:]] or [0]
    N, iters = 1024, 1000
    M = N // 2
    b = pqp_amd.Batch(1, N).generate(seed=1, inst0=0, M=M)
    P = dict(Qd=b.qd_rowmajor(0), Fd=b.Fd[0, :N].cpu().numpy(), Md=b.Md[:1].cpu().numpy(),
             Qp=np.zeros(M * M, np.float32), Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32),
             Mp=np.zeros(1, np.float32), Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32), N=N, M=M)
    L = pqp_amd.lib()
    res = {g: [] for g in gates}
    ref = None
    same = {}
    with pqp_amd.Problem(P) as prob:
        for rep in range(5):
            for g in gates:
                os.environ[AB_ENV] = str(g)
                t0 = time.perf_counter()
                r = prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
                res[g].append((time.perf_counter() - t0) / (iters - 1) * 1e6)
                assert L.pqp_tune_last_path(None) == 1, "not the persistent launch"
                y = np.asarray(r["Y"], np.float32).view(np.uint32)
                if ref is None:
                    ref = y
                same[g] = same.get(g, True) and bool(np.array_equal(y, ref))
    os.environ.pop(AB_ENV, None)
    out = {f"gate_{g:#x}": {"us_per_update_median": float(np.median(v[1:])), "all": v, "bit_identical": same[g]}
           for g, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
