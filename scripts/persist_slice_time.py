"""configs[2] slice-size A/B: one library build (PQP_LIB=ab/libpqp_NAME.so from
scripts/build_variant.sh NAME pqp_persist "-DPQP_PERSIST_SLICES=P0,P1,PW"), the
persistent fixed-mode launch of one n_dual 1024 problem, 1000 iterations,
median of 6 solves, and a hash of Y* so that builds can be checked bit for bit.
Usage: PQP_LIB=... python scripts/persist_slice_time.py NAME"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main():
    import numpy as np

    import pqp_amd

    N, iters = 1024, 1000
    M = N // 2
    b = pqp_amd.Batch(1, N).generate(seed=1, inst0=0, M=M)
    P = dict(Qd=b.qd_rowmajor(0), Fd=b.Fd[0, :N].cpu().numpy(), Md=b.Md[:1].cpu().numpy(),
             Qp=np.zeros(M * M, np.float32), Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32),
             Mp=np.zeros(1, np.float32), Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32), N=N, M=M)
    ts = []
    with pqp_amd.Problem(P) as prob:
        for _ in range(7):
            t0 = time.perf_counter()
            r = prob.solve(mode=pqp_amd.MODE_FIXED, num_iter=iters)
            ts.append((time.perf_counter() - t0) / iters * 1e6)
            assert pqp_amd.tune_get("last_path") == 1
    y = np.asarray(r["Y"], np.float32)
    print(json.dumps({"build": sys.argv[1] if len(sys.argv) > 1 else os.environ.get("PQP_LIB", "default"),
                      "us_per_update_median": float(np.median(ts[1:])), "all": [round(t, 4) for t in ts],
                      "y_sha": hashlib.sha256(y.tobytes()).hexdigest()[:16]}))


if __name__ == "__main__":
    main()
