"""configs[2] experiment: the persistent fixed-mode
launch (k_split_persist, one problem of n_dual 1024, 1000 iterations) with its
64 workgroups packed onto x XCDs (pqp_tune persist_xcds: 8 spreads them, the
default 0 means 4), alternating in one process, bits compared.  With
KNOB=converge_xcds the converge-mode launch (k_converge_persist, capped at 2000
updates) instead.
Usage: python scripts/persist_xcd_ab.py [xcds ...]"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main():
    import os

    import numpy as np

    import pqp_amd

    knob = os.environ.get("KNOB", "persist_xcds")
    arms = [int(a) for a in sys.argv[1:]] or ([8, 4, 3] if knob == "persist_xcds" else [0, 7, 6])
    N, iters = 1024, 1000
    M = N // 2
    if knob == "persist_xcds":
        b = pqp_amd.Batch(1, N).generate(seed=1, inst0=0, M=M)
        P = dict(Qd=b.qd_rowmajor(0), Fd=b.Fd[0, :N].cpu().numpy(), Md=b.Md[:1].cpu().numpy(),
                 Qp=np.zeros(M * M, np.float32), Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32),
                 Mp=np.zeros(1, np.float32), Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32), N=N, M=M)
        kw, path, per = dict(mode=pqp_amd.MODE_FIXED, num_iter=iters), 1, iters
    else:  # converge mode: the single_converge leg's problem, capped at 2000 updates
        pb = pqp_amd.ProblemBatch.synthetic(1, 0, 1, N)
        P = pb.problem(0)
        del pb
        kw, path, per = dict(max_updates=2000), 3, 2001
    res = {a: [] for a in arms}
    ref, same = None, {}
    with pqp_amd.Problem(P) as prob:
        for _ in range(6):
            for a in arms:
                old = pqp_amd.tune(knob, a)
                try:
                    t0 = time.perf_counter()
                    r = prob.solve(**kw)
                    res[a].append((time.perf_counter() - t0) / per * 1e6)
                    assert pqp_amd.tune_get("last_path") == path, ("not the persistent launch", pqp_amd.tune_get("last_path"))
                finally:
                    pqp_amd.tune(knob, old)
                y = np.asarray(r["Y"], np.float32).view(np.uint32)
                ref = y if ref is None else ref
                same[a] = same.get(a, True) and bool(np.array_equal(y, ref))
    print(json.dumps({"knob": knob, **{f"{knob}_{a}": {"us_per_update_median": float(np.median(v[1:])),
                                                        "all": [round(x, 4) for x in v], "bit_identical": same[a]}
                                         for a, v in res.items()}}))


if __name__ == "__main__":
    main()
