"""configs[2] A/B: the persistent fixed-mode launch of one
n_dual 1024 problem, 1000 iterations, in its split form (64 workgroups over 4
XCDs, sc1 granules: the default) and its one-XCD lean form (32
workgroups, Qd in LDS, plain granule stores: persist_lean 1), alternating in
one process, bits compared.  Usage: python scripts/persist_lean_ab.py [reps]"""
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

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N, iters = 1024, 1000
    M = N // 2
    b = pqp_amd.Batch(1, N).generate(seed=1, inst0=0, M=M)
    P = dict(Qd=b.qd_rowmajor(0), Fd=b.Fd[0, :N].cpu().numpy(), Md=b.Md[:1].cpu().numpy(),
             Qp=np.zeros(M * M, np.float32), Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32),
             Mp=np.zeros(1, np.float32), Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32), N=N, M=M)
    # name: (persist_lean, persist_lean_flags, last_path, bits expected equal to split)
    arms = {"split": (0, 0, 1, True), "lean": (1, 0, 6, True), "lean_sc1": (1, 1, 6, True),
            "lean_spread": (1, 2, 6, True), "lean_nodiag": (1, 4, 6, False)}
    res = {a: [] for a in arms}
    ys = {}
    with pqp_amd.Problem(P) as prob:
        for _ in range(reps):
            for a, (knob, flags, path, _) in arms.items():
                old = pqp_amd.tune("persist_lean", knob)
                oldf = pqp_amd.tune("persist_lean_flags", flags)
                try:
                    t0 = time.perf_counter()
                    r = prob.solve(mode=pqp_amd.MODE_FIXED, num_iter=iters)
                    res[a].append((time.perf_counter() - t0) / iters * 1e6)
                    got = pqp_amd.tune_get("last_path")
                    assert got == path, (a, got)
                finally:
                    pqp_amd.tune("persist_lean", old)
                    pqp_amd.tune("persist_lean_flags", oldf)
                ys[a] = np.asarray(r["Y"], np.float32).view(np.uint32).copy()
    out = {a: {"us_per_update_median": float(np.median(v[1:])), "all": [round(x, 4) for x in v]} for a, v in res.items()}
    for a, (_, _, _, exact) in arms.items():
        out[a]["bit_identical_to_split"] = bool(np.array_equal(ys["split"], ys[a]))
        assert out[a]["bit_identical_to_split"] or not exact, a
    print(json.dumps(out))


if __name__ == "__main__":
    main()
