"""configs[2] converge-mode A/B across library builds (PQP_LIB=ab/libpqp_NAME.so
from scripts/build_variant.sh NAME pqp_converge "-D..."): the persistent
pipelined launch (k_converge_persist) on the single_converge leg's problem,
capped at 2000 updates, median of 5 solves, and a hash of Y* / U* so that
builds can be checked bit for bit.  Usage: PQP_LIB=... python scripts/converge_build_time.py NAME"""
from __future__ import annotations

import hashlib
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main():
    import numpy as np

    import pqp_amd

    N = 1024
    pb = pqp_amd.ProblemBatch.synthetic(1, 0, 1, N)
    P = pb.problem(0)
    del pb
    ts = []
    with pqp_amd.Problem(P) as prob:
        for _ in range(6):
            t0 = time.perf_counter()
            r = prob.solve(max_updates=2000)
            ts.append((time.perf_counter() - t0) / 2001 * 1e6)
            assert pqp_amd.tune_get("last_path") == 3
    h = hashlib.sha256(np.asarray(r["Y"], np.float32).tobytes() + np.asarray(r["U"], np.float32).tobytes())
    print(json.dumps({"build": sys.argv[1] if len(sys.argv) > 1 else "default", "us_per_iter_median": float(np.median(ts[1:])),
                      "all": [round(t, 4) for t in ts], "h": int(r["h"]), "yu_sha": h.hexdigest()[:16]}))


if __name__ == "__main__":
    main()
