"""Time the bundled example (BASELINE configs[1]) through the C ABI: the
problem is uploaded once; each solve is one pqp_problem_solve call.  Run under
rocprofv3 --kernel-trace --stats to split kernel time from launch/readback."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(reps: int = 50):
    import pqp_amd

    P = pqp_amd.example_problem(ROOT / "tests" / "golden" / "example")
    out = {}
    with pqp_amd.Problem(P) as prob:
        for name, kw in (("fixed1000", dict(mode=pqp_amd.MODE_FIXED, num_iter=1000)), ("converge", dict(max_updates=200000))):
            prob.solve(**kw)
            t0 = time.perf_counter()
            for _ in range(reps):
                r = prob.solve(**kw)
            dt = (time.perf_counter() - t0) / reps
            out[name] = {"ms_per_solve": dt * 1e3, "h": r["h"], "iter_per_s": (r["h"] - 1 if name == "fixed1000" else r["h"]) / dt}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
