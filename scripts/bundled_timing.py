"""Time the bundled example (BASELINE configs[1]) through the C ABI: the
problem is uploaded once; each solve is one pqp_problem_solve call (launch,
synchronisation, results on the host).  Forms, alternating in one process:
  new    k_fixed_one (sparse form where the split rows allow) / k_solve_quintet,
         results written by the kernel to pinned host memory
  np4    k_solve_quintet with four B and four C waves (the default: three of
         each since round 6)
  apoll  the update wave reads the decision word every update (default: only
         when its ring is full); np2_apoll is round 5's kernel
  dense  k_fixed_one's dense form only (pqp_tune tiny_dense)
  old    the round-4 k_fixed_tiny / k_solve_wave with state copies (tiny_old)
Each solve's bits are checked against tests/golden/bundled.npz.  Run under
rocprofv3 --kernel-trace --stats to split kernel time from launch/readback."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))

FORMS = {"new": {}, "ablk1": {"tiny_ablk": 1}, "apoll": {"tiny_apoll": 1}, "np4": {"tiny_np": 4}}


def main(reps: int = 200, rounds: int = 3):
    import pqp_amd

    g = np.load(ROOT / "tests" / "golden" / "bundled.npz")
    P = pqp_amd.example_problem(ROOT / "tests" / "golden" / "example")
    modes = (("fixed1000", dict(mode=pqp_amd.MODE_FIXED, num_iter=1000)), ("converge", dict(max_updates=200000)))
    out = {f"{m}_{f}": [] for m, _ in modes for f in FORMS}
    bits = {}
    with pqp_amd.Problem(P) as prob:
        for _ in range(rounds):
            for form, knobs in FORMS.items():
                old = {k: pqp_amd.tune(k, v) for k, v in knobs.items()}
                try:
                    for name, kw in modes:
                        r = prob.solve(**kw)
                        t0 = time.perf_counter()
                        for _ in range(reps):
                            r = prob.solve(**kw)
                        dt = (time.perf_counter() - t0) / reps
                        out[f"{name}_{form}"].append(dt * 1e3)
                        if name == "fixed1000":
                            ok = r["Y"].tobytes() == g["Y_fixed999"].tobytes() and r["h"] == 1000
                        else:
                            ok = (r["Y"].tobytes() == g["Ystar"].tobytes() and r["U"].tobytes() == g["Ustar"].tobytes()
                                  and r["h"] == int(g["h"]) and np.float32(r["Jp"]) == g["Jp"] and np.float32(r["Jd"]) == g["Jd"])
                        bits[f"{name}_{form}"] = bits.get(f"{name}_{form}", True) and bool(ok)
                finally:
                    for k, v in old.items():
                        pqp_amd.tune(k, v)
    res = {k: {"ms_per_solve_median": float(np.median(v)), "ms_all": [round(x, 4) for x in v],
               "bit_exact": bits[k]} for k, v in out.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
