"""Diagnostic: the growing-Y problem of tests/test_gpu_mid.py (Y overflows
after ~285 updates) solved in converge mode by every path-3 form at several
caps, against the oracle's h (which is infeasible until h = 280)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))


def main():
    import pqp_amd
    from test_gpu_mid import KEYS, _growing
    from oracle import Oracle

    orc = Oracle()
    P = _growing(112, 28, 1)
    out = {}
    forms = {"pair": {"mid2_pair": 1, "mid2_min_n": 0}, "row": {"mid2_pair": 2, "mid2_min_n": 0},
             "v1": {"mid_v1": 1}, "off": {"mid_off": 1}}
    for cap in (100, 123, 124, 125, 200, 350):
        h, Y, U = orc.solve(P, max_updates=cap)
        rec = {"oracle_h": h}
        for name, kn in forms.items():
            old = {k: pqp_amd.tune(k, v) for k, v in kn.items()}
            try:
                pb = pqp_amd.ProblemBatch(1, 112, 28)
                for k in KEYS:
                    pb.set(k, np.asarray(P[k], np.float32).reshape(1, -1))
                pb.solve(max_updates=cap)
                y = pb.Y[0].cpu().numpy()
                rec[name] = {"h": int(pb.h[0]), "status": int(pb.status[0]), "kernel": pqp_amd.tune_get("last_batch_kernel"),
                             "Y_same": bool(np.array_equal(y.view(np.uint32), Y.view(np.uint32)))}
            finally:
                for k, v in old.items():
                    pqp_amd.tune(k, v)
        out[cap] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
