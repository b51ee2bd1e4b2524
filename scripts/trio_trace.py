"""Per-wave shader clocks of k_solve_quintet on the bundled example (configs[1],
converge mode): each wave's total clocks, the clocks it spent waiting on its
producer (or, wave A, on the ring's room) and its iterates.  The wave that
never waits is the bound."""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(reps: int = 5):
    import torch

    import pqp_amd

    L = pqp_amd.lib()
    P = pqp_amd.example_problem(ROOT / "tests" / "golden" / "example")
    buf = torch.zeros(24, dtype=torch.int64, device="cuda")
    out = []
    with pqp_amd.Problem(P) as prob:
        for _ in range(reps):
            assert L.pqp_tune_trace(b"tiny", buf.data_ptr(), 1) == 0
            r = prob.solve(max_updates=200000)
            assert L.pqp_tune_trace(b"tiny", None, 0) == 0
            t = buf.cpu().numpy()[:20].reshape(5, 4)
            ph = buf.cpu().numpy()[20:24]
            out.append({w: {"clk": int(t[k, 0]), "wait_clk": int(t[k, 1]), "iterates": int(t[k, 2]),
                            "busy_clk_per_iterate": float((t[k, 0] - t[k, 1]) / max(1, t[k, 2]))}
                        for k, w in enumerate(("A_update", "B0_even", "C0_even", "C1_odd", "B1_odd"))})
            out[-1]["h"] = r["h"]
            out[-1]["B0_phase_clk_per_own_iterate"] = {k: float(2 * v / r["h"]) for k, v in
                                                  zip(("wait", "y_reads_products_sum", "t_q_readlanes", "s2_publish"), ph)}
    print(json.dumps(out[-1]))
    print(json.dumps({"clk_per_iterate_total": [o["A_update"]["clk"] / o["h"] for o in out]}))


if __name__ == "__main__":
    main()
