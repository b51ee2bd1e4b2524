"""The bench's horizon workload (16384 MPC problems stacked H horizon stages,
seed 7, converge mode capped at 999) solved once after a warm-up, for
rocprofv3 passes over k_solve_mid2 (SQ / GRBM counters: VALU instructions
issued, busy cycles).  Prints h statistics so the counter record can be tied
to the bench's timed solve.  Usage: python scripts/horizon_pmc.py H"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(H: int, knobs=(), B: int = 16384):
    import torch

    import pqp_amd

    for kv in knobs:  # key=value pqp_tune settings (A/B runs)
        k, v = kv.split("=")
        pqp_amd.tune(k, int(v))

    ex = ROOT / "tests" / "golden" / "example"
    E = pqp_amd.read_example(ex)
    xs = pqp_amd.perturbed_states(E["x"], B * H, seed=7).reshape(B, H, -1)
    pb = pqp_amd.horizon_batch(ex, H, xs)
    pb.solve(max_updates=999)  # warm (dispatch 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pb.solve(max_updates=999)  # the measured solve (dispatch 2)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    h = pb.h.cpu().numpy()
    print(json.dumps({"H": H, "knobs": list(knobs), "n_dual": pb.N, "m": pb.M, "problems": B, "converge_ms": dt * 1e3,
                      "kernel": pqp_amd.tune_get("last_batch_kernel"), "h_sum": int(h.sum()),
                      "h_mean": float(h.mean())}))


if __name__ == "__main__":
    main(int(sys.argv[1]), sys.argv[2:])
