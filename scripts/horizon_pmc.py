"""The bench's horizon workload (16384 MPC problems stacked H horizon stages,
seed 7, converge mode capped at 999) solved once after a warm-up, for
rocprofv3 passes over k_solve_mid2 (SQ / GRBM counters: VALU instructions
issued, busy cycles).  Prints h statistics so the counter record can be tied
to the bench's timed solve.  Usage: python scripts/horizon_pmc.py H [knob=v ...]
`H` = 2..5 (the stacked plant), or dN = the dense companion of bench.py's
horizon_dense leg at n_dual N (d112, d140)."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(H: str, knobs=(), B: int = 16384):
    import torch

    import pqp_amd

    for kv in knobs:  # key=value pqp_tune settings (A/B runs)
        k, v = kv.split("=")
        pqp_amd.tune(k, int(v))

    if H.startswith("d"):  # bench.py's horizon_dense workload
        sys.path.insert(0, str(ROOT))
        from bench import DENSE_SIZES, DENSE_UPDATES, dense_horizon_batch

        N = int(H[1:])
        pb = dense_horizon_batch(pqp_amd, N, dict(DENSE_SIZES)[N], B)
        cap = DENSE_UPDATES
    else:
        H = int(H)
        ex = ROOT / "tests" / "golden" / "example"
        E = pqp_amd.read_example(ex)
        xs = pqp_amd.perturbed_states(E["x"], B * H, seed=7).reshape(B, H, -1)
        pb = pqp_amd.horizon_batch(ex, H, xs)
        cap = 999
    pb.solve(max_updates=cap)  # warm (dispatch 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pb.solve(max_updates=cap)  # the measured solve (dispatch 2)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    h = pb.h.cpu().numpy()
    print(json.dumps({"H": H, "knobs": list(knobs), "n_dual": pb.N, "m": pb.M, "problems": B, "converge_ms": dt * 1e3,
                      "kernel": pqp_amd.tune_get("last_batch_kernel"), "h_sum": int(h.sum()),
                      "h_mean": float(h.mean())}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
