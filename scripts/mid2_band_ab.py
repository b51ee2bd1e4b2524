"""k_solve_mid2 band A/B on the bench's horizon workload (16384 problems,
seed 7, converge mode capped at 999): mid2_dense 1 (every k) against the
default band, alternating in one process, Y / U / h compared bit for bit,
plus fixed mode (314 iterations).  One JSON line per H.
Usage: python scripts/mid2_band_ab.py [H ...]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(Hs, B: int = 16384):
    import torch

    import pqp_amd

    ex = ROOT / "tests" / "golden" / "example"
    E = pqp_amd.read_example(ex)
    for H in Hs:
        xs = pqp_amd.perturbed_states(E["x"], B * H, seed=7).reshape(B, H, -1)
        pb = pqp_amd.horizon_batch(ex, H, xs)
        out = {"H": H, "n_dual": pb.N}
        for mode in ("converge", "fixed"):
            ts, res = {"dense": [], "band": []}, {}
            for rep in range(3):
                for name, dense in (("dense", 1), ("band", 0)):
                    old = pqp_amd.tune("mid2_dense", dense)
                    try:
                        run = (lambda: pb.solve(max_updates=999)) if mode == "converge" else \
                            (lambda: pb.solve(pqp_amd.MODE_FIXED, num_iter=314))
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        run()
                        torch.cuda.synchronize()
                        if rep:
                            ts[name].append((time.perf_counter() - t0) * 1e3)
                    finally:
                        pqp_amd.tune("mid2_dense", old)
                    res[name] = (pb.Y.clone(), pb.U.clone(), pb.h.clone())
            a, b = res["dense"], res["band"]
            same = bool(torch.equal(a[0].view(torch.int32), b[0].view(torch.int32)) and
                        torch.equal(a[1].view(torch.int32), b[1].view(torch.int32)) and torch.equal(a[2], b[2]))
            out[mode] = {k: round(min(v), 3) for k, v in ts.items()}
            out[mode]["same_bits"] = same
            out[mode]["h_sum"] = int(b[2].sum())
            out[mode]["kernel"] = pqp_amd.tune_get("last_batch_kernel")
        print(json.dumps(out), flush=True)
        del pb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main([int(v) for v in sys.argv[1:]] or [2, 3, 4, 5])
