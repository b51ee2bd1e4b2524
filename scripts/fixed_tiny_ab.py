"""Fixed mode of the bundled problem (N = 28): k_fixed_tiny with the iterate in
registers (y_k on lane 2k, v_readlane broadcasts) vs through LDS, for one
problem (configs[1]: pqp_problem_solve, 1000 iterations) and for batches of
bundled-plant problems (pqp_batch_solve).  Bit-identical results checked."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(reps: int = 50):
    import numpy as np
    import torch

    import pqp_amd

    L = pqp_amd.lib()
    P = pqp_amd.example_problem(ROOT / "tests" / "golden" / "example")
    out = {"single": {}, "batch": {}}
    ys = {}
    with pqp_amd.Problem(P) as prob:
        for name, mb in (("registers", 1 << 30), ("lds", 0)):
            L.pqp_tune_fixed_rl_max_b(mb)
            prob.solve(pqp_amd.MODE_FIXED, num_iter=1000)
            t0 = time.perf_counter()
            for _ in range(reps):
                r = prob.solve(pqp_amd.MODE_FIXED, num_iter=1000)
            dt = (time.perf_counter() - t0) / reps
            out["single"][name] = {"ms_per_solve": dt * 1e3, "iter_per_s": 999 / dt}
            ys[name] = r["Y"]
    out["single"]["bit_identical"] = bool(np.array_equal(ys["registers"].view(np.uint32), ys["lds"].view(np.uint32)))
    ex = pqp_amd.read_example(ROOT / "tests" / "golden" / "example")
    rng = np.random.default_rng(5)
    for B in (1024, 16384):
        res = {}
        xs = (ex["x"][None, :] * (1.0 + 0.05 * rng.standard_normal((B, ex["ns"])))).astype(np.float32)
        pb = pqp_amd.mpc_batch(ROOT / "tests" / "golden" / "example", xs)
        for name, mb in (("registers", 1 << 30), ("lds", 0)):
            L.pqp_tune_fixed_rl_max_b(mb)
            pb.solve(pqp_amd.MODE_FIXED, num_iter=1000)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pb.solve(pqp_amd.MODE_FIXED, num_iter=1000)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res[name] = {"ms": dt * 1e3, "instance_iter_per_s": B * 999 / dt}
            ys[name] = pb.Y.cpu().numpy().copy()
        if len(res) == 2:
            res["bit_identical"] = bool(np.array_equal(ys["registers"].view(np.uint32), ys["lds"].view(np.uint32)))
            out["batch"][str(B)] = res
    L.pqp_tune_fixed_rl_max_b(1024)  # the library default
    print(json.dumps(out))


if __name__ == "__main__":
    main()
