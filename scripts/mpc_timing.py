"""Converge-mode throughput of many small MPC problems (the bundled plant,
N = 28, M = 7, at B perturbed states): the one-wave solver (k_solve_wave)
against the four-wave solver (k_solve_tiny) for several batch sizes, with
the per-problem h checked equal.  Run on the GPU box:
python scripts/mpc_timing.py"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main():
    import numpy as np
    import torch

    import pqp_amd

    L = pqp_amd.lib()
    ex_dir = ROOT / "tests" / "golden" / "example"
    ex = pqp_amd.read_example(ex_dir)
    out = {}
    for B in (1, 256, 2048, 16384, 65536):
        rng = np.random.default_rng(5)
        xs = (ex["x"][None, :] * (1.0 + 0.05 * rng.standard_normal((B, ex["ns"])))).astype(np.float32)
        pb = pqp_amd.mpc_batch(ex_dir, xs)
        row = {}
        hs = {}
        for name, thr, pipe in (("wave_pipelined", 1, 1 << 30), ("wave_plain", 1, 0), ("tiny", 1 << 30, 0)):
            L.pqp_tune_wave_min_b(thr)
            L.pqp_tune_wave_pipe_max_b(pipe)
            pb.solve(max_updates=200000)
            torch.cuda.synchronize()
            reps = 3 if B >= 16384 else 10
            t0 = time.perf_counter()
            for _ in range(reps):
                pb.solve(max_updates=200000)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            h = pb.h.cpu().numpy()
            hs[name] = h.copy()
            row[name] = {"ms": dt * 1e3, "qp_solves_per_s": B / dt, "iterations_per_s": float(h.sum()) / dt}
        row["h_identical"] = all(bool(np.array_equal(hs[k], hs["tiny"])) for k in hs)
        row["speedup_best_wave_vs_tiny"] = row["tiny"]["ms"] / min(row["wave_pipelined"]["ms"], row["wave_plain"]["ms"])
        out[f"B{B}"] = row
        print(json.dumps({f"B{B}": row}), flush=True)
        del pb
        torch.cuda.empty_cache()
    L.pqp_tune_wave_min_b(1)
    L.pqp_tune_wave_pipe_max_b(4096)


if __name__ == "__main__":
    main()
