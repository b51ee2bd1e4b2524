"""BASELINE configs[2]: ONE synthetic dense problem, n_dual = 1024 (M = 512),
1000 fixed-mode iterations on one MI355X.  Compares the multi-workgroup
split-matrix path (k_split_update, default) with the one-workgroup solver
(k_solve_single), checks they agree bit for bit, and reports iter/s and the
algorithmic GB/s of the update kernel (8 N^2 B of stored split matrices per
iteration; cache-resident at this size)."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(N: int = 1024, iters: int = 1000, reps: int = 5):
    import numpy as np

    import pqp_amd

    M = N // 2
    b = pqp_amd.Batch(1, N).generate(seed=1, inst0=0, M=M)
    P = dict(Qd=b.qd_rowmajor(0), Fd=b.Fd[0, :N].cpu().numpy(), Md=b.Md[:1].cpu().numpy(),
             Qp=np.zeros(M * M, np.float32), Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32),
             Mp=np.zeros(1, np.float32), Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32), N=N, M=M)
    L = pqp_amd.lib()
    out = {"n_dual": N, "iterations": iters}
    with pqp_amd.Problem(P) as prob:
        ys = {}
        variants = [("split_multi_wg", 0)]
        for lwsel, lw in ((1, 8), (2, 16), (4, 64)):
            variants.append((f"relay_w8s16_lw{lw}", lwsel << 17))
        variants.append(("single_wg", 0x200))
        variants.insert(0, ("persistent", 0))
        for name, var in variants:
            L.pqp_tune_set_variant(var)
            L.pqp_tune_persist(0 if name == "persistent" else 1)
            prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
            t0 = time.perf_counter()
            for _ in range(reps):
                r = prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
            dt = (time.perf_counter() - t0) / reps
            ys[name] = r["Y"]
            out[name] = {"ms_per_solve": dt * 1e3, "us_per_iter": dt / (iters - 1) * 1e6,
                         "iter_per_s": (iters - 1) / dt}
        L.pqp_tune_set_variant(0)
        L.pqp_tune_persist(0)
    out["bit_identical"] = all(bool(np.array_equal(y.view(np.uint32), ys["single_wg"].view(np.uint32)))
                               for y in ys.values())
    out["split_alg_GBps"] = 8 * N * N / (out["split_multi_wg"]["us_per_iter"] * 1e-6) / 1e9
    out["persistent_alg_GBps"] = 8 * N * N / (out["persistent"]["us_per_iter"] * 1e-6) / 1e9
    bb = pqp_amd.Batch(1, N).generate(seed=1, inst0=0, M=M)
    bb.iterate(3)
    import torch

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bb.iterate(iters - 1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out["batch_kernel_B1"] = {"us_per_iter": dt / (iters - 1) * 1e6, "iter_per_s": (iters - 1) / dt}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
