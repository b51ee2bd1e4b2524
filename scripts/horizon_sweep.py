"""Batched converge mode across MPC horizon lengths (the reference report's
stated goal is varying the horizon): the bundled plant as H diagonal blocks
(scripts/problems.py block_diag_problem: n_dual 28H, M 7H; every iterate feasible, and the
reference stops at h = 313 for every H), B copies solved at once
(ProblemBatch, one workgroup per problem) and one copy alone (Problem, the
single-problem path).  Prints one JSON line per H.
Usage: python scripts/horizon_sweep.py [H ...]"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
sys.path.insert(0, str(ROOT / "scripts"))


def main(Hs):
    import numpy as np
    import torch

    import pqp_amd
    from problems import block_diag_problem, bundled_problem

    base = bundled_problem()
    for H in Hs:
        P = block_diag_problem(base, H)
        N, M = P["N"], P["M"]
        B = max(64, min(16384, (1 << 31) // (4 * N * N)))  # <= 2 GiB of Qd
        B = B // 64 * 64
        pb = pqp_amd.ProblemBatch.replicate(P, B)
        path = pqp_amd.lib().pqp_batch_solve_path(N, M)
        pb.solve(max_updates=200000)  # warm (and prepare)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pb.solve(max_updates=200000)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        h = pb.h.cpu().numpy()
        ok = bool((h == 313).all())
        # bytes per problem-iteration the batched solver reads on feasible
        # iterates: Qd (update, Y'Qd fused), Gp twice, Qp_inv, Qp
        alg = 4.0 * N * N + 8.0 * N * M + 8.0 * M * M
        it = float(h.sum())
        ab = {}
        if path == 3:  # the same batch with k_solve_mid turned off: time and bits
            Y3 = pb.Y.clone()
            old = pqp_amd.tune("mid_off", 1)
            try:
                pb.solve(max_updates=200000)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pb.solve(max_updates=200000)
                torch.cuda.synchronize()
                ab = {"mid_off_path": pqp_amd.lib().pqp_batch_solve_path(N, M),
                      "mid_off_batch_ms": (time.perf_counter() - t0) * 1e3,
                      "mid_off_same_bits": bool(torch.equal(pb.Y.view(torch.int32), Y3.view(torch.int32)))}
            finally:
                pqp_amd.tune("mid_off", old)
        if path == 2:  # the same batch on k_solve_single (Gp read twice): time and bits
            Y2 = pb.Y.clone()
            kern = pqp_amd.tune_get("last_batch_kernel")
            old = pqp_amd.tune("pipe_off", 1)
            try:
                pb.solve(max_updates=200000)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pb.solve(max_updates=200000)
                torch.cuda.synchronize()
                ab = {"batch_kernel": "k_solve_pipe" if kern else "k_solve_single",
                      "pipe_off_batch_ms": (time.perf_counter() - t0) * 1e3,
                      "pipe_off_same_bits": bool(torch.equal(pb.Y.view(torch.int32), Y2.view(torch.int32)))}
            finally:
                pqp_amd.tune("pipe_off", old)
        with pqp_amd.Problem(P) as prob:
            prob.solve(max_updates=200000)
            ts = []
            for _ in range(3):
                t1 = time.perf_counter()
                r = prob.solve(max_updates=200000)
                ts.append(time.perf_counter() - t1)
            single = sorted(ts)[1]
        print(json.dumps({"H": H, "n_dual": N, "m": M, "batch": B, "batch_path": path, "all_h_313": ok,
                          "batch_ms": dt * 1e3, "qp_solves_per_s": B / dt, "instance_iter_per_s": it / dt,
                          "alg_GBps": alg * it / dt / 1e9, "single_h": r["h"], "single_ms": single * 1e3,
                          "single_us_per_iter": single / r["h"] * 1e6, **ab}), flush=True)
        del pb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [1, 2, 4, 8, 16, 32])
