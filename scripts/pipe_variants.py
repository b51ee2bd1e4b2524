"""k_solve_pipe build variants (pqp_tune "pipe_variant") on the bench's
batch_converge workload: steady-state ms per iteration (3K-call minus K-call,
as bench.py's leg) on infeasible and all-feasible iterates, and each variant's
phase trace.  Usage: python scripts/pipe_variants.py [variants, e.g. 0,3]"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(variants):
    import numpy as np
    import torch

    import pqp_amd

    B, N, M, K, ntr = 4096, 1024, 512, 4, 256
    pb = pqp_amd.ProblemBatch.synthetic(1, 0, B, N, M)
    kp = pb.Kp.clone()
    buf = torch.zeros(ntr * 16, dtype=torch.int64, device="cuda")

    def call(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pb.solve(max_updates=k)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    if os.environ.get("PIPE_OFF"):  # k_solve_single (pipe_variant 5: its round-3 form)
        pqp_amd.tune("pipe_off", 1)
    for v in variants:
        pqp_amd.tune("pipe_variant", v)
        for case in ("infeasible", "feasible"):
            pb.Kp.copy_(kp)
            if case == "feasible":
                pb.Kp.fill_(1e30)
            call(1)
            a, b = call(K), call(3 * K)
            per = (b - a) / (2 * K)
            alg = 4.0 * N * N + 4.0 * N * M + 4.0 * M * M * (2 if case == "feasible" else 1)
            buf.zero_()
            pqp_amd._check(pqp_amd.lib().pqp_tune_trace(b"mid", C.c_void_p(buf.data_ptr()), ntr))
            try:
                pb.solve(max_updates=8)
                torch.cuda.synchronize()
            finally:
                pqp_amd.lib().pqp_tune_trace(b"mid", None, 0)
            T = buf.view(ntr, 16).cpu().numpy().astype(np.float64)
            it = T[:, 4]
            ok = it > 0
            ph = [float(np.median(T[ok, c] / it[ok])) for c in range(3)]
            print(json.dumps({"variant": v, "case": case, "ms_per_iter": per * 1e3, "TBps": alg * B / per / 1e12,
                              "kernel": pqp_amd.tune_get("last_batch_kernel"), "cyc_X": ph[0], "cyc_Y": ph[1],
                              "cyc_cost": ph[2]}), flush=True)
    pqp_amd.tune("pipe_variant", 0)


if __name__ == "__main__":
    main([int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,3").split(",")])
