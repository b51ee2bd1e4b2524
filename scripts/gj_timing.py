"""Batched Gauss_Jordan timing (PQP_CPU.c:251-326): B
matrices of n x n (the synthetic problems' setup: Qp = inverse(Qp_inv)),
k_gj_blocked3 (default: only the columns that can still change an output) and
the one-pivot-per-sweep kernel, bit-identical outputs (k_gj_blocked /
k_gj_blocked2 were removed in round 6; their numbers are in profiles/r05).
Usage: python scripts/gj_timing.py [n B]"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(n=512, B=4096):
    import ctypes as C

    import torch

    import pqp_amd

    L = pqp_amd.lib()
    g = torch.Generator(device="cuda").manual_seed(n)
    A = torch.randn(B, n * n, device="cuda", generator=g)
    A.view(B, n, n).diagonal(dim1=1, dim2=2).add_(float(n))
    R = torch.empty_like(A)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {"n": n, "matrices": B}
    res = {}
    for name, off in (("blocked3", 0), ("per_sweep", 1), ("blocked3_again", 0)):
        prev = L.pqp_tune_gj_blocked(off)
        ts = []
        for _ in range(2 if name == "per_sweep" else 3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pqp_amd._check(L.pqp_batch_gauss_jordan(B, n, C.c_void_p(A.data_ptr()), C.c_void_p(R.data_ptr()), s))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        L.pqp_tune_gj_blocked(prev)
        res[name] = R.clone()
        t = min(ts)
        # the reference's operations: n pivots x (n-1) rows x 2n columns of one
        # multiply and one subtract, plus the row scaling
        ops = 2.0 * n * (n - 1) * 2 * n + 2.0 * n * n
        out[name] = {"s": t, "matrices_per_s": B / t, "Gops": ops * B / t / 1e9}
    out["bit_identical"] = all(torch.equal(res[k].view(torch.int32), res["per_sweep"].view(torch.int32))
                               for k in ("blocked3", "blocked3_again"))
    out["speedup_vs_per_sweep"] = out["per_sweep"]["s"] / out["blocked3"]["s"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:3]])
