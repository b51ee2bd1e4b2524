"""Setup GEMMs: pqp_batch_convert_to_dual on B problems of
n_dual N / M primal with a dense Qp_inv, LDS-tiled (k_matmul_tiled) vs the
one-thread-per-output k_matmul_seq, bit-identical results compared; GFLOP/s
of the two GEMMs (Gp Qp_inv: 2NM^2, (Gp Qp_inv) Gp': 2N^2M per problem).
Usage: python scripts/setup_timing.py [N M B]"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "pqp-for-mpc_amd"), str(ROOT / "tests" / "golden")]


def main(N=1024, M=512, B=64):
    import numpy as np
    import torch

    import pqp_amd
    from pqp_amd import dense_qinv

    L = pqp_amd.lib()
    pb = pqp_amd.ProblemBatch(B, N, M)
    pqp_amd._check(L.pqp_batch_synth_primal(3, 0, B, N, M, *[pb._p(getattr(pb, k)) for k in pb.PRIMAL], pb._s()))
    pb.Qp_inv.copy_(torch.from_numpy(dense_qinv(3, M)).cuda().expand(B, -1))
    out = {"n_dual": N, "m": M, "problems": B}
    res = {}
    for name, off in (("tiled", 0), ("seq", 1), ("tiled_again", 0)):
        prev = L.pqp_tune_matmul_tiled(off)
        pb.convert_to_dual()  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pb.convert_to_dual()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        L.pqp_tune_matmul_tiled(prev)
        res[name] = pb.Qd.clone()
        flops = B * (2.0 * N * M * M + 2.0 * N * N * M)
        out[name] = {"ms": dt * 1e3, "problems_per_s": B / dt, "gemm_TFLOPs": flops / dt / 1e12}
    out["bit_identical"] = bool(torch.equal(res["tiled"].view(torch.int32), res["seq"].view(torch.int32)))
    out["speedup"] = out["seq"]["ms"] / out["tiled"]["ms"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:4]])
