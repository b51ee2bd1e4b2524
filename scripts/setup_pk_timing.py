"""Setup GEMMs on the packed 128 x 128 k_matmul_pk against
the 64 x 64 k_matmul_tiled (pqp_tune("matmul_pk_off", 1)), same process and
box, alternating: pqp_batch_convert_to_dual of B problems (n_dual N, M
primal, dense Qp_inv); bits compared.  FLOPs of the two GEMMs per problem:
2NM^2 (Gp Qp_inv) + 2N^2M ((Gp Qp_inv) Gp').
Usage: python scripts/setup_pk_timing.py [N M B reps]"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "pqp-for-mpc_amd")]


def main(N=1024, M=512, B=64, reps=3):
    import torch

    import pqp_amd
    from pqp_amd import dense_qinv

    L = pqp_amd.lib()
    pb = pqp_amd.ProblemBatch(B, N, M)
    pqp_amd._check(L.pqp_batch_synth_primal(3, 0, B, N, M, *[pb._p(getattr(pb, k)) for k in pb.PRIMAL], pb._s()))
    pb.Qp_inv.copy_(torch.from_numpy(dense_qinv(3, M)).cuda().expand(B, -1))
    flops = B * (2.0 * N * M * M + 2.0 * N * N * M)
    out = {"n_dual": N, "m": M, "problems": B}
    res, times = {}, {"pk": [], "tiled": []}
    for r in range(reps):
        for name, knob, off in (("pk", "matmul_pk_off", 0), ("tiled", "matmul_pk_off", 1)):
            prev = pqp_amd.tune(knob, off)
            try:
                pb.convert_to_dual()  # warm
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pb.convert_to_dual()
                torch.cuda.synchronize()
                times[name].append(time.perf_counter() - t0)
            finally:
                pqp_amd.tune(knob, prev)
            res[name] = torch.cat([pb.Qd.reshape(-1), pb.Fd.reshape(-1), pb.Md.reshape(-1)]).clone()
    for name, ts in times.items():
        dt = sorted(ts)[len(ts) // 2]
        out[name] = {"ms": dt * 1e3, "gemm_TFLOPs": flops / dt / 1e12, "all_ms": [t * 1e3 for t in ts]}
    out["bit_identical"] = bool(torch.equal(res["pk"].view(torch.int32), res["tiled"].view(torch.int32)))
    out["speedup"] = out["tiled"]["ms"] / out["pk"]["ms"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:5]])
