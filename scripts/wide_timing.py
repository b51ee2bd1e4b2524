"""Converge-mode time per iteration of ONE synthetic problem: the wide path
(multi-workgroup terminate() + relay update, pqp_wide.hip) vs the
one-workgroup solver (k_solve_single).  Capped solves (the synthetic problems
do not converge at these sizes), bit-identical results checked."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "pqp-for-mpc_amd", ROOT / "oracle"):
    sys.path.insert(0, str(p))


def main():
    import numpy as np

    import pqp_amd
    from oracle import Oracle

    sizes = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "192,256,384,512,1024,2048,4096").split(",")]
    orc = Oracle()
    L = pqp_amd.lib()
    for N in sizes:
        M = N // 2
        pb = pqp_amd.ProblemBatch(1, N, M)
        prim = orc.synth_primal(1, 0, N, M)
        for k in pqp_amd.ProblemBatch.PRIMAL:
            pb.set(k, np.asarray(prim[k], np.float32)[None])
        pb.gauss_jordan().convert_to_dual()
        P = {k: getattr(pb, k)[0].cpu().numpy() for k in ("Qd", "Fd", "Qp", "Qp_inv", "Fp", "Gp", "Kp")}
        P.update(Md=pb.Md[:1].cpu().numpy(), Mp=pb.Mp[:1].cpu().numpy(), N=N, M=M)
        out = {"n_dual": N, "m": M}
        ys = {}
        with pqp_amd.Problem(P) as prob:
            arms = [("wide", 0, 200), ("single_wg", 0x200, 20)]
            for name, var, cap in arms:
                L.pqp_tune_set_variant(var)
                prob.solve(max_updates=2)
                t0 = time.perf_counter()
                r = prob.solve(max_updates=cap)
                dt = time.perf_counter() - t0
                out[name] = {"updates": cap, "us_per_iter": dt / (cap + 1) * 1e6}
                ys[name] = (r, cap)
            L.pqp_tune_set_variant(0)
            r = prob.solve(max_updates=20)
        out["bit_identical_at_20"] = bool(np.array_equal(r["Y"].view(np.uint32), ys["single_wg"][0]["Y"].view(np.uint32)))
        out["speedup"] = out["single_wg"]["us_per_iter"] / out["wide"]["us_per_iter"]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
