"""A/B of pqp_batch_iterate's kernels on the headline workload (configs[3]:
4096 synthetic problems of n_dual 1024, 10 updates per launch), alternating
in one process: k_batch_resident (the default at n_dual 1024, round 6; kind 3
its LDS + L2 form without the register blocks),
k_batch_stream (round 5, pqp_tune iterate_kind 2) and k_batch_iterate
(rounds 1-4, iterate_kind 1).  Reports the
launch time (HIP events) and TB/s of algorithmic bytes; checks that every
variant gives the same bits."""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(B: int = 4096, N: int = 1024, chunk: int = 10, rounds: int = 4, reps: int = 5):
    import torch

    import pqp_amd

    b = pqp_amd.Batch(B, N).generate(1, 0)
    alg = (4 * N * N + 16 * N) * B * chunk
    res = {}
    ref = None
    for _ in range(rounds):
        for v in (0, 3, 2, 1):
            old = pqp_amd.tune("iterate_kind", v)
            try:
                b.iterate(chunk)
                torch.cuda.synchronize()
                if ref is None:
                    ref = b.Y.clone()
                same = bool(torch.equal(b.Y, ref))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    b.iterate(chunk)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
            finally:
                pqp_amd.tune("iterate_kind", old)
            r = res.setdefault(v, {"ms": [], "same_bits": True})
            r["ms"].append(round(ms, 3))
            r["same_bits"] &= same
    names = {0: "k_batch_resident", 1: "k_batch_iterate", 2: "k_batch_stream", 3: "k_batch_resident_lds_only"}
    out = {names[v]: {"ms_per_launch": r["ms"], "TBps_best": alg / min(r["ms"]) / 1e9,
                                   "frac_of_8TBps_best": alg / min(r["ms"]) / 1e9 / 8.0, "same_bits": r["same_bits"]}
           for v, r in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
