"""Interleaved A/B of the batched update kernel variants in ONE process
(cdna_hip_programming.md §5.4 rule 24), plus the practical HBM read ceiling of
the same access pattern (k_stream_read).  Run on the GPU box:

    python scripts/ab_batch.py [--n 1024] [--batch 4096] [--rounds 5] [--launches 10]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))

VARIANTS = {0: "U16+nt (default)", 1: "U8", 2: "U8+nt", 3: "U4+nt", 4: "U32+nt", 5: "U16", 6: "U16+nt max-terms (timing only)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch

    import pqp_amd

    L = pqp_amd.lib()
    N, B = a.n, a.batch
    alg = (4 * N * N + 16 * N) * B
    b = pqp_amd.Batch(B, N).generate(1)
    out = torch.empty(B * 256, device="cuda")
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)

    # correctness: every variant gives the same bits
    ref = None
    for v in VARIANTS:
        L.pqp_tune_set_variant(v)
        y = b.iterate(3).result()
        if ref is None:
            ref = y
        assert np.array_equal(y.view(np.uint32), ref.view(np.uint32)), f"variant {v} differs"
    L.pqp_tune_set_variant(0)

    def t_iter(v, chunk=1):
        L.pqp_tune_set_variant(v)
        b.iterate(chunk)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.launches):
            b.iterate(chunk, from_start=False)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / a.launches / chunk

    def t_read(nt):
        L.pqp_tune_stream_read(B, N, C.c_void_p(b.QdT.data_ptr()), b.ldq, b.qstride, C.c_void_p(out.data_ptr()), nt, sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.launches):
            L.pqp_tune_stream_read(B, N, C.c_void_p(b.QdT.data_ptr()), b.ldq, b.qstride, C.c_void_p(out.data_ptr()),
                                   nt, sp)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / a.launches

    arms = [(f"iterate {VARIANTS[v]}", (lambda v=v: t_iter(v))) for v in VARIANTS]
    arms += [("iterate default chunk10", lambda: t_iter(0, 10)), ("stream_read", lambda: t_read(0)),
             ("stream_read nt", lambda: t_read(1))]
    res = {name: [] for name, _ in arms}
    for _ in range(a.rounds):
        for name, fn in arms:
            res[name].append(fn())
    L.pqp_tune_set_variant(0)
    rows = []
    for name, ts in res.items():
        med, mn = statistics.median(ts), min(ts)
        rows.append({"arm": name, "median_ms": med, "min_ms": mn, "GBps_median": alg / med / 1e6,
                     "frac_of_8TBs": alg / med / 1e6 / 8000})
        print(f"{name:22s} median {med:8.4f} ms  min {mn:8.4f} ms  {alg / med / 1e6:8.1f} GB/s "
              f"({alg / med / 1e6 / 80:5.1f}% of 8 TB/s)", flush=True)
    print(json.dumps({"n": N, "batch": B, "rounds": a.rounds, "launches": a.launches, "arms": rows}))


if __name__ == "__main__":
    main()
