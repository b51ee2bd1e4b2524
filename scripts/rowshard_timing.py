"""Row-block update timing on one GPU: one problem of
n_dual = N in `blocks` equal row blocks, updates timed with HIP events
(eager launches of pqp_rowblock_update), and algorithmic GB/s of the stored
split matrices (8 N^2 B per update)."""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,4096,8192,16384,32768")
    ap.add_argument("--blocks", type=int, default=1)
    ap.add_argument("--updates", type=int, default=50)
    ap.add_argument("--variants", default="0", help="pqp_tune_set_variant values to time (comma separated)")
    a = ap.parse_args()
    import torch

    import pqp_amd
    from pqp_amd.rowshard import row_plan

    L = pqp_amd.lib()
    for N, var in ((int(s), int(v, 0)) for s in a.sizes.split(",") for v in a.variants.split(",")):
        L.pqp_tune_set_variant(var)
        R, plan = row_plan(N, a.blocks)
        blocks = [pqp_amd.RowBlock.synthetic(1, 0, N, r0, rows)[0] for r0, rows in plan]
        Y = torch.full((N,), 1000.0, device="cuda")
        Yn = torch.empty(N, device="cuda")

        def step(Y, Yn):
            for b in blocks:
                if b.rows:
                    b.update(Y, Yn[b.row0:b.row0 + b.rows])

        for _ in range(3):
            step(Y, Yn)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.updates):
            step(Y, Yn)
            Y, Yn = Yn, Y
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.updates * 1e3
        print(json.dumps({"n_dual": N, "variant": hex(var), "blocks": a.blocks, "us_per_update": us,
                          "alg_split_GBps": 8.0 * N * N / (us * 1e-6) / 1e9,
                          "finite": bool(torch.isfinite(Y[:N]).all().item())}), flush=True)
        del blocks
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
