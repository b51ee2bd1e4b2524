"""One large problem's fixed-mode update as one row block (pqp_rowblock_update),
and the per-rank blocks of a row-sharded one:
the lean relay (Qd, 4 B per entry) vs the split-matrix relay (8 B per entry),
n_dual 2048..16384, us per update and algorithmic GB/s of each layout; the
two iterates compared bit for bit."""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main():
    import numpy as np
    import torch

    import pqp_amd

    L = pqp_amd.lib()
    sizes = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "2048,4096,8192,16384").split(",")]
    # whole problems, then the per-rank blocks of a row-sharded n_dual = 16384
    # problem at 8 and 4 ranks (2048 and 4096 rows)
    cases = [(N, N) for N in sizes] + [(16384, 2048), (16384, 4096)]
    for N, rows in cases:
        out = {"n_dual": N, "rows": rows}
        ys = {}
        for name, min_n in (("lean", 1), ("split", 0)):
            prev = L.pqp_tune_lean_min_n(min_n)
            blk, _, _ = pqp_amd.RowBlock.synthetic(7, 0, N, 0, rows)
            L.pqp_tune_lean_min_n(prev)
            Y = torch.full((N,), 1000.0, device="cuda")
            Yn = torch.full((N,), 1000.0, device="cuda")
            for _ in range(3):
                blk.update(Y, Yn[:rows])
                Y, Yn = Yn, Y
            torch.cuda.synchronize()
            ups = 200 if N <= 8192 else 60
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(ups):
                blk.update(Y, Yn[:rows])
                Y, Yn = Yn, Y
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / ups * 1e3
            bpe = 4 if name == "lean" else 8
            out[name] = {"us_per_update": us, "alg_GBps": bpe * rows * N / us / 1e3}
            ys[name] = Y.cpu().numpy()
            del blk
            torch.cuda.empty_cache()
        out["bit_identical"] = bool(np.array_equal(ys["lean"].view(np.uint32), ys["split"].view(np.uint32)))
        out["speedup"] = out["split"]["us_per_update"] / out["lean"]["us_per_update"]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
