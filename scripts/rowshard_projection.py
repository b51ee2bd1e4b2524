"""Per-rank compute time of the row-sharded update at
world sizes 1..8, measured on ONE GPU: rank 0's row block of an N-row problem
is what each rank runs per update when the job has `world` ranks (the blocks
are equal but for the last).  The RCCL all-gather between updates is not in
these numbers (one GPU cannot measure xGMI); DESIGN.md section 6 adds it.

Usage: python scripts/rowshard_projection.py [N ...]   (default 16384 32768)
Prints one JSON object.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pqp-for-mpc_amd"))

import torch  # noqa: E402

import pqp_amd  # noqa: E402
from pqp_amd.rowshard import row_plan  # noqa: E402


def time_block(N: int, world: int, updates: int = 200) -> dict:
    dev = torch.device("cuda", 0)
    R, plan = row_plan(N, world)
    row0, rows = plan[0]
    blk, _, _ = pqp_amd.RowBlock.synthetic(7, 0, N, row0, rows, device=dev)
    Y = torch.full((N,), 1000.0, dtype=torch.float32, device=dev)
    Yr = torch.empty(max(1, R), dtype=torch.float32, device=dev)
    for _ in range(5):
        blk.update(Y, Yr)
    torch.cuda.synchronize(dev)
    # device time per update: back-to-back launches on one stream, HIP events
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(updates):
        blk.update(Y, Yr)
    e1.record()
    torch.cuda.synchronize(dev)
    dev_us = e0.elapsed_time(e1) * 1e3 / updates
    # latency of one update as a rank sees it between two all-gathers: launch + run + sync
    lat = []
    for _ in range(50):
        t0 = time.perf_counter()
        blk.update(Y, Yr)
        torch.cuda.synchronize(dev)
        lat.append(time.perf_counter() - t0)
    lat.sort()
    blk.check()
    del blk
    torch.cuda.empty_cache()
    return {"world": world, "rows": rows, "device_us_per_update": dev_us,
            "launch_sync_us_median": lat[len(lat) // 2] * 1e6,
            "matrix_GBps": 4.0 * rows * N / (dev_us * 1e-6) / 1e9}


def main():
    Ns = [int(a) for a in sys.argv[1:]] or [16384, 32768]
    out = {"note": "rank 0's row block on one GPU; the all-gather of 4N bytes per update is not included", "runs": []}
    for N in Ns:
        for world in (1, 2, 4, 8):
            r = time_block(N, world)
            r["n_dual"] = N
            out["runs"].append(r)
            print(json.dumps(r), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
