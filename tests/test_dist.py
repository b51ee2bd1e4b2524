"""Multi-process sharding logic on CPU (gloo, world size 2): every rank
computes its shard of problems (with the oracle standing in for the GPU
kernel, which these CPU tests must not call), rank 0 gathers, and the result
equals the single-process computation over all problems, in problem order."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N, PER_RANK, UPDATES, SEED = 16, 3, 5, 4


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import sys

    from conftest import ROOT

    for p in (ROOT / "pqp-for-mpc_amd", ROOT / "oracle"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    from oracle import Oracle
    from pqp_amd.shard import gather_rows, scatter_plan

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seed, inst0, count = scatter_plan(dist, rank, world, PER_RANK, SEED, torch.device("cpu"))
    assert (seed, inst0, count) == (SEED, rank * PER_RANK, PER_RANK)
    orc = Oracle()
    rows = []
    for j in range(count):
        P = orc.synth_problem(seed, inst0 + j, N, N // 2, with_qp=False)
        rows.append(orc.iterate(P["Qd"], P["Fd"], N, UPDATES))
    full = gather_rows(dist, rank, world, torch.from_numpy(np.stack(rows)))
    if rank == 0:
        np.save(out_path, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_scatter_gather(tmp_path, orc):
    out = tmp_path / "y.npy"
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    got = np.load(out)
    want = []
    for b in range(2 * PER_RANK):
        P = orc.synth_problem(SEED, b, N, N // 2, with_qp=False)
        want.append(orc.iterate(P["Qd"], P["Fd"], N, UPDATES))
    assert np.array_equal(got.view(np.uint32), np.stack(want).view(np.uint32))


def test_shard_plan_partitions_problems():
    import sys

    from conftest import ROOT

    sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
    from pqp_amd.shard import shard_plan

    plan = shard_plan(8, 4096, 1)
    starts = [p[1] for p in plan]
    assert starts == [r * 4096 for r in range(8)] and all(p[2] == 4096 for p in plan)
