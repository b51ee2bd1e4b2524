"""Problem sharding on the GPU: ranks run their own block of
problems through the batched kernel, rank 0 gathers Y* in problem order, and
the result is bit-identical to the oracle over all problems.

Ranks share the one GPU of the test box, so the collectives go over gloo
(RCCL refuses two ranks on one device); the data path is the same as
bench.py's (`scatter_plan`, `Batch.generate(seed, inst0)`, `gather_rows`).
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from conftest import ROOT, assert_bitwise

pytestmark = pytest.mark.gpu

N, PER_RANK, UPDATES, SEED = 260, 3, 7, 11


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out):
    import sys

    for p in (ROOT / "pqp-for-mpc_amd", ROOT / "oracle"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    import pqp_amd
    from pqp_amd.shard import gather_rows, scatter_plan

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    seed, inst0, count = scatter_plan(dist, rank, world, PER_RANK, SEED, dev)
    assert (seed, inst0, count) == (SEED, rank * PER_RANK, PER_RANK)
    b = pqp_amd.Batch(count, N, device=dev).generate(seed, inst0=inst0, M=N // 2)
    b.iterate(UPDATES)
    torch.cuda.synchronize(dev)
    full = gather_rows(dist, rank, world, b.Y[:, :N].contiguous())
    if rank == 0:
        np.save(out, full.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_batches_gathered_in_problem_order(gpu_lib, orc, tmp_path, world):
    import torch.multiprocessing as mp

    out = str(tmp_path / "y.npy")
    mp.spawn(_rank_main, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    assert got.shape == (world * PER_RANK, N)
    for b in range(world * PER_RANK):
        P = orc.synth_problem(SEED, b, N, N // 2, with_qp=False)
        assert_bitwise(got[b], orc.iterate(P["Qd"], P["Fd"], N, UPDATES), f"problem {b}")
