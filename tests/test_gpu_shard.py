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


def _rccl_one_rank_main(rank, world, port, out):
    import sys

    for p in (ROOT / "pqp-for-mpc_amd", ROOT / "oracle"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    import pqp_amd
    from pqp_amd.shard import gather_rows, scatter_plan

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)  # bench.py's init
    seed, inst0, B = scatter_plan(dist, rank, world, 3, 11, dev, collective_at_one=True)
    b = pqp_amd.Batch(B, 300, device=dev).generate(seed, inst0=inst0, M=150)
    b.iterate(4)
    torch.cuda.synchronize(dev)
    y = b.Y[:, :300].contiguous()
    full = gather_rows(dist, rank, world, y, collective_at_one=True)
    t = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the bench's max-over-ranks timing
    dist.barrier()
    np.save(out + ".npy", full.cpu().numpy())
    np.save(out + ".plan.npy", np.array([seed, inst0, B, int(t[1].item() == 2.5)]))
    dist.destroy_process_group()


def test_rccl_scatter_gather_one_rank(gpu_lib, orc, tmp_path):
    """bench.py's RCCL calls -- nccl init with device_id, the shard-plan
    scatter, the Y* gather, the max all-reduce, the barrier -- over a one-rank
    group (RCCL refuses two ranks on one GPU), with the gathered iterates
    checked against the oracle."""
    import torch.multiprocessing as mp

    out = str(tmp_path / "r")
    mp.spawn(_rccl_one_rank_main, args=(1, _free_port(), out), nprocs=1, join=True)
    seed, inst0, B, ok = (int(v) for v in np.load(out + ".plan.npy"))
    assert (seed, inst0, B, ok) == (11, 0, 3, 1)
    full = np.load(out + ".npy")
    for j in range(B):
        P = orc.synth_problem(11, j, 300, 150, with_qp=False)
        assert_bitwise(full[j], orc.iterate(P["Qd"], P["Fd"], 300, 4), f"problem {j}")


CFG4_N, CFG4_PER_RANK, CFG4_WORLD, CFG4_SEED, CFG4_UPDATES = 1024, 4096, 8, 1, 10


def _configs4_rank_main(rank, world, port, out):
    """One rank of configs[4]'s layout: the bench's shard plan (8 ranks x
    4096 problems of n_dual 1024, seed 1) scattered from rank 0; the rank runs
    the first two and the last problem of ITS shard (inst0 = r * 4096) through
    the fused kernel for one bench launch (10 updates); rank 0 gathers."""
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
    seed, inst0, count = scatter_plan(dist, rank, world, CFG4_PER_RANK, CFG4_SEED, dev)
    assert (seed, inst0, count) == (CFG4_SEED, rank * CFG4_PER_RANK, CFG4_PER_RANK)
    N = CFG4_N
    ys = []
    for first, n in ((inst0, 2), (inst0 + count - 1, 1)):
        b = pqp_amd.Batch(n, N, device=dev).generate(seed, inst0=first, M=N // 2)
        b.iterate(CFG4_UPDATES)
        ys.append(b.Y[:, :N].clone())
    torch.cuda.synchronize(dev)
    full = gather_rows(dist, rank, world, torch.cat(ys, 0).contiguous())
    if rank == 0:
        np.save(out, full.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_configs4_shards_pinned_to_oracle(gpu_lib, orc, tmp_path):
    """configs[4]'s own problem ids on 8 ranks (gloo, all on this
    box's one GPU): the shard plan gives rank r problems [r * 4096, (r+1) *
    4096); each rank's first two and last problem are iterated on the GPU and
    gathered on rank 0 in rank order.  Every shard's first problem (and the
    job's last, 32767) bit-exact against the oracle's updates
    (PQP_CPU.c:603-618, the testing/ loop of PQP_GPU_optimized.cu:799); all 24
    equal a one-process batch of the same ids."""
    import torch
    import torch.multiprocessing as mp

    out = str(tmp_path / "y.npy")
    mp.spawn(_configs4_rank_main, args=(CFG4_WORLD, _free_port(), out), nprocs=CFG4_WORLD, join=True)
    got = np.load(out)
    N = CFG4_N
    assert got.shape == (CFG4_WORLD * 3, N)
    ids = [i for r in range(CFG4_WORLD) for i in (r * CFG4_PER_RANK, r * CFG4_PER_RANK + 1,
                                                   (r + 1) * CFG4_PER_RANK - 1)]
    for row, inst in enumerate(ids):
        b = gpu_lib.Batch(1, N, device="cuda:0").generate(CFG4_SEED, inst0=inst, M=N // 2)
        b.iterate(CFG4_UPDATES)
        assert_bitwise(got[row], b.result()[0], f"gathered problem {inst}")
    torch.cuda.empty_cache()
    for row, inst in enumerate(ids):
        if inst % CFG4_PER_RANK == 0 or inst == CFG4_WORLD * CFG4_PER_RANK - 1:
            P = orc.synth_problem(CFG4_SEED, inst, N, N // 2, with_qp=False)
            assert_bitwise(got[row], orc.iterate(P["Qd"], P["Fd"], N, CFG4_UPDATES), f"problem {inst} vs oracle")
