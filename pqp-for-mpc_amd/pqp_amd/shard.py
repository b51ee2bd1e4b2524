"""Problem sharding across ranks (one process per GPU).

Independent MPC problems are the natural unit of parallelism: rank r owns the
contiguous block of problems [r*B, (r+1)*B).  The only collectives are at the
ends -- rank 0 scatters each rank's (seed, first problem, count) and gathers
every rank's Y* -- so the iteration data path has no communication (weak
scaling).  Backend-agnostic: "nccl" (RCCL over xGMI) on the GPUs, "gloo" in
the CPU tests.
"""
from __future__ import annotations


def shard_plan(world: int, per_rank: int, seed: int) -> list[tuple[int, int, int]]:
    """(seed, first problem, count) for every rank."""
    return [(int(seed), r * int(per_rank), int(per_rank)) for r in range(int(world))]


def scatter_plan(dist, rank: int, world: int, per_rank: int, seed: int, device,
                 collective_at_one: bool = False) -> tuple[int, int, int]:
    """Rank 0 hands every rank its shard description (one small scatter).
    `collective_at_one`: run the collective even for one rank (tests of the
    RCCL path on a one-GPU box)."""
    import torch

    mine = torch.zeros(3, dtype=torch.int64, device=device)
    if dist is None or (world == 1 and not collective_at_one):
        return shard_plan(1, per_rank, seed)[0]
    parts = None
    if rank == 0:
        parts = [torch.tensor(p, dtype=torch.int64, device=device) for p in shard_plan(world, per_rank, seed)]
    dist.scatter(mine, parts, src=0)
    s, i0, n = (int(v) for v in mine.tolist())
    return s, i0, n


def gather_rows(dist, rank: int, world: int, y, collective_at_one: bool = False):
    """Concatenate every rank's [count, N] block on rank 0 (rank order =
    problem order).  Returns the full tensor on rank 0, None elsewhere."""
    import torch

    if dist is None or (world == 1 and not collective_at_one):
        return y
    y = y.contiguous()
    outs = [torch.empty_like(y) for _ in range(world)] if rank == 0 else None
    dist.gather(y, outs, dst=0)
    return torch.cat(outs, 0) if rank == 0 else None
