"""Row-sharded single problem, host logic on CPU.

The driver (pqp_amd.rowshard) runs world-size 2 and 3 with gloo.  A test-only
block that computes its rows with the oracle stands in for the GPU kernel,
which these CPU tests must not call.  The assembled iterate must equal the
single-process oracle iterate bit for bit, including ragged partitions
(N not a multiple of the world size) and ranks left with no rows."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
from pqp_amd.rowshard import row_plan  # noqa: E402

SEED, UPDATES = 6, 6


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _OracleBlock:
    """Test-only stand-in for pqp_amd.RowBlock: rows of the oracle's updateY2."""

    def __init__(self, orc, Qd, theta, Fd, N, row0, rows):
        self.orc, self.Qd, self.theta, self.Fd, self.N = orc, Qd, theta, Fd, N
        self.row0, self.rows = row0, rows

    def update(self, Y, Y_rows):
        import torch

        full = self.orc.update(Y[: self.N].numpy().copy(), self.Qd, self.theta, self.Fd, self.N)
        Y_rows[: self.rows] = torch.from_numpy(full[self.row0:self.row0 + self.rows].copy())


def _worker(rank, world, port, N, out_path):
    for p in (ROOT / "pqp-for-mpc_amd", ROOT / "oracle"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    from oracle import Oracle
    from pqp_amd.rowshard import RowShardedSolver, row_plan

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = Oracle()
    P = orc.synth_problem(SEED, 0, N, max(1, N // 2), with_qp=False)
    theta = orc.theta(P["Qd"], N)
    _, plan = row_plan(N, world)
    row0, rows = plan[rank]
    blk = _OracleBlock(orc, P["Qd"], theta, P["Fd"], N, row0, rows)
    solver = RowShardedSolver(blk, N, torch.device("cpu"), dist=dist)
    # a gloo group cannot be captured: every rank declines and stays eager
    assert solver.capture(2) is False and solver.graph is None
    y = solver.run(UPDATES + 1)
    np.save(f"{out_path}.{rank}.npy", y.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 16), (3, 10), (4, 5)])
def test_rowsharded_iterate_equals_single_process(tmp_path, orc, world, N):
    out = str(tmp_path / "y")
    mp.spawn(_worker, args=(world, _free_port(), N, out), nprocs=world, join=True)
    P = orc.synth_problem(SEED, 0, N, max(1, N // 2), with_qp=False)
    want = orc.iterate(P["Qd"], P["Fd"], N, UPDATES)
    for r in range(world):  # every rank holds the whole iterate
        got = np.load(f"{out}.{r}.npy")
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"rank {r}"


@pytest.mark.parametrize("N", [1, 5, 28, 1000, 1024, 38400])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_row_plan_partitions_rows(N, world):
    R, plan = row_plan(N, world)
    assert len(plan) == world and R == -(-N // world)
    covered = []
    for r, (row0, rows) in enumerate(plan):
        assert 0 <= rows <= R and row0 + rows <= N
        if rows:
            assert row0 == r * R  # all-gather slot of rank r
        covered += range(row0, row0 + rows)
    assert covered == list(range(N))
