"""One large dual problem row-sharded across ranks.

Rank r owns the contiguous rows [r*R, r*R + rows_r) of updateY2
(PQP_CPU.c:603-618), R = ceil(N / world), as a :class:`pqp_amd.RowBlock`.
Every update needs the whole iterate, so each step is

    block.update(Y, Y_local)                   # this rank's rows of Y_next
    all_gather_into_tensor(Y_next, Y_local)    # RCCL over xGMI

with Y kept in a padded [world*R] buffer (rows >= N are never read: the
update kernel reads only Y[0:N]).  Row i's sums still run over k = 0..N-1 in
order on one lane, so the result is bit-identical to the single-process
solve for any world size.  Fixed-iteration mode only (the testing/ harness
mode): converge mode's terminate() needs the full Qd for Jd and stays on the
single-device solver.
"""
from __future__ import annotations


def row_plan(N: int, world: int) -> tuple[int, list[tuple[int, int]]]:
    """(R, [(row0, rows) for every rank]); the last ranks may get fewer (or 0) rows."""
    N, world = int(N), int(world)
    if N <= 0 or world <= 0:
        raise ValueError("N and world must be positive")
    R = -(-N // world)
    return R, [(min(r * R, N), max(0, min(R, N - r * R))) for r in range(world)]


class RowShardedSolver:
    """Fixed-mode solve of one problem whose rows are spread over the ranks.

    `block` is this rank's row block: anything with ``row0``, ``rows`` and
    ``update(Y, Y_rows)`` (a :class:`pqp_amd.RowBlock` on the GPU).  `dist` is
    ``torch.distributed`` (or None for one rank); the backend is the caller's
    ("nccl" = RCCL on the GPUs, "gloo" in the CPU tests).
    """

    def __init__(self, block, N: int, device, dist=None, group=None):
        import torch

        self.torch = torch
        self.block = block
        self.N = int(N)
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist is not None else 1
        self.rank = dist.get_rank(group) if dist is not None else 0
        self.R, plan = row_plan(self.N, self.world)
        if (block.row0, block.rows) != plan[self.rank]:
            raise ValueError(f"rank {self.rank}: block rows {(block.row0, block.rows)} != plan {plan[self.rank]}")
        kw = dict(dtype=torch.float32, device=device)
        self.Y = torch.empty(self.world * self.R, **kw)
        self.Y2 = torch.empty(self.world * self.R, **kw)
        self.local = torch.zeros(self.R, **kw)

    def step(self):
        """One updateY2 of the whole problem: Y <- Y_next."""
        if self.world == 1:
            self.block.update(self.Y, self.Y2)
        else:
            self.block.update(self.Y, self.local)
            self.dist.all_gather_into_tensor(self.Y2, self.local, group=self.group)
        self.Y, self.Y2 = self.Y2, self.Y

    def check(self):
        """Raise if any of this rank's block updates since the last check
        reported an expired in-kernel wait (blocks without a ``check`` -- the
        CPU stand-ins of the tests -- cannot fail that way)."""
        chk = getattr(self.block, "check", None)
        if chk is not None:
            chk()

    def run(self, num_iter: int = 1000, y0: float = 1000.0):
        """The reference's fixed mode: Y = 1000, then num_iter-1 updates
        (``while (h < NUM_ITER)``).  Returns the final Y (N) on every rank."""
        self.Y.fill_(y0)
        for _ in range(max(0, int(num_iter) - 1)):
            self.step()
        self.check()
        return self.Y[: self.N]
