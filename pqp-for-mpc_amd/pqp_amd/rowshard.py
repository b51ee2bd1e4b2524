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
        self.device = torch.device(device)
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
        self.graph = None  # (torch.cuda.CUDAGraph, steps) once capture() succeeded
        self.capture_error = None

    def step(self):
        """One updateY2 of the whole problem: Y <- Y_next.  With a process
        group the new rows always go through the all-gather, also at world
        size 1 (a one-rank RCCL group then exercises the captured collective)."""
        if self.dist is None:
            self.block.update(self.Y, self.Y2)
        else:
            self.block.update(self.Y, self.local)
            self.dist.all_gather_into_tensor(self.Y2, self.local, group=self.group)
        self.Y, self.Y2 = self.Y2, self.Y

    def block_steps(self, updates: int):
        """`updates` block updates with NO collective (Y is left as it is):
        what each update costs this rank without the all-gather, for the
        bench's `allgather_us_per_update` (the eager step minus this)."""
        out = self.local if self.dist is not None else self.Y2
        for _ in range(int(updates)):
            self.block.update(self.Y, out)

    def capture(self, steps: int = 16) -> bool:
        """Record `steps` (even) updates -- each rank's block update and the
        RCCL all-gather -- as ONE hipGraph, replayed by :meth:`run`.  This
        removes the per-update host launches and the cross-stream event waits
        the eager collective adds between the update kernel and the gather.

        Every rank must call it (the ranks agree on the outcome over an eager
        all-reduce, so either all of them replay or none does).  Returns False
        (and stays eager) where capture is not possible: gloo groups (CPU
        collectives) or a capture error on any rank.  Clobbers Y: call it
        before :meth:`run`, which re-fills Y."""
        torch = self.torch
        steps = int(steps)
        if steps <= 0 or steps % 2:
            raise ValueError("capture(steps): steps must be a positive even number (Y / Y2 end where they began)")
        gloo = self.dist is not None and self.dist.get_backend(self.group) == "gloo"
        ok = self.device.type == "cuda" and not gloo
        if ok:
            try:
                self.Y.fill_(0.0)
                for _ in range(2):  # communicator and kernels set up outside the capture
                    self.step()
                torch.cuda.synchronize(self.device)
                self._graph_in = self.Y  # the buffer every replay starts from (and ends in: steps is even)
                g = torch.cuda.CUDAGraph()
                side = torch.cuda.Stream(self.device)
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.graph(g, stream=side):
                    for _ in range(steps):
                        self.step()
                torch.cuda.current_stream(self.device).wait_stream(side)
            except Exception as e:  # noqa: BLE001 -- reported through the agreement below
                self.capture_error = f"{type(e).__name__}: {e}"
                ok = False
                g = None
        if self.dist is not None and not gloo:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
            self.dist.all_reduce(flag, op=self.dist.ReduceOp.MIN, group=self.group)
            ok = bool(flag.item())
        self.graph = (g, steps) if ok else None
        return ok

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
        self.advance(max(0, int(num_iter) - 1))
        self.check()
        return self.Y[: self.N]

    def advance(self, updates: int):
        """`updates` steps: whole replays of the captured graph (if any), then
        eager steps for the remainder."""
        left = int(updates)
        if self.graph is not None and left >= self.graph[1]:
            g, steps = self.graph
            if self.Y is not self._graph_in:  # odd eager steps since capture: the graph reads the other buffer
                self._graph_in.copy_(self.Y)
                self.Y, self.Y2 = self.Y2, self.Y
            while left >= steps:
                g.replay()
                left -= steps
        for _ in range(left):
            self.step()
