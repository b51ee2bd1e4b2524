"""GPU parity of the row-sharded single-problem path:
pqp_rowblock_* / pqp_synth_rows through the C ABI and the
pqp_amd.rowshard driver.  Bar: bit-exact against the reference's golden
vectors and the oracle, for any partition of the rows."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from conftest import ROOT, assert_bitwise

pytestmark = pytest.mark.gpu


def _blocks(N, cuts):
    edges = [0] + list(cuts) + [N]
    return [(a, b - a) for a, b in zip(edges[:-1], edges[1:])]


def _run_blocks(torch, blocks, N, updates):
    """Assemble Y_next from the blocks after every update (single process)."""
    Y = torch.full((N,), 1000.0, device="cuda")
    for _ in range(updates):
        Yn = torch.empty(N, device="cuda")
        for blk in blocks:
            if blk.rows:
                blk.update(Y, Yn[blk.row0:blk.row0 + blk.rows])
        Y = Yn
    return Y.cpu().numpy()


@pytest.mark.parametrize("N,cuts", [(28, [9, 10]), (300, [64, 65, 255]), (1025, [1, 512, 1000])])
def test_rowblocks_assemble_updateY2(gpu_lib, orc, N, cuts):
    import torch

    P = orc.synth_problem(13, 2, N, max(1, N // 2), with_qp=False)
    Qd = torch.from_numpy(P["Qd"]).cuda()
    Fd = torch.from_numpy(P["Fd"]).cuda()
    blocks = [gpu_lib.RowBlock(Qd[r0 * N:], Fd, N, r0, rows) for r0, rows in _blocks(N, cuts)]
    got = _run_blocks(torch, blocks, N, 5)
    assert_bitwise(got, orc.iterate(P["Qd"], P["Fd"], N, 5), f"N={N} cuts={cuts}")


_VARIANT_CASES = {}


def _variant_case(orc, N):
    if N not in _VARIANT_CASES:
        P = orc.synth_problem(17, 1, N, max(1, N // 2), with_qp=False)
        _VARIANT_CASES[N] = (P, orc.iterate(P["Qd"], P["Fd"], N, 3))
    return _VARIANT_CASES[N]


@pytest.mark.parametrize("lwsel", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("N", [28, 1025, 2100])
def test_split_kernel_variants_vs_oracle(gpu_lib, orc, lwsel, N):
    """The relay update behind pqp_rowblock_update (k_split_relay) at every
    workgroup width (8..64 row sides per workgroup, pqp_tune_set_variant), on
    ragged blocks; at N = 2100 a wave sums several segments."""
    import torch

    P, want = _variant_case(orc, N)
    Qd = torch.from_numpy(P["Qd"]).cuda()
    Fd = torch.from_numpy(P["Fd"]).cuda()
    L = gpu_lib.lib()
    prev = L.pqp_tune_set_variant(lwsel << 17)
    try:
        cuts = [N // 3, N // 3 + min(33, N // 3)]
        blocks = [gpu_lib.RowBlock(Qd[r0 * N:], Fd, N, r0, rows) for r0, rows in _blocks(N, cuts)]
        got = _run_blocks(torch, blocks, N, 3)
    finally:
        L.pqp_tune_set_variant(prev)
    assert_bitwise(got, want, f"lw={lwsel} N={N}")


def test_rowblock_bundled_fixed_999(gpu_lib, golden_bundled):
    import torch

    g = golden_bundled
    N = int(g["N"])
    Qd = torch.from_numpy(np.ascontiguousarray(g["Qd"], np.float32)).cuda()
    Fd = torch.from_numpy(np.ascontiguousarray(g["Fd"], np.float32)).cuda()
    blocks = [gpu_lib.RowBlock(Qd[r0 * N:], Fd, N, r0, rows) for r0, rows in _blocks(N, [7, 14, 21])]
    assert_bitwise(_run_blocks(torch, blocks, N, 999), g["Y_fixed999"], "row blocks, 999 updates")


@pytest.mark.parametrize("tag", ["n1024_m512_s1_i0", "n1000_m500_s2_i7"])
def test_synth_rows_and_solver_match_reference(gpu_lib, golden_large, tag):
    """pqp_synth_rows blocks + RowShardedSolver (one rank) against the
    compiled reference's Fd / Md / Y after `ups` updates."""
    import torch

    from pqp_amd.rowshard import RowShardedSolver

    N, M, seed, inst, ups = (int(v) for v in golden_large[f"{tag}_meta"])
    blk, Fd, Md = gpu_lib.RowBlock.synthetic(seed, inst, N, 0, N, M=M)
    assert_bitwise(Fd.cpu().numpy(), golden_large[f"{tag}_Fd"], "Fd")
    assert_bitwise(Md.cpu().numpy(), golden_large[f"{tag}_Md"], "Md")
    y = RowShardedSolver(blk, N, torch.device("cuda")).run(ups + 1)
    assert_bitwise(y.cpu().numpy(), golden_large[f"{tag}_Y"], "row-sharded Y")
    # the same problem in ragged synthetic blocks
    parts = [gpu_lib.RowBlock.synthetic(seed, inst, N, r0, rows, M=M)[0] for r0, rows in _blocks(N, [100, 101, 700])]
    assert_bitwise(_run_blocks(torch, parts, N, ups), golden_large[f"{tag}_Y"], "ragged synthetic blocks")


def test_rowsharded_full_size_vs_batch_kernel(gpu_lib):
    """A large single problem (N = 8192, 512 MiB of split matrices) in four
    blocks == the oracle-pinned batched kernel on the same problem."""
    import torch

    N, ups = 8192, 3
    R = N // 4
    blocks = [gpu_lib.RowBlock.synthetic(21, 3, N, r * R, R)[0] for r in range(4)]
    got = _run_blocks(torch, blocks, N, ups)
    want = gpu_lib.Batch(1, N).generate(21, inst0=3).iterate(ups).result()[0]
    assert_bitwise(got, want, "N=8192 row blocks vs batch kernel")
    assert np.all(np.isfinite(got)) and np.all(got >= 0)
    del blocks
    torch.cuda.empty_cache()


def test_rowblock_argument_validation(gpu_lib):
    import torch

    Q = torch.zeros(16, device="cuda")
    Fd = torch.zeros(4, device="cuda")
    with pytest.raises(gpu_lib.PQPError):
        gpu_lib.RowBlock(Q, Fd, 4, 3, 2)  # rows past N
    with pytest.raises(gpu_lib.PQPError):
        gpu_lib.RowBlock(Q, Fd, 40000, 0, 0)  # y does not fit in LDS
    empty = gpu_lib.RowBlock(None, Fd, 4, 4, 0)  # a rank with no rows
    empty.update(torch.zeros(4, device="cuda"), torch.zeros(0, device="cuda"))


# ---------------------------------------------------------------------------
# two processes on the one GPU.  RCCL needs one device per rank, so this
# test moves the all-gather through gloo on host copies (test-only adapter);
# the product code path (RowBlock + RowShardedSolver) is unchanged.
# ---------------------------------------------------------------------------
class _HostStagedDist:
    def __init__(self, dist):
        self.d = dist

    def get_world_size(self, group=None):
        return self.d.get_world_size()

    def get_rank(self, group=None):
        return self.d.get_rank()

    def all_gather_into_tensor(self, out, inp, group=None):
        o = out.cpu()
        self.d.all_gather_into_tensor(o, inp.cpu())
        out.copy_(o)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, N, ups, out):
    import sys

    for p in (ROOT / "pqp-for-mpc_amd", ROOT / "oracle"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    import pqp_amd
    from pqp_amd.rowshard import RowShardedSolver, row_plan

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    _, plan = row_plan(N, world)
    blk, _, _ = pqp_amd.RowBlock.synthetic(5, 9, N, *plan[rank])
    y = RowShardedSolver(blk, N, torch.device("cuda"), dist=_HostStagedDist(dist)).run(ups + 1)
    np.save(f"{out}.{rank}.npy", y.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 1030), (3, 4)])
def test_rowsharded_two_processes(gpu_lib, orc, tmp_path, world, N):
    """2 ranks on a ragged N, and 3 ranks on N = 4 (the last rank owns no rows)."""
    import torch.multiprocessing as mp

    ups = 6
    out = str(tmp_path / "y")
    mp.spawn(_rank_main, args=(world, _free_port(), N, ups, out), nprocs=world, join=True)
    P = orc.synth_problem(5, 9, N, max(1, N // 2), with_qp=False)
    want = orc.iterate(P["Qd"], P["Fd"], N, ups)
    for r in range(world):
        assert_bitwise(np.load(f"{out}.{r}.npy"), want, f"rank {r}")


def _graph_rank_main(rank, world, port, N, ups, out):
    import sys

    for p in (ROOT / "pqp-for-mpc_amd", ROOT / "oracle"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    import pqp_amd
    from pqp_amd.rowshard import RowShardedSolver

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    blk, _, _ = pqp_amd.RowBlock.synthetic(5, 9, N, 0, N)
    solver = RowShardedSolver(blk, N, dev, dist=dist)
    ok = solver.capture(4)
    y = solver.run(ups + 1)  # 3 replays of 4 updates + 1 eager step at ups = 13
    np.save(f"{out}.npy", y.cpu().numpy())
    np.save(f"{out}.ok.npy", np.array([1 if ok else 0]))
    dist.destroy_process_group()


def test_rowsharded_graph_rccl_one_rank(gpu_lib, orc, tmp_path):
    """RowShardedSolver.capture over a one-rank RCCL group: the block update
    and the all-gather recorded as one hipGraph, replayed three times plus an
    eager remainder, give the oracle's iterate bit for bit."""
    import torch.multiprocessing as mp

    N, ups = 1030, 13
    out = str(tmp_path / "g")
    mp.spawn(_graph_rank_main, args=(1, _free_port(), N, ups, out), nprocs=1, join=True)
    assert int(np.load(f"{out}.ok.npy")[0]) == 1, "capture over RCCL failed"
    P = orc.synth_problem(5, 9, N, max(1, N // 2), with_qp=False)
    assert_bitwise(np.load(f"{out}.npy"), orc.iterate(P["Qd"], P["Fd"], N, ups), "graph-replayed row shard")


def test_rowsharded_graph_no_group(gpu_lib, orc):
    """capture() without a process group (one GPU): block updates only."""
    import torch

    from pqp_amd.rowshard import RowShardedSolver

    N, ups = 300, 9
    blk, _, _ = gpu_lib.RowBlock.synthetic(5, 9, N, 0, N)
    solver = RowShardedSolver(blk, N, torch.device("cuda"))
    assert solver.capture(2)
    P = orc.synth_problem(5, 9, N, max(1, N // 2), with_qp=False)
    want = orc.iterate(P["Qd"], P["Fd"], N, ups)
    assert_bitwise(solver.run(ups + 1).cpu().numpy(), want, "graph replays, no group")
    assert_bitwise(solver.run(ups + 1).cpu().numpy(), want, "graph replays, second run")
    with pytest.raises(ValueError):
        solver.capture(3)


@pytest.mark.parametrize("num_iter", [2, 257, 300, 513])
def test_fixed_mode_graph_chunks(gpu_lib, num_iter):
    """Fixed mode of a large problem replays 256-update graph chunks plus a
    remainder graph: every split of the update count gives the iterate of
    the (oracle-pinned) batched kernel run for num_iter - 1 updates."""
    N, M = 400, 200
    pb = gpu_lib.ProblemBatch.synthetic(4, 2, 1, N, M)
    P = pb.problem(0)
    with gpu_lib.Problem(P) as prob:
        r = prob.solve(gpu_lib.MODE_FIXED, num_iter=num_iter)
        r2 = prob.solve(gpu_lib.MODE_FIXED, num_iter=num_iter)  # graphs replayed
    b = gpu_lib.Batch(1, N).load(P["Qd"][None, :], P["Fd"][None, :])
    want = b.iterate(num_iter - 1).result()[0]
    assert r["h"] == num_iter
    assert_bitwise(r["Y"], want, f"num_iter={num_iter}")
    assert_bitwise(r2["Y"], want, f"num_iter={num_iter} (replay)")
