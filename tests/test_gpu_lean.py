"""GPU parity of the lean relay update (k_lean_relay): one large problem's
updateY2 streaming Qd itself (4 B per entry; lanes 2i and 2i + 1 read row i's
packet and form its num / den terms in registers) instead of the stored split
matrices.  Default for blocks of rows x n_dual >= 4096^2; forced here at every
size through pqp_tune_lean_min_n.  Bar: bit-exact against the oracle (inf /
NaN / -0 included), the golden fixed-999 iterate, and the split-matrix relay."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import CAP, assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture
def lean(gpu_lib):
    L = gpu_lib.lib()
    prev = L.pqp_tune_lean_min_n(1)
    yield L
    L.pqp_tune_lean_min_n(prev)


def _blocks(N, cuts):
    edges = [0] + list(cuts) + [N]
    return [(a, b - a) for a, b in zip(edges[:-1], edges[1:])]


def _run_blocks(torch, blocks, N, updates, Y0=None):
    Y = torch.full((N,), 1000.0, device="cuda") if Y0 is None else torch.as_tensor(Y0, device="cuda")
    for _ in range(updates):
        Yn = torch.empty(N, device="cuda")
        for blk in blocks:
            if blk.rows:
                blk.update(Y, Yn[blk.row0:blk.row0 + blk.rows])
        Y = Yn
    return Y.cpu().numpy()


def _same_bits_or_both_nan(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(nan | (a.view(np.uint32) == b.view(np.uint32))))


@pytest.mark.parametrize("N,cuts", [(1, []), (28, [9, 10]), (63, [8, 9, 40]), (300, [64, 65, 255]),
                                    (1025, [1, 512, 1000]), (2100, [700, 733])])
def test_lean_rowblocks_vs_oracle(gpu_lib, orc, lean, N, cuts):
    """Ragged row blocks (diagonals at every offset of a segment and of a
    workgroup, one-row blocks, several segments per wave at N = 2100)."""
    import torch

    P = orc.synth_problem(13, 2, N, max(1, N // 2), with_qp=False)
    Qd = torch.from_numpy(P["Qd"]).cuda()
    Fd = torch.from_numpy(P["Fd"]).cuda()
    blocks = [gpu_lib.RowBlock(Qd[r0 * N:], Fd, N, r0, rows) for r0, rows in _blocks(N, cuts)]
    got = _run_blocks(torch, blocks, N, 5)
    assert_bitwise(got, orc.iterate(P["Qd"], P["Fd"], N, 5), f"N={N} cuts={cuts}")


def test_lean_rowblock_bundled_fixed_999(gpu_lib, golden_bundled, lean):
    import torch

    g = golden_bundled
    N = int(g["N"])
    Qd = torch.from_numpy(np.ascontiguousarray(g["Qd"], np.float32)).cuda()
    Fd = torch.from_numpy(np.ascontiguousarray(g["Fd"], np.float32)).cuda()
    blocks = [gpu_lib.RowBlock(Qd[r0 * N:], Fd, N, r0, rows) for r0, rows in _blocks(N, [7, 14, 21])]
    assert_bitwise(_run_blocks(torch, blocks, N, 999), g["Y_fixed999"], "lean row blocks, 999 updates")


@pytest.mark.parametrize("N", [7, 300, 1030])
def test_lean_special_values_vs_oracle(gpu_lib, orc, lean, N):
    """inf / NaN / +-0 in Qd, Fd and Y propagate exactly as in the literal
    reference formula (the lean form's z = 0*y, the literal diagonal)."""
    import torch

    rng = np.random.default_rng(N + 1)
    Qd = rng.standard_normal((N, N)).astype(np.float32)
    Qd[rng.random((N, N)) < 0.1] = 0.0
    Qd[rng.random((N, N)) < 0.05] = -0.0
    Qd[rng.random((N, N)) < 0.002] = np.nan
    Qd = Qd.reshape(-1)
    Fd = rng.standard_normal(N).astype(np.float32)
    Fd[::7] = -0.0
    th = orc.theta(Qd, N)
    dQ, dF = torch.from_numpy(Qd).cuda(), torch.from_numpy(Fd).cuda()
    blocks = [gpu_lib.RowBlock(dQ[r0 * N:], dF, N, r0, rows) for r0, rows in _blocks(N, [N // 2] if N > 1 else [])]
    for trial in range(3):
        Y = (rng.random(N) * 100).astype(np.float32)
        if trial >= 1:
            Y[rng.integers(0, N, 3)] = np.inf
            Y[rng.integers(0, N, 2)] = 0.0
        if trial == 2:
            Y[rng.integers(0, N, 2)] = np.nan
        want = orc.update(Y, Qd, th, Fd, N)
        got = _run_blocks(torch, blocks, N, 1, Y0=Y)
        assert _same_bits_or_both_nan(got, want), f"N={N} trial={trial}"


@pytest.mark.parametrize("num_iter", [2, 257, 300])
def test_lean_problem_fixed_mode(gpu_lib, lean, num_iter):
    """Fixed mode of a large problem (the graph-replayed relay, N > 1024) on
    the lean layout == the oracle-pinned batched kernel."""
    N, M = 1500, 750
    pb = gpu_lib.ProblemBatch.synthetic(4, 2, 1, N, M)
    P = pb.problem(0)
    with gpu_lib.Problem(P) as prob:
        r = prob.solve(gpu_lib.MODE_FIXED, num_iter=num_iter)
    want = gpu_lib.Batch(1, N).load(P["Qd"][None, :], P["Fd"][None, :]).iterate(num_iter - 1).result()[0]
    assert r["h"] == num_iter
    assert_bitwise(r["Y"], want, f"num_iter={num_iter}")


def test_lean_converge_graph_chain_testfile(gpu_lib, orc, lean, tmp_path):
    """Converge mode of testing/ test1.txt (n_dual 1500: the graph chain of
    pqp_wide.hip) with its update on the lean layout: the reference's h = 4,
    Y and U bit for bit."""
    from test_gpu_wide import _testing_file

    P = gpu_lib.testfile_problem(_testing_file("test1.txt", tmp_path))
    r = gpu_lib.solve_dual(P, max_updates=CAP)
    h, Y, U = orc.solve(P, max_updates=CAP)
    assert r["h"] == abs(h) and r["converged"] == (h > 0)
    assert_bitwise(r["Y"], Y, "Y")
    assert_bitwise(r["U"], U, "U")


def test_lean_matches_split_relay_large(gpu_lib):
    """n_dual 4608 in 3 ragged blocks: the lean relay and the split-matrix
    relay give the same bits."""
    import torch

    N, ups = 4608, 3
    L = gpu_lib.lib()
    cuts = [1500, 1501]
    got = {}
    for name, min_n in (("lean", 1), ("split", 0)):
        prev = L.pqp_tune_lean_min_n(min_n)
        try:
            blocks = [gpu_lib.RowBlock.synthetic(9, 1, N, r0, rows)[0] for r0, rows in _blocks(N, cuts)]
            got[name] = _run_blocks(torch, blocks, N, ups)
        finally:
            L.pqp_tune_lean_min_n(prev)
        del blocks
    assert_bitwise(got["lean"], got["split"], "lean vs split")
    assert np.all(np.isfinite(got["lean"]))
