"""GPU parity of converge mode over many workgroups (pqp_wide.hip): one
problem's terminate() as multi-workgroup mat-vecs plus the relay update,
replayed from a hipGraph.  Bar: the reference's h, and Y*, U*, Jp, Jd bit
for bit (golden fixtures from the compiled reference, and the oracle)."""
from __future__ import annotations

import gzip

import numpy as np
import pytest

from conftest import CAP, GOLDEN, assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture
def wide_everywhere(gpu_lib):
    """Route every converge-mode solve, LDS-sized ones included, to the wide path."""
    L = gpu_lib.lib()
    prev = L.pqp_tune_wide_min_n(0)
    yield
    L.pqp_tune_wide_min_n(prev)


def test_wide_converge_fixtures(gpu_lib, golden_converge, orc, wide_everywhere):
    """The converging synthetic cases (h from 3 to several thousand, odd and
    even) against the reference's Y* and U*."""
    cases, Ys, Us = golden_converge["cases"], golden_converge["Y"], golden_converge["U"]
    yo = uo = 0
    for (N, M, seed, h_ref) in cases:
        N, M = int(N), int(M)
        P = orc.synth_problem(int(seed), 0, N, M)
        r = gpu_lib.solve_dual(P, max_updates=CAP)
        assert r["converged"] and r["h"] == int(h_ref), (N, M, seed, r["h"])
        assert_bitwise(r["Y"], Ys[yo:yo + N], f"Y {N}/{M}/{seed}")
        assert_bitwise(r["U"], Us[uo:uo + M], f"U {N}/{M}/{seed}")
        yo += N
        uo += M


def test_wide_bundled_converge(gpu_lib, golden_bundled, wide_everywhere):
    g = golden_bundled
    P = {k: np.ascontiguousarray(g[k], dtype=np.float32) for k in
         ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
    P.update(N=int(g["N"]), M=int(g["M"]))
    r = gpu_lib.solve_dual(P, max_updates=CAP)
    assert r["converged"] and r["h"] == 313
    assert_bitwise(r["Y"], g["Ystar"], "Y*")
    assert_bitwise(r["U"], g["Ustar"], "U*")
    assert np.float32(r["Jp"]) == g["iter_Jp"][-1] and np.float32(r["Jd"]) == g["iter_Jd"][-1]


def _testing_file(name, tmp_path):
    """The reference's testing/sample test/<name> (committed, gzip'd for the
    two large ones)."""
    plain = GOLDEN / "testing" / name
    if plain.exists():
        return plain
    out = tmp_path / name
    out.write_bytes(gzip.decompress((GOLDEN / "testing" / (name + ".gz")).read_bytes()))
    return out


@pytest.mark.parametrize("name,cap", [("test1.txt", CAP), ("test2.txt", CAP), ("test3.txt", 60)])
def test_wide_testing_files_vs_oracle(gpu_lib, orc, name, cap, tmp_path):
    """The reference's testing/ sample problems (n_dual 1500, 400, 1200) on
    the default routing (all >= the wide threshold): test1/test2 converge in a
    few iterations, test3 is capped."""
    P = gpu_lib.testfile_problem(_testing_file(name, tmp_path))
    assert P["N"] >= 384
    r = gpu_lib.solve_dual(P, max_updates=cap)
    h, Y, U = orc.solve(P, max_updates=cap)
    assert r["h"] == abs(h) and r["converged"] == (h > 0), (r["h"], h)
    assert_bitwise(r["Y"], Y, f"{name} Y")
    assert_bitwise(r["U"], U, f"{name} U")


def test_wide_matches_one_workgroup_solver(gpu_lib, orc):
    """A capped synthetic n_dual = 1024 solve: the wide path and the
    one-workgroup k_solve_single give the same h, Y, U, Jp, Jd, and both
    equal the oracle."""
    N, M, cap = 1024, 512, 25
    P = orc.synth_problem(3, 1, N, M)
    L = gpu_lib.lib()
    wide = gpu_lib.solve_dual(P, max_updates=cap)
    prev = L.pqp_tune_set_variant(0x200)  # one workgroup
    try:
        single = gpu_lib.solve_dual(P, max_updates=cap)
    finally:
        L.pqp_tune_set_variant(prev)
    assert wide["h"] == single["h"] == cap + 1 and not wide["converged"]
    for k in ("Y", "U"):
        assert_bitwise(wide[k], single[k], k)
    assert (np.isnan(wide["Jp"]) and np.isnan(single["Jp"])) or np.float32(wide["Jp"]) == np.float32(single["Jp"])
    h, Y, U = orc.solve(P, max_updates=cap)
    assert abs(h) == wide["h"]
    assert_bitwise(wide["Y"], Y, "Y vs oracle")
    assert_bitwise(wide["U"], U, "U vs oracle")


def test_wide_repeated_solves_and_odd_even(gpu_lib, golden_converge, orc, wide_everywhere):
    """The captured graph is reused across solves and caps (odd and even
    update counts leave the iterate in either ping-pong buffer)."""
    N, M, seed, h_ref = (int(v) for v in golden_converge["cases"][0])
    P = orc.synth_problem(seed, 0, N, M)
    with gpu_lib.Problem(P) as prob:
        for cap in (7, 8, 7, CAP):
            r = prob.solve(max_updates=cap)
            h, Y, U = orc.solve(P, max_updates=cap)
            assert r["h"] == abs(h)
            assert_bitwise(r["Y"], Y, f"cap {cap}")
            assert_bitwise(r["U"], U, f"cap {cap}")


def test_device_synthetic_primal_matches_oracle(gpu_lib, orc):
    """pqp_batch_synth_primal + Gauss_Jordan + convertToDual on the device ==
    the oracle's generator and setup, for every array."""
    B, N, M = 3, 300, 150
    pb = gpu_lib.ProblemBatch.synthetic(5, 11, B, N, M)
    for b in range(B):
        got = pb.problem(b)
        want = orc.synth_problem(5, 11 + b, N, M)
        for k in ("Qp_inv", "Gp", "Kp", "Fp", "Mp", "Qp", "Qd", "Fd", "Md"):
            assert_bitwise(got[k], np.asarray(want[k], np.float32).reshape(-1), f"problem {b} {k}")


@pytest.mark.parametrize("n,B", [(64, 1), (130, 2), (300, 1)])
def test_gauss_jordan_many_workgroups_vs_oracle(gpu_lib, orc, n, B):
    """Gauss_Jordan of large matrices, one launch per pivot: bit-identical to
    the reference's restatement, including the bubble pass on column 0
    (column 0 random, so rows are swapped)."""
    import torch

    rng = np.random.default_rng(n)
    A = rng.standard_normal((B, n, n)).astype(np.float32)
    A += np.eye(n, dtype=np.float32)[None] * n  # well conditioned
    dA = torch.from_numpy(A.reshape(B, -1)).cuda()
    dR = torch.zeros_like(dA)
    L = gpu_lib.lib()
    gpu_lib._check(L.pqp_batch_gauss_jordan(B, n, gpu_lib.C.c_void_p(dA.data_ptr()),
                                            gpu_lib.C.c_void_p(dR.data_ptr()),
                                            gpu_lib.C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    got = dR.cpu().numpy()
    for b in range(B):
        assert_bitwise(got[b], orc.gauss_jordan(A[b].reshape(-1), n), f"inverse {b}")


def test_problem_beyond_one_workgroup_budget(gpu_lib, orc):
    """n_dual = 9000 is past the one-workgroup solver's LDS budget: the problem
    handle still solves it in converge mode (wide path) and fixed mode (relay
    update), bit-identical to the oracle on the same dual data."""
    N, M, cap = 9000, 4500, 2
    pb = gpu_lib.ProblemBatch.synthetic(8, 0, 1, N, M)
    P = pb.problem(0)
    del pb
    with gpu_lib.Problem(P) as prob:
        r = prob.solve(max_updates=cap)
        f = prob.solve(gpu_lib.MODE_FIXED, num_iter=3)
    h, Y, U = orc.solve(P, max_updates=cap)
    assert r["h"] == abs(h) == cap + 1
    assert_bitwise(r["Y"], Y, "converge Y")
    assert_bitwise(r["U"], U, "converge U")
    assert_bitwise(f["Y"], orc.iterate(P["Qd"], P["Fd"], N, 2), "fixed-mode Y")


def _gj_batch(gpu_lib, A, form):
    """pqp_batch_gauss_jordan of the matrices A (B x n x n) on `form`: 3
    k_gj_blocked3, 0 the per-sweep kernel (k_gj_blocked / k_gj_blocked2, the
    forms 1 and 2 of rounds 3-5, were removed in round 6); B > 8 keeps large n
    off the one-launch-per-pivot path (replicated)."""
    import torch

    B, n = A.shape[0], A.shape[1]
    L = gpu_lib.lib()
    reps = 9 if n >= 64 and B <= 8 else 1
    dA = torch.from_numpy(np.ascontiguousarray(A).reshape(B, -1)).cuda().repeat(reps, 1)
    dR = torch.zeros_like(dA)
    prev = L.pqp_tune_gj_blocked(0 if form else 1)
    try:
        gpu_lib._check(L.pqp_batch_gauss_jordan(B * reps, n, gpu_lib.C.c_void_p(dA.data_ptr()),
                                                gpu_lib.C.c_void_p(dR.data_ptr()),
                                                gpu_lib.C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    finally:
        L.pqp_tune_gj_blocked(prev)
    return dR.cpu().numpy().reshape(reps, B, n * n)


def _same_bits_or_nan(got, want, what):
    got, want = np.asarray(got, np.float32), np.asarray(want, np.float32)
    nan = np.isnan(got) & np.isnan(want)
    bad = np.nonzero(~nan & (got.view(np.uint32) != want.view(np.uint32)))[0]
    assert bad.size == 0, f"{what}: {bad.size} values differ; first at {bad[0]}: {got[bad[0]]!r} vs {want[bad[0]]!r}"


@pytest.mark.parametrize("kind", ["zero_pivot", "nan_entry", "inf_entry", "neg_zero", "singular_late"])
@pytest.mark.parametrize("n", [20, 100, 300])
def test_gauss_jordan_nonfinite_vs_oracle(gpu_lib, orc, n, kind):
    """Inputs that make a multiplier inf or NaN (a zero pivot, a NaN or inf
    entry, a row that turns singular late) or carry -0: k_gj_blocked3 skips
    right columns that are still exactly zero only while every multiplier is
    finite, so these must match the reference as the full kernels do (NaN
    positions; every other bit)."""
    rng = np.random.default_rng(77 + n)
    A = rng.standard_normal((2, n, n)).astype(np.float32)
    A += np.eye(n, dtype=np.float32)[None] * n
    if kind == "zero_pivot":
        A[:, 3, :] = 0.0  # row 3 all zero: its pivot is 0, t = m / 0
    elif kind == "nan_entry":
        A[0, n // 2, n // 3] = np.nan
        A[1, 5, 7] = np.nan
    elif kind == "inf_entry":
        A[0, n - 2, 1] = np.inf
        A[1, 2, n - 1] = -np.inf
    elif kind == "neg_zero":
        A[:, :, n // 2] = -0.0
        A[:, n // 2, n // 2] = 1.0
    else:  # row n - 5 a copy of row n - 6: its pivot cancels to zero late
        A[:, n - 5, :] = A[:, n - 6, :]
    want = [orc.gauss_jordan(A[b].reshape(-1), n) for b in range(2)]
    for form in (3, 0):
        if form == 0 and n >= 300:
            continue  # the per-sweep kernel at this size only costs time
        got = _gj_batch(gpu_lib, A, form)
        for r in range(got.shape[0]):
            for b in range(2):
                _same_bits_or_nan(got[r, b], want[b], f"{kind} form {form} inverse {b} copy {r}")


@pytest.mark.parametrize("n,B", [(1, 3), (7, 5), (15, 2), (16, 2), (17, 2), (63, 2), (100, 3), (256, 2), (300, 2),
                                 (385, 1), (512, 2), (640, 1), (1024, 1)])
@pytest.mark.parametrize("blocked", [3, 0])
def test_gauss_jordan_blocked_vs_oracle(gpu_lib, orc, n, B, blocked):
    """The blocked batched Gauss_Jordan (pivots 16 or 8 at a time, one pass
    over the augmented matrix per panel: k_gj_blocked3 over the columns that
    can still change an output) and
    the one-pivot-per-sweep kernel: bit-identical to the reference's
    restatement (PQP_CPU.c:251-326), including the bubble pass (column 0
    random, rows swapped), ragged panels and both register layouts (n <= 512:
    16-pivot panels, above: 8)."""
    import torch

    if n >= 640 and not blocked:
        pytest.skip("the per-sweep kernel at this size only costs time")
    rng = np.random.default_rng(1000 + n)
    A = rng.standard_normal((B, n, n)).astype(np.float32)
    A += np.eye(n, dtype=np.float32)[None] * n  # well conditioned
    dA = torch.from_numpy(A.reshape(B, -1)).cuda()
    dR = torch.zeros_like(dA)
    L = gpu_lib.lib()
    prev = L.pqp_tune_gj_blocked(0 if blocked else 1)
    try:
        # B > 8 keeps large n off the one-launch-per-pivot path: replicate
        reps = 9 if n >= 64 else 1
        dA9 = dA.repeat(reps, 1)
        dR9 = torch.zeros_like(dA9)
        gpu_lib._check(L.pqp_batch_gauss_jordan(B * reps, n, gpu_lib.C.c_void_p(dA9.data_ptr()),
                                                gpu_lib.C.c_void_p(dR9.data_ptr()),
                                                gpu_lib.C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    finally:
        L.pqp_tune_gj_blocked(prev)
    got = dR9.cpu().numpy()
    for b in range(B):
        want = orc.gauss_jordan(A[b].reshape(-1), n)
        for r in range(reps):
            assert_bitwise(got[r * B + b], want, f"inverse {b} copy {r}")
