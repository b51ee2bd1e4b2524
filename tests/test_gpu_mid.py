"""Batched solves of mid-size problems on k_solve_mid: one
workgroup per problem with Gp, Qp_inv, Qp and either the reference's stored
split matrices (where they fit, about N <= 100) or Qd held in LDS once, the
update's split entries then formed on the fly (v_max_f32 form when the
problem's Qd holds no NaN, the reference's selects otherwise).
Bar: the oracle's h, Y and U bit for bit -- the bundled plant over H horizon
blocks (stops at the reference's h = 313), synthetic problems capped with
infeasible and all-feasible iterates, ragged sizes, a non-symmetric Qd, a NaN
in Qd, fixed mode, chunked launches -- and the same bits with the path turned
off (mid_off: k_solve_small / k_solve_single)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import CAP, assert_bitwise

pytestmark = pytest.mark.gpu

KEYS = ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")
MID = 3


def _batch(gpu_lib, Ps):
    N, M = int(Ps[0]["N"]), int(Ps[0]["M"])
    pb = gpu_lib.ProblemBatch(len(Ps), N, M)
    for k in KEYS:
        pb.set(k, np.stack([np.asarray(P[k], np.float32).reshape(-1) for P in Ps]))
    return pb


def _check(pb, b, h, Y, U, what):
    assert int(pb.h[b]) == abs(h), (what, int(pb.h[b]), h)
    assert int(pb.status[b]) == (1 if h > 0 else 2), (what, int(pb.status[b]))
    assert_bitwise(pb.Y[b].cpu().numpy(), Y, f"{what} Y")
    assert_bitwise(pb.U[b].cpu().numpy(), U, f"{what} U")


@pytest.fixture
def knobs(gpu_lib):
    """pqp_tune settings restored after the test."""
    saved = []

    def set_(key, value):
        saved.append((key, gpu_lib.tune(key, value)))

    yield set_
    for key, old in reversed(saved):
        gpu_lib.tune(key, old)


def _bundled(golden_bundled):
    P = {k: np.ascontiguousarray(golden_bundled[k], dtype=np.float32) for k in KEYS}
    P.update(N=int(golden_bundled["N"]), M=int(golden_bundled["M"]))
    return P


@pytest.mark.parametrize("H", [2, 3, 4, 5])
@pytest.mark.parametrize("mid_off,split", [(0, 0), (0, 1), (1, 0)])
def test_horizon_blocks_stop_like_reference(gpu_lib, golden_bundled, orc, knobs, H, mid_off, split):
    """The bundled plant as H diagonal blocks (n_dual 28 H) stops at h = 313
    (the oracle's, itself pinned to oracle/_ref for 9 and 36 blocks): 8 copies
    in one launch, every value bit for bit."""
    from oracle import block_diag_problem

    Q = block_diag_problem(_bundled(golden_bundled), H)
    knobs("mid_off", mid_off)
    knobs("mid_split", split)
    if not mid_off:
        assert gpu_lib.lib().pqp_batch_solve_path(Q["N"], Q["M"]) == MID
    pb = _batch(gpu_lib, [Q] * 8).solve(max_updates=CAP)
    h, Y, U = orc.solve(Q, max_updates=CAP)
    assert h == 313
    for b in (0, 7):
        _check(pb, b, h, Y, U, f"H={H} copy {b} mid_off={mid_off}")


@pytest.mark.parametrize("chunk", [1, 7, 50])
def test_horizon_blocks_chunked(gpu_lib, golden_bundled, orc, knobs, chunk):
    """Launches of `chunk` iterates per problem, resumed from Y in HBM: the
    stop lands inside a later launch, same bits."""
    from oracle import block_diag_problem

    Q = block_diag_problem(_bundled(golden_bundled), 3)
    knobs("batch_chunk", chunk)
    pb = _batch(gpu_lib, [Q] * 3).solve(max_updates=CAP)
    h, Y, U = orc.solve(Q, max_updates=CAP)
    for b in range(3):
        _check(pb, b, h, Y, U, f"chunk={chunk} copy {b}")


@pytest.mark.parametrize("N,M", [(33, 5), (40, 20), (57, 57), (64, 16), (100, 50), (127, 31), (150, 40)])
@pytest.mark.parametrize("feasible", [False, True])
@pytest.mark.parametrize("split", [0, 1])
def test_synthetic_capped_vs_oracle(gpu_lib, orc, knobs, N, M, feasible, split):
    """Capped solves of synthetic problems; `feasible`: Kp = 1e30, so every
    iterate runs all of computeCost and, from the second on, the Y'Qd sums
    ride in the update rows.  split 1: the stored-split form where its LDS
    fits (N <~ 100), 0: the Qd form (default)."""
    knobs("mid_split", split)
    assert gpu_lib.lib().pqp_batch_solve_path(N, M) == MID
    B, cap = 3, 9
    Ps = [orc.synth_problem(31, b, N, M) for b in range(B)]
    if feasible:
        for P in Ps:
            P["Kp"] = np.full(N, 1e30, np.float32)
    pb = _batch(gpu_lib, Ps).solve(max_updates=cap)
    for b, P in enumerate(Ps):
        h, Y, U = orc.solve(P, max_updates=cap)
        _check(pb, b, h, Y, U, f"{N}/{M} problem {b} feasible={feasible}")


@pytest.mark.parametrize("N,M", [(48, 24), (101, 25)])
@pytest.mark.parametrize("split", [0, 1])
def test_fixed_mode_vs_oracle(gpu_lib, orc, knobs, N, M, split):
    knobs("mid_split", split)
    Ps = [orc.synth_problem(32, b, N, M) for b in range(4)]
    pb = _batch(gpu_lib, Ps).solve(gpu_lib.MODE_FIXED, num_iter=40)
    assert np.all(pb.h.cpu().numpy() == 40)
    for b in (0, 3):
        _, Y, _ = orc.solve(Ps[b], mode=1, num_iter=40)
        assert_bitwise(pb.Y[b].cpu().numpy(), Y, f"fixed {b}")


@pytest.mark.parametrize("feasible", [False, True])
@pytest.mark.parametrize("split", [0, 1])
def test_non_symmetric_qd_mixed(gpu_lib, orc, knobs, feasible, split):
    """Problem 0's Qd is bit-symmetric, problem 1's is not (dense Qp_inv):
    the Y'Qd columns then run beside the update rows instead of inside them."""
    from pqp_amd import dense_qinv

    knobs("mid_split", split)
    N, M, cap = 96, 24, 7
    P0 = orc.synth_problem(33, 0, N, M)
    P1 = orc.synth_primal(33, 1, N, M)
    P1["Qp_inv"] = dense_qinv(33, M)
    P1["Qd"], P1["Fd"], P1["Md"] = orc.convert_to_dual(P1["Qp_inv"], P1["Gp"], P1["Kp"], P1["Fp"], P1["Mp"], N, M)
    P1["Qp"] = orc.gauss_jordan(P1["Qp_inv"], M)
    P1.update(N=N, M=M)
    Q1 = P1["Qd"].reshape(N, N)
    assert not np.array_equal(Q1.view(np.uint32), Q1.T.view(np.uint32))
    if feasible:
        for P in (P0, P1):
            P["Kp"] = np.full(N, 1e30, np.float32)
    pb = _batch(gpu_lib, [P0, P1]).solve(max_updates=cap)
    for b, P in enumerate((P0, P1)):
        h, Y, U = orc.solve(P, max_updates=cap)
        _check(pb, b, h, Y, U, f"problem {b} feasible={feasible}")


@pytest.mark.parametrize("split", [0, 1])
def test_nan_in_qd_takes_the_select_form(gpu_lib, orc, knobs, split):
    """One NaN off the diagonal of row 5: the reference's selects keep it
    (row 5's sums turn NaN), a v_max_f32 form would drop it.  Fixed mode, one
    and two updates: NaN where the oracle has NaN, every other value bit for
    bit; problem 1 (no NaN) unaffected.  (The stored-split form keeps the
    reference's literal entries, NaN included.)"""
    knobs("mid_split", split)
    N, M = 48, 12
    P0 = orc.synth_problem(34, 0, N, M)
    P1 = orc.synth_problem(34, 1, N, M)
    Qd = P0["Qd"].reshape(N, N).copy()
    Qd[5, 9] = np.nan
    P0["Qd"] = Qd.reshape(-1)
    for n in (2, 3):
        pb = _batch(gpu_lib, [P0, P1]).solve(gpu_lib.MODE_FIXED, num_iter=n)
        for b, P in enumerate((P0, P1)):
            _, Y, _ = orc.solve(P, mode=1, num_iter=n)
            got = pb.Y[b].cpu().numpy()
            assert np.array_equal(np.isnan(got), np.isnan(Y)), (n, b)
            assert np.isnan(Y).any() == (b == 0)
            ok = ~np.isnan(Y)
            assert_bitwise(got[ok], Y[ok], f"num_iter={n} problem {b}")
