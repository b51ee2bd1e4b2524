"""k_solve_pipe: batched converge mode of problems too large
for LDS with Gp read once per iteration.  The update to Y_{h+1} runs first
(speculatively: updateY2 needs only Y_h, PQP_CPU.c:603-618), then one pass
over Gp in 64 x 64 LDS tiles gives checkFeas(h)'s rows Gp U_h (:636, j in
order) and the next iterate's Gp'Y_{h+1} (:355, i in order).  Bar: the
reference's h, Y, U (and, through h, Jp / Jd) bit for bit against the oracle,
and the same bits as k_solve_single (pipe_off), on infeasible and all-feasible
iterates, tile-ragged N and M, M > N, chunked launches and a problem that
stops inside a launch.  Shapes with M < N / 3, which the library sends to
k_solve_single by default, run here with pqp_tune("pipe_force", 1)."""
from __future__ import annotations

import numpy as np
import pytest

import pqp_amd
from conftest import CAP, assert_bitwise

pytestmark = pytest.mark.gpu


def _check(pb, b, h, Y, U, what):
    assert int(pb.h[b]) == abs(h), (what, int(pb.h[b]), h)
    assert int(pb.status[b]) == (1 if h > 0 else 2), (what, int(pb.status[b]))
    assert_bitwise(pb.Y[b].cpu().numpy(), Y, f"{what} Y")
    assert_bitwise(pb.U[b].cpu().numpy(), U, f"{what} U")


def _solve(gpu_lib, N, M, B, cap, feasible, pipe_off=0, chunk=0, seed=9, inst0=4, variant=0):
    prev = pqp_amd.tune("pipe_off", pipe_off)
    prev_chunk = pqp_amd.tune("batch_chunk", chunk)
    prev_variant = pqp_amd.tune("pipe_variant", variant)
    prev_force = pqp_amd.tune("pipe_force", 1)  # also the M < N / 3 shapes
    try:
        pb = gpu_lib.ProblemBatch.synthetic(seed, inst0, B, N, M)
        if feasible:
            pb.Kp.fill_(1e30)
        pb.solve(max_updates=cap)
        kernel = pqp_amd.tune_get("last_batch_kernel")
    finally:
        pqp_amd.tune("pipe_off", prev)
        pqp_amd.tune("batch_chunk", prev_chunk)
        pqp_amd.tune("pipe_variant", prev_variant)
        pqp_amd.tune("pipe_force", prev_force)
    return pb, kernel


@pytest.mark.parametrize("variant", [0, 3], ids=["tiles128x96", "tiles64"])
@pytest.mark.parametrize("N,M", [(256, 128), (260, 132), (128, 200), (320, 64), (512, 256)])
@pytest.mark.parametrize("feasible", [False, True])
def test_pipe_capped_vs_oracle(gpu_lib, orc, N, M, feasible, variant):
    """Capped solves through k_solve_pipe: 64-aligned and ragged tiles (N 260,
    M 132: partial row and column tiles), M > N, one column tile (M 64);
    `feasible`: Kp = 1e30 seen by checkFeas only, so every iterate runs all of
    computeCost and the fused Y'Qd rides in the speculative update."""
    B, cap = 3, 6
    pb, kernel = _solve(gpu_lib, N, M, B, cap, feasible, variant=variant)
    assert kernel == 1, "k_solve_pipe not taken"
    for b in range(B):
        P = orc.synth_problem(9, 4 + b, N, M)
        if feasible:
            P["Kp"] = np.full(N, 1e30, np.float32)
        h, Y, U = orc.solve(P, max_updates=cap)
        _check(pb, b, h, Y, U, f"pipe N={N} M={M} feasible={feasible} b={b}")


@pytest.mark.parametrize("variant", [0, 3], ids=["tiles128x96", "tiles64"])
@pytest.mark.parametrize("chunk", [1, 2, 5])
@pytest.mark.parametrize("feasible", [False, True])
def test_pipe_chunked_launches_vs_oracle(gpu_lib, orc, chunk, feasible, variant):
    """A solve split over launches of `chunk` iterates: each launch re-forms
    tM_h from the Y it resumes from, and the last iterate of a launch skips the
    speculative update (it breaks before its update whatever terminate() says)."""
    N, M, B, cap = 256, 128, 2, 7
    pb, kernel = _solve(gpu_lib, N, M, B, cap, feasible, chunk=chunk, variant=variant)
    assert kernel == 1
    for b in range(B):
        P = orc.synth_problem(9, 4 + b, N, M)
        if feasible:
            P["Kp"] = np.full(N, 1e30, np.float32)
        h, Y, U = orc.solve(P, max_updates=cap)
        _check(pb, b, h, Y, U, f"pipe chunk={chunk} feasible={feasible} b={b}")


@pytest.mark.parametrize("feasible", [False, True])
def test_pipe_same_bits_as_single_at_bench_size(gpu_lib, feasible):
    """n_dual 1024, M 512 (the batch_converge bench leg's shape): k_solve_pipe
    and k_solve_single (pipe_off) give the same h, Y, U for every problem."""
    N, M, B, cap = 1024, 512, 8, 5
    a, ka = _solve(gpu_lib, N, M, B, cap, feasible)
    b, kb = _solve(gpu_lib, N, M, B, cap, feasible, pipe_off=1)
    c, kc = _solve(gpu_lib, N, M, B, cap, feasible, variant=3)
    assert (ka, kb, kc) == (1, 0, 1)
    assert_bitwise(c.Y.cpu().numpy(), b.Y.cpu().numpy(), "Y pipe 64x64 tiles vs single")
    assert_bitwise(c.U.cpu().numpy(), b.U.cpu().numpy(), "U pipe 64x64 tiles vs single")
    assert np.array_equal(a.h.cpu().numpy(), b.h.cpu().numpy())
    assert np.array_equal(a.status.cpu().numpy(), b.status.cpu().numpy())
    assert_bitwise(a.Y.cpu().numpy(), b.Y.cpu().numpy(), "Y pipe vs single")
    assert_bitwise(a.U.cpu().numpy(), b.U.cpu().numpy(), "U pipe vs single")


def test_pipe_whole_bench_batch_same_bits_as_single(gpu_lib):
    """VERDICT r3 (weak 1): the batch_converge leg's whole workload -- 4096
    problems of n_dual 1024, M 512 from the bench's seed (1, problems 0..4095)
    -- capped at 2 updates through k_solve_pipe and through k_solve_single
    (pipe_off): h, status, Y and U the same for every problem.  (Problems 0
    and 1 of this batch against the oracle: the two tests below.)"""
    import torch

    N, M, B, cap = 1024, 512, 4096, 2
    a, ka = _solve(gpu_lib, N, M, B, cap, False, seed=1, inst0=0)
    got = [a.h.cpu().numpy(), a.status.cpu().numpy(), a.Y.cpu().numpy(), a.U.cpu().numpy()]
    del a
    torch.cuda.empty_cache()
    b, kb = _solve(gpu_lib, N, M, B, cap, False, seed=1, inst0=0, pipe_off=1)
    assert (ka, kb) == (1, 0)
    assert (got[1] == 2).all(), "the generator's problems are capped, every iterate infeasible"
    assert np.array_equal(got[0], b.h.cpu().numpy())
    assert np.array_equal(got[1], b.status.cpu().numpy())
    assert_bitwise(got[2], b.Y.cpu().numpy(), "Y pipe vs single, 4096 problems")
    assert_bitwise(got[3], b.U.cpu().numpy(), "U pipe vs single, 4096 problems")


def test_pipe_bench_size_vs_oracle(gpu_lib, orc):
    """One n_dual 1024 problem of the bench's batch against the oracle, with
    every iterate feasible (the fused Y'Qd, Qp pass and costs each iterate)."""
    N, M, cap = 1024, 512, 3
    pb, kernel = _solve(gpu_lib, N, M, 1, cap, True, seed=3, inst0=0)
    assert kernel == 1
    P = orc.synth_problem(3, 0, N, M)
    P["Kp"] = np.full(N, 1e30, np.float32)
    h, Y, U = orc.solve(P, max_updates=cap)
    _check(pb, 0, h, Y, U, "pipe n_dual 1024 feasible")


def test_pipe_bench_size_infeasible_vs_oracle(gpu_lib, orc):
    """the batch_converge leg's timed case -- n_dual 1024, M 512,
    the generator's problems, whose every iterate fails checkFeas (terminate()
    returns at PQP_CPU.c:677 with no computeCost) -- through k_solve_pipe,
    two problems of the bench's own batch (seed 1, problems 0 and 1) against
    the oracle, capped at 3 updates."""
    N, M, cap = 1024, 512, 3
    pb, kernel = _solve(gpu_lib, N, M, 2, cap, False, seed=1, inst0=0)
    assert kernel == 1
    for b in range(2):
        P = orc.synth_problem(1, b, N, M)
        assert not orc.feasible(orc.u_from_y(np.full(N, 1000.0, np.float32), P["Fp"], P["Gp"], P["Qp_inv"], N, M),
                                P["Gp"], P["Kp"], N, M), "want the infeasible case"
        h, Y, U = orc.solve(P, max_updates=cap)
        assert h == -(cap + 1) or h == cap + 1, h
        _check(pb, b, h, Y, U, f"pipe n_dual 1024 infeasible b={b}")


@pytest.mark.parametrize("chunk", [0, 1, 2])
def test_pipe_testfile_stops_like_reference(gpu_lib, orc, tmp_path, chunk):
    """testing/ test2 (n_dual 400, M 100) converges at the reference's h = 3:
    the stop falls inside a launch (chunk 0, 2) or on a launch boundary (1);
    the speculative Y_{h+1} is dropped."""
    from test_gpu_wide import _testing_file

    P = gpu_lib.testfile_problem(_testing_file("test2.txt", tmp_path))
    h, Y, U = orc.solve(P, max_updates=CAP)
    assert h > 0
    prev = pqp_amd.tune("batch_chunk", chunk)
    prev_force = pqp_amd.tune("pipe_force", 1)  # M = N / 4
    try:
        pb = gpu_lib.ProblemBatch.replicate(P, 3)
        pb.solve(max_updates=CAP)
        kernel = pqp_amd.tune_get("last_batch_kernel")
    finally:
        pqp_amd.tune("batch_chunk", prev)
        pqp_amd.tune("pipe_force", prev_force)
    assert kernel == 1
    for b in range(3):
        _check(pb, b, h, Y, U, f"test2 copy {b} chunk={chunk}")


def test_pipe_mixed_symmetric_and_not(gpu_lib, orc):
    """A bit-symmetric Qd beside a non-symmetric one (dense Qp_inv): the fused
    Y'Qd for the first only, the separate pass over Qd for the second."""
    from pqp_amd import dense_qinv

    N, M, cap = 256, 64, 5
    P0 = orc.synth_problem(13, 0, N, M)
    P1 = orc.synth_primal(13, 1, N, M)
    P1["Qp_inv"] = dense_qinv(13, M)
    P1["Qd"], P1["Fd"], P1["Md"] = orc.convert_to_dual(P1["Qp_inv"], P1["Gp"], P1["Kp"], P1["Fp"], P1["Mp"], N, M)
    P1["Qp"] = orc.gauss_jordan(P1["Qp_inv"], M)
    Q1 = P1["Qd"].reshape(N, N)
    assert not np.array_equal(Q1.view(np.uint32), Q1.T.view(np.uint32)), "want a non-symmetric Qd here"
    for P in (P0, P1):
        P["Kp"] = np.full(N, 1e30, np.float32)
    pb = gpu_lib.ProblemBatch(2, N, M)
    for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp"):
        pb.set(k, np.stack([np.asarray(P[k], np.float32).reshape(-1) for P in (P0, P1)]))
    prev_force = pqp_amd.tune("pipe_force", 1)  # M = N / 4
    try:
        pb.solve(max_updates=cap)
        assert pqp_amd.tune_get("last_batch_kernel") == 1
    finally:
        pqp_amd.tune("pipe_force", prev_force)
    for b, P in enumerate((P0, P1)):
        h, Y, U = orc.solve(P, max_updates=cap)
        _check(pb, b, h, Y, U, f"mixed {b}")


def test_pipe_routing_by_shape(gpu_lib):
    """Auto routing of path 2: k_solve_pipe where M >= N / 3 (the second
    pass over Gp it saves is a large part of the bytes), k_solve_single below
    (profiles/r03/pipe/horizon_pipe_vs_single.jsonl), whatever the caller
    leaves in pipe_force."""
    prev = pqp_amd.tune("pipe_force", 0)
    try:
        for N, M, want in ((256, 128, 1), (300, 100, 1), (256, 64, 0), (400, 100, 0)):
            pb = gpu_lib.ProblemBatch.synthetic(9, 0, 2, N, M)
            pb.solve(max_updates=2)
            assert pqp_amd.tune_get("last_batch_kernel") == want, (N, M)
    finally:
        pqp_amd.tune("pipe_force", prev)
