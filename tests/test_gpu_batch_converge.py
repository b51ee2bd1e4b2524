"""Batched converge mode at larger sizes: pqp_batch_solve,
one workgroup per problem from global memory (k_solve_single).  Problems whose
Qd is bit-symmetric (diagonal Qp_inv: the synthetic and testing/ problems)
skip the column-major copy; after a feasible terminate() the next Y'Qd
(PQP_CPU.c:648-653) rides in the same pass over Qd as the speculative update
to Y_{h+1} (:603-618) (opts bit 0 turns that off), and Gp / Qp_inv are read
through transposes (prepared once per ProblemBatch; opts bit 1: made per
call by the unprepared pqp_batch_solve).  Bar: the reference's h, Y and U bit
for bit (oracle) in every setting, and a batch mixing both kinds of Qd.  N and
M multiples of 4 take the 8/16-byte load forms of k_solve_single; opts bit 2
(and ragged N, M) the 4-byte form."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import CAP, assert_bitwise

pytestmark = pytest.mark.gpu


def _check(pb, b, h, Y, U, what):
    assert int(pb.h[b]) == abs(h), (what, int(pb.h[b]), h)
    assert int(pb.status[b]) == (1 if h > 0 else 2), (what, int(pb.status[b]))
    assert_bitwise(pb.Y[b].cpu().numpy(), Y, f"{what} Y")
    assert_bitwise(pb.U[b].cpu().numpy(), U, f"{what} U")


@pytest.mark.parametrize("opts,tr,prep", [(0, True, True), (0, False, True), (1, True, True), (4, True, True),
                                           (0, False, False), (2, False, False), (3, False, False), (6, False, False)])
def test_batch_testfile_converges_like_reference(gpu_lib, orc, tmp_path, opts, tr, prep):
    from test_gpu_wide import _testing_file

    L = gpu_lib.lib()
    P = gpu_lib.testfile_problem(_testing_file("test2.txt", tmp_path))
    h, Y, U = orc.solve(P, max_updates=CAP)
    prev = L.pqp_tune_batch_converge(opts)
    try:
        pb = gpu_lib.ProblemBatch.replicate(P, 3)
        pb.transposes = tr
        pb.solve(max_updates=CAP, prepared=prep)
        if prep:
            pb.solve(max_updates=CAP)  # again on the kept prepared data
    finally:
        L.pqp_tune_batch_converge(prev)
    for b in range(3):
        _check(pb, b, h, Y, U, f"test2 copy {b} opts={opts} transposes={tr} prepared={prep}")


@pytest.mark.parametrize("opts,tr,N,M", [(0, True, 256, 128), (0, False, 256, 128), (1, True, 256, 128),
                                         (4, True, 256, 128), (16, True, 256, 128), (0, True, 512, 64),
                                         (16, True, 512, 64), (0, True, 201, 61), (0, True, 204, 62)])
@pytest.mark.parametrize("feasible", [False, True])
def test_batch_synthetic_capped_vs_oracle(gpu_lib, orc, opts, tr, N, M, feasible):
    """Capped solves; `feasible`: Kp = 1e30 seen by checkFeas only, so every
    iterate runs all of computeCost (and the fused Y'Qd pass where enabled)."""
    L = gpu_lib.lib()
    B, cap = 3, 6
    prev = L.pqp_tune_batch_converge(opts)
    try:
        pb = gpu_lib.ProblemBatch.synthetic(9, 4, B, N, M, transposes=tr)
        if feasible:
            pb.Kp.fill_(1e30)
        pb.solve(max_updates=cap)
    finally:
        L.pqp_tune_batch_converge(prev)
    for b in range(B):
        P = orc.synth_problem(9, 4 + b, N, M)
        if feasible:
            P["Kp"] = np.full(N, 1e30, np.float32)
        h, Y, U = orc.solve(P, max_updates=cap)
        _check(pb, b, h, Y, U, f"synthetic {b} opts={opts} transposes={tr} feasible={feasible}")


@pytest.mark.parametrize("opts,prep", [(0, True), (1, True), (0, False)])
def test_batch_mixed_symmetric_and_not(gpu_lib, orc, opts, prep):
    """Problem 0's Qd is bit-symmetric (diagonal Qp_inv), problem 1's is not
    (dense Qp_inv): one launch, the packed column-major copy, and (opts 1) a
    per-problem choice of the fused pass."""
    from pqp_amd import dense_qinv

    N, M, cap = 200, 60, 5
    P0 = orc.synth_problem(5, 0, N, M)
    P1 = orc.synth_primal(5, 1, N, M)
    P1["Qp_inv"] = dense_qinv(5, M)
    P1["Qd"], P1["Fd"], P1["Md"] = orc.convert_to_dual(P1["Qp_inv"], P1["Gp"], P1["Kp"], P1["Fp"], P1["Mp"], N, M)
    P1["Qp"] = orc.gauss_jordan(P1["Qp_inv"], M)
    Q1 = P1["Qd"].reshape(N, N)
    assert not np.array_equal(Q1.view(np.uint32), Q1.T.view(np.uint32)), "want a non-symmetric Qd here"
    pb = gpu_lib.ProblemBatch(2, N, M)
    for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp"):
        pb.set(k, np.stack([np.asarray(P0[k], np.float32).reshape(-1), np.asarray(P1[k], np.float32).reshape(-1)]))
    L = gpu_lib.lib()
    prev = L.pqp_tune_batch_converge(opts)
    try:
        pb.solve(max_updates=cap, prepared=prep)
    finally:
        L.pqp_tune_batch_converge(prev)
    if prep:
        assert pb._prep["QdT"] is not None and not pb._prep["all_sym"]
    for b, P in enumerate((P0, P1)):
        h, Y, U = orc.solve(P, max_updates=cap)
        _check(pb, b, h, Y, U, f"mixed {b}")


@pytest.mark.parametrize("opts", [0, 1])
def test_batch_fits_only_unfused(gpu_lib, orc, opts):
    """n_dual 9600, M 4 fits the one-workgroup solver's LDS only
    without the fused Y'Qd vector (3 ldq + 3 ldm floats <= 150 KiB < 4 ldq +
    3 ldm).  It must solve in both settings (fusion turned off for the call
    where it does not fit), bit for bit with the oracle."""
    N, M, cap = 9600, 4, 2
    L = gpu_lib.lib()
    prev = L.pqp_tune_batch_converge(opts)
    try:
        pb = gpu_lib.ProblemBatch.synthetic(11, 0, 1, N, M).solve(max_updates=cap)
    finally:
        L.pqp_tune_batch_converge(prev)
    P = orc.synth_problem(11, 0, N, M)
    h, Y, U = orc.solve(P, max_updates=cap)
    _check(pb, 0, h, Y, U, f"n_dual {N} opts={opts}")


def test_prepared_data_follow_new_qd(gpu_lib, orc):
    """A solve, new problems written through set() (the prepared Theta and
    flags are dropped and rebuilt), a solve: the second problem set's bits."""
    N, M, cap = 256, 128, 5
    pb = gpu_lib.ProblemBatch.synthetic(12, 0, 2, N, M)
    pb.solve(max_updates=cap)
    first = pb._prep
    other = [orc.synth_problem(12, 5 + b, N, M) for b in range(2)]
    for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp"):
        pb.set(k, np.stack([np.asarray(P[k], np.float32).reshape(-1) for P in other]))
    assert pb._prep is None
    pb.solve(max_updates=cap)
    assert pb._prep is not first
    for b, P in enumerate(other):
        h, Y, U = orc.solve(P, max_updates=cap)
        _check(pb, b, h, Y, U, f"reloaded {b}")


@pytest.mark.parametrize("how", ["index", "copy_"])
def test_prepared_data_follow_in_place_writes(gpu_lib, orc, how):
    """Qd, Gp and Qp_inv written IN PLACE (no set(), no
    invalidate()) after a prepared solve: solve() sees torch's version counter
    move and prepares again, so the second solve has the new problems' bits
    (a stale symmetry flag or Qp_inv' would give silently wrong ones)."""
    from pqp_amd import dense_qinv

    N, M, cap = 256, 128, 5
    pb = gpu_lib.ProblemBatch.synthetic(14, 0, 2, N, M)
    pb.solve(max_updates=cap)
    # problem 1 becomes a dense-Qp_inv problem: its Qd is not bit-symmetric
    P = orc.synth_primal(14, 9, N, M)
    P["Qp_inv"] = dense_qinv(14, M)
    P["Qd"], P["Fd"], P["Md"] = orc.convert_to_dual(P["Qp_inv"], P["Gp"], P["Kp"], P["Fp"], P["Mp"], N, M)
    P["Qp"] = orc.gauss_jordan(P["Qp_inv"], M)
    T = lambda a: pb.torch.as_tensor(np.asarray(a, np.float32).reshape(-1), device=pb.device)  # noqa: E731
    for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp"):
        t = getattr(pb, k)
        if how == "index":
            t[1] = T(P[k]) if t.dim() == 2 else T(P[k])[0]
        else:
            t[1:2].copy_(T(P[k]).reshape(t[1:2].shape))
    pb.solve(max_updates=cap)
    assert pb._prep["QdT"] is not None and not pb._prep["all_sym"]
    h, Y, U = orc.solve(P, max_updates=cap)
    _check(pb, 1, h, Y, U, f"in-place ({how}) problem 1")
    P0 = orc.synth_problem(14, 0, N, M)
    h, Y, U = orc.solve(P0, max_updates=cap)
    _check(pb, 0, h, Y, U, "untouched problem 0")


def test_prepare_needs_qdt_status_and_gpt_only_for_single(gpu_lib):
    """pqp_batch_prepare asks for the column-major copy with its own
    status (PQP_ERR_NEEDS_QDT), the retried pqp_batch_solve leaves no error
    text behind, and Gp' (B*N*M floats) is allocated only where path 2 runs
    k_solve_single (pqp_batch_solve_kernel 0), never for k_solve_pipe."""
    import ctypes as C

    import pqp_amd
    from pqp_amd import dense_qinv

    L = gpu_lib.lib()
    N, M = 256, 128
    assert L.pqp_batch_solve_kernel(N, M) == 1 and L.pqp_batch_solve_kernel(256, 64) == 0
    pb = gpu_lib.ProblemBatch.synthetic(15, 0, 2, N, M)
    pb.Qp_inv[1] = pb.torch.as_tensor(dense_qinv(15, M), device=pb.device)
    pb.convert_to_dual()
    f = dict(dtype=pb.torch.float32, device=pb.device)
    theta, sym = pb.torch.empty(2, N, **f), pb.torch.empty(2, dtype=pb.torch.int32, device=pb.device)
    all_sym = C.c_int(7)
    rc = L.pqp_batch_prepare(2, N, M, pb._p(pb.Qd), pb._p(pb.Gp), pb._p(pb.Qp_inv), None, pb._p(theta), pb._p(sym),
                             None, None, C.byref(all_sym), pb._s())
    assert rc == pqp_amd.PQP_ERR_NEEDS_QDT and all_sym.value == 0
    assert sym.cpu().tolist()[0] != 0 and sym.cpu().tolist()[1] == 0
    rc = L.pqp_batch_solve(2, N, M, *[pb._p(getattr(pb, k)) for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp",
                                                                       "Gp", "Kp")],
                           0, 1000, 3, pb._p(pb.Y), pb._p(pb.U), pb._p(pb.h), pb._p(pb.status), pb._s())
    assert rc == pqp_amd.PQP_OK and pqp_amd.last_error() == ""
    pb.solve(max_updates=3)
    assert pb._prep["GpT"] is None and pb._prep["QinvT"] is not None  # the pipe: no Gp'
    prev = pqp_amd.tune("pipe_off", 1)
    try:
        assert L.pqp_batch_solve_kernel(N, M) == 0
        pb.solve(max_updates=3)  # the route moved: prepared again, now with Gp'
        assert pb._prep["GpT"] is not None
    finally:
        pqp_amd.tune("pipe_off", prev)


@pytest.mark.parametrize("occ", [3, 4, 5])
@pytest.mark.parametrize("feasible", [False, True])
def test_single_register_capped_builds_vs_oracle(gpu_lib, orc, occ, feasible):
    """k_solve_single's builds capped to 4 and 5 workgroups per CU
    (taken by the launch only for batches above ~3 x the CU count at n_dual <=
    768) forced on a small batch: n_dual 256, M 64 (M < N / 3, so path 2 runs
    k_solve_single, not the pipe), infeasible and all-feasible iterates, the
    oracle's h, Y and U bit for bit."""
    B, N, M, cap = 3, 256, 64, 6
    prev = gpu_lib.tune("single_occ", occ)
    try:
        pb = gpu_lib.ProblemBatch.synthetic(21, 0, B, N, M)
        if feasible:
            pb.Kp.fill_(1e30)
        pb.solve(max_updates=cap)
        assert gpu_lib.tune_get("last_batch_kernel") == 0
    finally:
        gpu_lib.tune("single_occ", prev)
    for b in range(B):
        P = orc.synth_problem(21, b, N, M)
        if feasible:
            P["Kp"] = np.full(N, 1e30, np.float32)
        h, Y, U = orc.solve(P, max_updates=cap)
        _check(pb, b, h, Y, U, f"single_occ={occ} feasible={feasible} problem {b}")
