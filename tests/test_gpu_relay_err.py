"""The relay kernels' bounded hand-off waits report, not corrupt: a wait that
expires inside k_split_relay / k_lean_relay / k_gemv_relay sets a sticky
device error word that the host turns into PQP_ERR_HIP (fixed-mode relay
solves, the converge-mode graph chain, pqp_rowblock_check).  The expiry is
forced with pqp_tune_relay_spin_max(-1), then the default budget is restored
and the same handle solves bit-exactly again (the error word was cleared and
the graphs recaptured)."""
from __future__ import annotations

import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu

PQP_ERR_HIP = -2


@pytest.fixture
def forced_expiry(gpu_lib):
    L = gpu_lib.lib()
    prev = L.pqp_tune_relay_spin_max(-1)
    yield L
    L.pqp_tune_relay_spin_max(prev)


def test_fixed_relay_reports_expired_wait(gpu_lib, orc, forced_expiry):
    L = forced_expiry
    N, M = 300, 150
    P = orc.synth_problem(3, 1, N, M)
    prev_persist = L.pqp_tune_persist(1)  # fixed mode through the graph-replayed relay
    try:
        with gpu_lib.Problem(P) as prob:
            with pytest.raises(gpu_lib.PQPError) as ei:
                prob.solve(gpu_lib.MODE_FIXED, num_iter=20)
            assert ei.value.code == PQP_ERR_HIP and "relay" in str(ei.value)
            L.pqp_tune_relay_spin_max(0)
            r = prob.solve(gpu_lib.MODE_FIXED, num_iter=20)
            assert_bitwise(r["Y"], orc.iterate(P["Qd"], P["Fd"], N, 19), "after the error")
    finally:
        L.pqp_tune_persist(prev_persist)


def test_converge_chain_reports_expired_wait(gpu_lib, orc, forced_expiry):
    L = forced_expiry
    N, M = 400, 200
    P = orc.synth_problem(5, 2, N, M)
    prev = L.pqp_tune_converge_persist(1)  # converge mode through the graph chain (pqp_wide.hip)
    try:
        with gpu_lib.Problem(P) as prob:
            with pytest.raises(gpu_lib.PQPError) as ei:
                prob.solve(max_updates=6)
            assert ei.value.code == PQP_ERR_HIP
            L.pqp_tune_relay_spin_max(0)
            r = prob.solve(max_updates=6)  # capped (no error): the word was cleared
            assert r["h"] == 7 and not r["converged"]
    finally:
        L.pqp_tune_converge_persist(prev)


def test_rowblock_check_reports_expired_wait(gpu_lib, orc, forced_expiry):
    import torch

    L = forced_expiry
    N = 260
    P = orc.synth_problem(7, 0, N, N // 2, with_qp=False)
    Qd = torch.from_numpy(P["Qd"]).cuda()
    Fd = torch.from_numpy(P["Fd"]).cuda()
    blk = gpu_lib.RowBlock(Qd, Fd, N, 0, N)
    Y = torch.full((N,), 1000.0, device="cuda")
    Yn = torch.empty(N, device="cuda")
    blk.update(Y, Yn)
    with pytest.raises(gpu_lib.PQPError) as ei:
        blk.check()
    assert ei.value.code == PQP_ERR_HIP
    L.pqp_tune_relay_spin_max(0)
    blk.update(Y, Yn)
    blk.check()  # cleared by the failed check; a good update leaves it clear
    assert_bitwise(Yn.cpu().numpy(), orc.iterate(P["Qd"], P["Fd"], N, 1), "row block after the error")
