"""Residency of the persistent single-problem launches: k_split_persist (fixed
mode) and k_converge_persist (converge mode) run only when occupancy x CUs
covers their grid; otherwise -- forced here with pqp_tune_persist_fit_cus(1)
-- the solve takes the graph-replayed relay / chain, with the same bits
(both paths follow PQP_CPU.c:603-618 and :673-687 exactly)."""
from __future__ import annotations

import ctypes as C

import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu

FIXED_PERSIST, FIXED_RELAY, CONV_PERSIST, CONV_WIDE = 1, 2, 3, 4


def _path(L):
    fb = C.c_longlong(0)
    return int(L.pqp_tune_last_path(C.byref(fb))), int(fb.value)


@pytest.fixture
def one_cu(gpu_lib):
    L = gpu_lib.lib()
    prev = L.pqp_tune_persist_fit_cus(0)
    L.pqp_tune_persist_fit_cus(prev)
    yield L
    L.pqp_tune_persist_fit_cus(prev)


def test_fixed_persist_does_not_fit_falls_back(gpu_lib, orc, one_cu):
    L = one_cu
    N, M = 1024, 512
    P = orc.synth_problem(2, 3, N, M)
    want = orc.iterate(P["Qd"], P["Fd"], N, 9)
    with gpu_lib.Problem(P) as prob:
        r = prob.solve(gpu_lib.MODE_FIXED, num_iter=10)
        assert _path(L)[0] == FIXED_PERSIST
        assert_bitwise(r["Y"], want, "persistent")
        L.pqp_tune_persist_fit_cus(1)  # 64 workgroups cannot be resident on one CU
        r = prob.solve(gpu_lib.MODE_FIXED, num_iter=10)
        assert _path(L)[0] == FIXED_RELAY
        assert_bitwise(r["Y"], want, "relay fallback")


def test_converge_persist_does_not_fit_falls_back(gpu_lib, orc, one_cu):
    L = one_cu
    N, M = 512, 256
    P = orc.synth_problem(4, 1, N, M)
    with gpu_lib.Problem(P) as prob:
        a = prob.solve(max_updates=12)
        assert _path(L)[0] == CONV_PERSIST
        L.pqp_tune_persist_fit_cus(1)
        b = prob.solve(max_updates=12)
        assert _path(L)[0] == CONV_WIDE
    assert a["h"] == b["h"] == 13
    assert_bitwise(b["Y"], a["Y"], "graph chain vs persistent")
    assert_bitwise(b["Y"], orc.iterate(P["Qd"], P["Fd"], N, 12), "vs oracle")


@pytest.fixture
def stall(gpu_lib):
    L = gpu_lib.lib()
    prev = L.pqp_tune_persist_stall(-1)
    yield L
    L.pqp_tune_persist_stall(prev)


@pytest.mark.parametrize("wg", [0, 5])
def test_fixed_persist_stall_restarts_on_relay(gpu_lib, orc, stall, wg):
    """a persistent fixed-mode launch that passed the residency
    check but whose waits still expire (one workgroup never runs, the others
    time out after 2 s with their error word set): the solve restarts on the
    relay from Y = 1000 with the oracle's bits, the fallback is counted, and
    the next solve with the hook cleared takes the persistent launch again
    (rings and error words reset per launch)."""
    L = stall
    N, M = 1024, 512
    P = orc.synth_problem(2, 4, N, M)
    want = orc.iterate(P["Qd"], P["Fd"], N, 29)
    with gpu_lib.Problem(P) as prob:
        _, fb0 = _path(L)
        L.pqp_tune_persist_stall(wg)
        r = prob.solve(gpu_lib.MODE_FIXED, num_iter=30)
        path, fb1 = _path(L)
        assert path == FIXED_RELAY and fb1 == fb0 + 1
        assert_bitwise(r["Y"], want, "after the stalled persistent launch")
        L.pqp_tune_persist_stall(-1)
        r = prob.solve(gpu_lib.MODE_FIXED, num_iter=30)
        assert _path(L) == (FIXED_PERSIST, fb1)
        assert_bitwise(r["Y"], want, "persistent again")


@pytest.mark.parametrize("wg", [0, -2])
def test_converge_persist_stall_restarts_on_chain(gpu_lib, orc, stall, wg):
    """The same for the persistent converge launch: workgroup 0 (an update
    workgroup) or the last one (the deciding workgroup, wg -2 here) never
    runs; the solve restarts on the graph chain with the oracle's h, Y, U,
    and the hook cleared, the persistent launch runs again on the same
    handle."""
    L = stall
    N, M = 512, 256
    P = orc.synth_problem(4, 2, N, M)
    h, Y, U = orc.solve(P, max_updates=14)
    with gpu_lib.Problem(P) as prob:
        prob.solve(max_updates=2)
        assert _path(L)[0] == CONV_PERSIST
        _, fb0 = _path(L)
        if wg == -2:  # the deciding workgroup is the launch's last
            G = L.pqp_tune_converge_grid(N, M)
            assert G > 0
            wg = G - 1
        L.pqp_tune_persist_stall(wg)
        r = prob.solve(max_updates=14)
        path, fb1 = _path(L)
        assert path == CONV_WIDE and fb1 == fb0 + 1
        assert r["h"] == abs(h)
        assert_bitwise(r["Y"], Y, "Y after the stall")
        assert_bitwise(r["U"], U, "U after the stall")
        L.pqp_tune_persist_stall(-1)
        r = prob.solve(max_updates=14)
        assert _path(L) == (CONV_PERSIST, fb1)
        assert r["h"] == abs(h)
        assert_bitwise(r["Y"], Y, "Y persistent again")
        assert_bitwise(r["U"], U, "U persistent again")
