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
