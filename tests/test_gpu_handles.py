"""Handles bound to their device and stream (Threading;
VERDICT r2 item 4): each pqp_problem records the device it was made on and
owns a stream (or takes the caller's), calls on it run there whatever device
the caller has current, and different handles solve concurrently from
different host threads (the reference's solver keeps no globals,
PQP_CPU.c:694).  Bar: every concurrent solve bit-identical to the oracle."""
from __future__ import annotations

import threading

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _cases(orc):
    """Three problems on three solver paths: converge mode on the persistent
    pipelined launch (n_dual 256), converge mode on the one-wave solver
    (n_dual 28, bundled-sized), fixed mode on the persistent launch (n_dual 512)."""
    return [
        (orc.synth_problem(21, 0, 256, 128), dict(max_updates=12)),
        (orc.synth_problem(21, 1, 24, 12), dict(max_updates=200000)),
        (orc.synth_problem(21, 2, 512, 256), dict(mode=1, num_iter=60)),
    ]


def _expect(orc, P, kw):
    if kw.get("mode") == 1:
        return None, orc.iterate(P["Qd"], P["Fd"], P["N"], kw["num_iter"] - 1), None
    return orc.solve(P, max_updates=kw["max_updates"])


def test_concurrent_handles_from_threads(gpu_lib, orc):
    cases = _cases(orc)
    want = [_expect(orc, P, kw) for P, kw in cases]
    probs = [gpu_lib.Problem(P) for P, _ in cases]
    errors, results = [], [[] for _ in cases]

    def work(i):
        try:
            for _ in range(6):
                results[i].append(probs[i].solve(**cases[i][1]))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(f"thread {i}: {e}")

    threads = [threading.Thread(target=work, args=(i,)) for i in range(len(cases))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in threads), "a solve thread did not finish"
    assert not errors, errors
    for i, ((P, kw), (h, Y, U)) in enumerate(zip(cases, want)):
        assert len(results[i]) == 6
        for r in results[i]:
            assert_bitwise(r["Y"], Y, f"case {i} Y")
            if h is not None:
                assert r["h"] == abs(h)
                assert_bitwise(r["U"], U, f"case {i} U")
    for p in probs:
        p.close()


def test_two_threads_one_handle_serialize(gpu_lib, orc):
    """Calls on ONE handle from two threads are serialized by its lock: both
    get the oracle's result."""
    P = orc.synth_problem(22, 0, 300, 150)
    h, Y, U = orc.solve(P, max_updates=9)
    out = []
    with gpu_lib.Problem(P) as prob:
        ts = [threading.Thread(target=lambda: out.extend(prob.solve(max_updates=9) for _ in range(4)))
              for _ in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
    assert len(out) == 8
    for r in out:
        assert r["h"] == abs(h)
        assert_bitwise(r["Y"], Y, "Y")
        assert_bitwise(r["U"], U, "U")


def test_handle_on_caller_stream(gpu_lib, orc):
    """pqp_problem_create_on(device 0, the caller's torch stream)."""
    import torch

    s = torch.cuda.Stream(device=0)
    P = orc.synth_problem(23, 0, 64, 32)
    h, Y, U = orc.solve(P, max_updates=15)
    with gpu_lib.Problem(P, device=0, stream=s) as prob:
        assert prob.device == 0
        r = prob.solve(max_updates=15)
    assert r["h"] == abs(h)
    assert_bitwise(r["Y"], Y, "Y")
    assert_bitwise(r["U"], U, "U")


def test_bad_device_is_an_error(gpu_lib, orc):
    import torch

    P = orc.synth_problem(23, 1, 16, 8)
    with pytest.raises(gpu_lib.PQPError) as e:
        gpu_lib.Problem(P, device=torch.cuda.device_count())
    assert e.value.code == gpu_lib.PQP_ERR_ARG


def test_wrong_current_device_still_solves(gpu_lib, orc):
    """A handle made on device 0, solved while device 1 is current: it runs on
    device 0 and leaves device 1 current.  (Needs two GPUs.)"""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU on this box")
    P = orc.synth_problem(24, 0, 256, 128)
    h, Y, U = orc.solve(P, max_updates=10)
    torch.cuda.set_device(0)
    prob = gpu_lib.Problem(P)
    torch.cuda.set_device(1)
    try:
        r = prob.solve(max_updates=10)
        assert torch.cuda.current_device() == 1 and prob.device == 0
    finally:
        prob.close()
        torch.cuda.set_device(0)
    assert r["h"] == abs(h)
    assert_bitwise(r["Y"], Y, "Y")
    assert_bitwise(r["U"], U, "U")
