"""One small problem in one launch (pqp_tiny.hip, configs[1]): k_fixed_one
(fixed mode; the sparse form where every split row has few nonzero entries,
else or on request the dense form) and k_solve_quintet (converge mode on five
waves), both writing their results to pinned host memory.  Bar: the
reference's bits (golden fixtures from PQP_CPU.c, and the oracle), identical
h, for every form; the sparse form's switch to the dense form at the first
non-finite y; the bounded waits' error path."""
from __future__ import annotations

from contextlib import contextmanager

import numpy as np
import pytest

from conftest import CAP, assert_bitwise

pytestmark = pytest.mark.gpu

KEYS = ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")
FORMS = {"sparse": {}, "dense": {"tiny_dense": 1}, "round4": {"tiny_old": 1}, "np2": {"tiny_np": 2},
         "np4": {"tiny_np": 4}, "apoll": {"tiny_apoll": 1}, "ablk1": {"tiny_ablk": 1}, "ablk1_np4": {"tiny_ablk": 1, "tiny_np": 4}}


@contextmanager
def tuned(gpu_lib, knobs):
    old = {k: gpu_lib.tune(k, v) for k, v in knobs.items()}
    try:
        yield
    finally:
        for k, v in old.items():
            gpu_lib.tune(k, v)


def bundled_problem(g):
    P = {k: np.ascontiguousarray(g[k], dtype=np.float32) for k in KEYS}
    P.update(N=int(g["N"]), M=int(g["M"]))
    return P


def _same_bits_or_both_nan(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(nan | (a.view(np.uint32) == b.view(np.uint32))))


@pytest.mark.parametrize("form", list(FORMS))
def test_bundled_both_modes_every_form(gpu_lib, golden_bundled, form):
    """configs[1] through one pqp_problem handle: converge (h = 313, Y*, U*,
    Jp, Jd), fixed 1000 and fixed k updates, repeated solves."""
    g = golden_bundled
    with tuned(gpu_lib, FORMS[form]), gpu_lib.Problem(bundled_problem(g)) as prob:
        for _ in range(2):
            r = prob.solve(max_updates=CAP)
            assert r["converged"] and r["h"] == int(g["h"]) == 313
            assert_bitwise(r["Y"], g["Ystar"], f"{form}: Y*")
            assert_bitwise(r["U"], g["Ustar"], f"{form}: U*")
            assert np.float32(r["Jp"]) == g["iter_Jp"][-1] and np.float32(r["Jd"]) == g["iter_Jd"][-1]
            f = prob.solve(gpu_lib.MODE_FIXED, num_iter=1000)
            assert f["h"] == 1000
            assert_bitwise(f["Y"], g["Y_fixed999"], f"{form}: fixed-999 Y")
        for k in (1, 2, 10, 100, 312):
            f = prob.solve(gpu_lib.MODE_FIXED, num_iter=k)
            assert_bitwise(f["Y"], g[f"Y_h{k}"], f"{form}: Y after {k - 1} updates")


@pytest.mark.parametrize("form", ["sparse", "dense", "np2", "np4", "apoll", "ablk1", "ablk1_np4"])
@pytest.mark.parametrize("cap", [1, 2, 3, 7, 8, 9, 16, 311])
def test_bundled_converge_capped(gpu_lib, golden_bundled, orc, form, cap):
    """A cap inside and at the ring's depth (8 iterates in flight): the solve
    ends on Y after `cap` updates, U from its terminate(), and the costs of
    the last feasible iterate, exactly as the one-wave solver."""
    g = golden_bundled
    P = bundled_problem(g)
    with tuned(gpu_lib, FORMS[form]):
        r = gpu_lib.solve_dual(P, max_updates=cap)
    assert not r["converged"] and r["h"] == cap + 1
    assert_bitwise(r["Y"], orc.iterate(P["Qd"], P["Fd"], P["N"], cap), "Y at the cap")
    flag, U, Jp, Jd = orc.terminate(r["Y"], *[P[k] for k in KEYS], P["N"], P["M"])
    assert flag == 0
    assert_bitwise(r["U"], U, "U of the last terminate()")
    with tuned(gpu_lib, {"tiny_old": 1}):
        o = gpu_lib.solve_dual(P, max_updates=cap)
    assert o["h"] == r["h"] and np.float32(o["Jp"]) == np.float32(r["Jp"]) and np.float32(o["Jd"]) == np.float32(r["Jd"])


def _growing_problem(N, M, seed):
    """Rows with three negative off-diagonal entries (a = 3 < 5 = Theta) and
    q_ii = 1: num / den = 8 / 6 per update, so y overflows to inf within a
    few hundred updates (then inf / inf = NaN); a few all-zero rows stay at
    their start.  Most entries are zero: the sparse form is taken."""
    rng = np.random.default_rng(seed)
    Q = np.zeros((N, N), np.float32)
    for i in range(N - 2):
        Q[i, i] = 1.0
        for j in rng.choice([k for k in range(N) if k != i], 3, replace=False):
            Q[i, j] = -1.0
    Fd = np.zeros(N, np.float32)
    Fd[: N // 2] = rng.standard_normal(N // 2).astype(np.float32)
    P = dict(Qd=Q.reshape(-1), Fd=Fd, Md=np.ones(1, np.float32), Qp=np.eye(M, dtype=np.float32).reshape(-1),
             Qp_inv=np.eye(M, dtype=np.float32).reshape(-1), Fp=rng.standard_normal(M).astype(np.float32),
             Mp=np.ones(1, np.float32), Gp=rng.integers(-1, 2, (N, M)).astype(np.float32).reshape(-1),
             Kp=(rng.random(N) * 10).astype(np.float32), N=N, M=M)
    return P


@pytest.mark.parametrize("N,M", [(8, 4), (28, 7), (32, 16)])
def test_sparse_form_hands_over_at_the_first_nonfinite_y(gpu_lib, orc, N, M):
    """y grows to inf and then NaN: the sparse form (which skips +-0 entries,
    exact only for a finite y) must hand over to the dense form in time --
    the fixed-mode Y equals the reference's update by update, NaN included."""
    P = _growing_problem(N, M, N)
    for k in (50, 200, 400, 1000):
        want = orc.iterate(P["Qd"], P["Fd"], N, k - 1)
        for form in ("sparse", "dense"):
            with tuned(gpu_lib, FORMS[form]):
                r = gpu_lib.solve_dual(P, mode=gpu_lib.MODE_FIXED, num_iter=k)
            assert _same_bits_or_both_nan(r["Y"], want), f"{form} N={N} after {k - 1} updates"
    assert not np.all(np.isfinite(orc.iterate(P["Qd"], P["Fd"], N, 999)))  # the case is exercised


@pytest.mark.parametrize("np_", [2, 3, 4])
@pytest.mark.parametrize("N,M", [(8, 4), (28, 7), (32, 16)])
def test_converge_sparse_update_past_overflow(gpu_lib, orc, N, M, np_):
    """Converge mode capped past the overflow: k_solve_quintet's update wave
    (sparse form, then dense) against the oracle's solve, Y and U; two and
    three B / C waves per role."""
    P = _growing_problem(N, M, N + 1)
    for cap in (100, 500):
        h, Y, U = orc.solve(P, 0, 1000, cap)
        with tuned(gpu_lib, {"tiny_np": np_, "tiny_ablk": {2: 1, 3: 2, 4: 1}[np_]}):
            r = gpu_lib.solve_dual(P, max_updates=cap)
        # the oracle returns -h when capped; a NaN cost passes every gap test
        # (NaN comparisons are false), so the reference may also stop there
        assert r["h"] == abs(h) and r["converged"] == (h > 0), (r["h"], h)
        assert _same_bits_or_both_nan(r["Y"], Y), f"N={N} cap={cap}"
        assert _same_bits_or_both_nan(r["U"], U), f"U N={N} cap={cap}"


@pytest.mark.parametrize("np_", [2, 3, 4])
def test_stalled_decision_reports_an_error(gpu_lib, golden_bundled, np_):
    """Every wait of k_solve_quintet is bounded: with its deciding waves
    stalled (test knob), the launch ends and the solve returns PQP_ERR_HIP
    instead of hanging; the next solve on the same handle is exact again."""
    g = golden_bundled
    with tuned(gpu_lib, {"tiny_np": np_}), gpu_lib.Problem(bundled_problem(g)) as prob:
        with tuned(gpu_lib, {"tiny_stall": 1}):
            with pytest.raises(gpu_lib.PQPError, match="hand-off wait expired"):
                prob.solve(max_updates=CAP)
        r = prob.solve(max_updates=CAP)
        assert r["h"] == 313
        assert_bitwise(r["Y"], g["Ystar"], "Y* after the error")


@pytest.mark.parametrize("np_", [2, 3, 4])
def test_repeated_one_shot_solves_stay_exact(gpu_lib, golden_bundled, np_):
    """A race between the waves (a ring slot read before it is written) shows
    up as a wrong h or wrong bits in some solves: 400 one-shot solves in a
    row, alternating modes, every one exact (k_solve_quintet's progress words
    are acquire / release at workgroup scope)."""
    g = golden_bundled
    P = bundled_problem(g)
    bad = []
    stale0 = gpu_lib.tune_get("tiny_stale")
    prev_np = gpu_lib.tune("tiny_np", np_)  # round 6: three B / C waves per role
    prev_ac = gpu_lib.tune("tiny_apoll", 1 if np_ == 2 else 0)  # np 2 with polling: round 5's kernel
    for n in range(200):
        r = gpu_lib.solve_dual(P, max_updates=CAP)
        if r["h"] != 313 or r["Y"].tobytes() != g["Ystar"].tobytes() or r["U"].tobytes() != g["Ustar"].tobytes():
            bad.append(("converge", n, r["h"]))
        # a short solve between the long ones: a stale pinned output would
        # hand the next solve this one's h (1 or 2)
        k = 1 + n % 2
        f = gpu_lib.solve_dual(P, mode=gpu_lib.MODE_FIXED, num_iter=k)
        if f["h"] != k or f["Y"].tobytes() != g[f"Y_h{k}"].tobytes():
            bad.append(("fixed", k, n, f["h"]))
        f = gpu_lib.solve_dual(P, mode=gpu_lib.MODE_FIXED, num_iter=1000)
        if f["Y"].tobytes() != g["Y_fixed999"].tobytes():
            bad.append(("fixed", 1000, n, f["h"]))
    gpu_lib.tune("tiny_np", prev_np)
    gpu_lib.tune("tiny_apoll", prev_ac)
    assert not bad, bad[:10]
    # every solve's pinned output carried its own launch's tag (the device-copy
    # fallback never ran)
    assert gpu_lib.tune_get("tiny_stale") == stale0


@pytest.mark.parametrize("chunk", [1, 7, 8, 100])
def test_bundled_resumed_over_launches(gpu_lib, golden_bundled, chunk):
    """a one-launch tiny solve is bounded to a chunk of iterates per
    launch and resumes from the device state (fresh = 0) in the next launch.
    With tiny chunks (the tiny_chunk knob) the bundled solves still stop at h =
    313 with the reference's Y*, U*, Jp, Jd, and the fixed solves give the
    reference's Y after 999 and after 99 updates."""
    g = golden_bundled
    with tuned(gpu_lib, {"tiny_chunk": chunk}), gpu_lib.Problem(bundled_problem(g)) as prob:
        r = prob.solve(max_updates=CAP)
        assert r["converged"] and r["h"] == 313
        assert_bitwise(r["Y"], g["Ystar"], f"chunk {chunk}: Y*")
        assert_bitwise(r["U"], g["Ustar"], f"chunk {chunk}: U*")
        assert np.float32(r["Jp"]) == g["iter_Jp"][-1] and np.float32(r["Jd"]) == g["iter_Jd"][-1]
        c = prob.solve(max_updates=16)
        assert not c["converged"] and c["h"] == 17
        f = prob.solve(gpu_lib.MODE_FIXED, num_iter=1000)
        assert f["h"] == 1000
        assert_bitwise(f["Y"], g["Y_fixed999"], f"chunk {chunk}: fixed-999 Y")
        f = prob.solve(gpu_lib.MODE_FIXED, num_iter=100)
        assert f["h"] == 100
        assert_bitwise(f["Y"], g["Y_h100"], f"chunk {chunk}: Y after 99 updates")


def test_device_copy_fallback_is_exact_and_reports_errors(gpu_lib, golden_bundled):
    """the path a solve takes when its pinned output lacks the
    launch's tag (forced by the tiny_fallback knob) reads Y, U, the state AND
    the error word from the device: exact results, and an expired wait still
    raises instead of relaunching forever."""
    g = golden_bundled
    stale0 = gpu_lib.tune_get("tiny_stale")
    with tuned(gpu_lib, {"tiny_fallback": 1}), gpu_lib.Problem(bundled_problem(g)) as prob:
        r = prob.solve(max_updates=CAP)
        assert r["h"] == 313
        assert_bitwise(r["Y"], g["Ystar"], "fallback: Y*")
        assert_bitwise(r["U"], g["Ustar"], "fallback: U*")
        f = prob.solve(gpu_lib.MODE_FIXED, num_iter=1000)
        assert_bitwise(f["Y"], g["Y_fixed999"], "fallback: fixed-999 Y")
        with tuned(gpu_lib, {"tiny_stall": 1}):
            with pytest.raises(gpu_lib.PQPError, match="hand-off wait expired"):
                prob.solve(max_updates=CAP)
        r = prob.solve(max_updates=CAP)
        assert r["h"] == 313
    assert gpu_lib.tune_get("tiny_stale") > stale0


def test_tiny_trace_buffer_too_small_is_rejected(gpu_lib):
    """the quintet's timeline writes 24 words; a shorter buffer is
    an argument error, not an out-of-bounds device write."""
    import torch

    buf = torch.zeros(24, dtype=torch.int64, device="cuda")
    with pytest.raises(gpu_lib.PQPError):
        gpu_lib._check(gpu_lib.lib().pqp_tune_trace(b"tiny", gpu_lib.C.c_void_p(buf.data_ptr()), 8))
    gpu_lib._check(gpu_lib.lib().pqp_tune_trace(b"tiny", gpu_lib.C.c_void_p(buf.data_ptr()), 24))
    gpu_lib._check(gpu_lib.lib().pqp_tune_trace(b"tiny", None, 0))
