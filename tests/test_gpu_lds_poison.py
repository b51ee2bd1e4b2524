"""LDS that a kernel never writes must never reach a result.  LDS keeps what
the previous kernel on that CU left; a kernel that reads its own padding
(vector entries past N or M) as if it were zero gets 0 * NaN = NaN once an
earlier kernel ran on non-finite data (round 5: k_solve_quintet read t's
padding, and the bundled solve stopped at h = 1 with U = NaN -- only after
test_gpu_mid's non-finite tests).  Each case here first fills every CU's LDS
with NaN or inf (pqp_tune_poison_lds), then runs a path on the bundled plant or
a ragged synthetic problem and checks the oracle's / the reference's bits."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import CAP, assert_bitwise

pytestmark = pytest.mark.gpu

KEYS = ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")
POISON = [float("nan"), float("inf"), -0.0]


def _bundled(g):
    P = {k: np.ascontiguousarray(g[k], dtype=np.float32) for k in KEYS}
    P.update(N=int(g["N"]), M=int(g["M"]))
    return P


def _batch(gpu_lib, Ps):
    N, M = int(Ps[0]["N"]), int(Ps[0]["M"])
    pb = gpu_lib.ProblemBatch(len(Ps), N, M)
    for k in KEYS:
        pb.set(k, np.stack([np.asarray(P[k], np.float32).reshape(-1) for P in Ps]))
    return pb


@pytest.fixture
def knobs(gpu_lib):
    saved = []

    def set_(key, value):
        saved.append((key, gpu_lib.tune(key, value)))

    yield set_
    for key, old in reversed(saved):
        gpu_lib.tune(key, old)


@pytest.mark.parametrize("poison", POISON)
@pytest.mark.parametrize("form", [{}, {"tiny_dense": 1}, {"tiny_old": 1}], ids=["sparse", "dense", "round4"])
def test_one_problem_after_poison(gpu_lib, golden_bundled, knobs, poison, form):
    """configs[1], one problem: converge (h = 313, Y*, U*) and fixed 1000."""
    g = golden_bundled
    P = _bundled(g)
    for k, v in form.items():
        knobs(k, v)
    gpu_lib.poison_lds(poison)
    r = gpu_lib.solve_dual(P, max_updates=CAP)
    assert r["h"] == 313 and r["converged"], (r["h"], r["Jp"], r["Jd"])
    assert_bitwise(r["Y"], g["Ystar"], "Y*")
    assert_bitwise(r["U"], g["Ustar"], "U*")
    gpu_lib.poison_lds(poison)
    f = gpu_lib.solve_dual(P, mode=gpu_lib.MODE_FIXED, num_iter=1000)
    assert_bitwise(f["Y"], g["Y_fixed999"], "fixed-999 Y")


@pytest.mark.parametrize("N,M", [(5, 3), (13, 7), (27, 5), (30, 2), (31, 31)])
def test_ragged_one_problem_after_poison(gpu_lib, orc, N, M):
    """Sizes off every instantiated width (padding in y, t and the lists):
    capped converge solves and fixed mode against the oracle."""
    P = orc.synth_problem(41, N, N, M)
    for cap in (3, 40):
        gpu_lib.poison_lds(float("nan"))
        if N + M < 64:
            h, Y, U = orc.solve(P, max_updates=cap)
            r = gpu_lib.solve_dual(P, max_updates=cap)
            assert r["h"] == abs(h)
            assert_bitwise(r["Y"], Y, f"{N}/{M} cap {cap} Y")
            assert_bitwise(r["U"], U, f"{N}/{M} cap {cap} U")
        gpu_lib.poison_lds(float("nan"))
        _, Y, _ = orc.solve(P, mode=1, num_iter=cap)
        f = gpu_lib.solve_dual(P, mode=gpu_lib.MODE_FIXED, num_iter=cap)
        assert_bitwise(f["Y"], Y, f"{N}/{M} fixed {cap}")


@pytest.mark.parametrize("knob", [{}, {"wave_pipe_max_b": 0}, {"wave_min_b": 1 << 30}], ids=["pipe", "plain", "tiny4"])
def test_bundled_batch_after_poison(gpu_lib, golden_bundled, knobs, knob):
    """Batched configs[1] (k_solve_wave pipelined / plain, k_solve_tiny)."""
    g = golden_bundled
    for k, v in knob.items():
        knobs(k, v)
    gpu_lib.poison_lds(float("nan"))
    pb = _batch(gpu_lib, [_bundled(g)] * 5).solve(max_updates=CAP)
    for b in (0, 4):
        assert int(pb.h[b]) == 313
        assert_bitwise(pb.Y[b].cpu().numpy(), g["Ystar"], f"copy {b} Y*")
        assert_bitwise(pb.U[b].cpu().numpy(), g["Ustar"], f"copy {b} U*")


@pytest.mark.parametrize("form", [(0, 2), (0, 1), (1, 0)], ids=["mid2", "pair", "v1"])
def test_horizon_batch_after_poison(gpu_lib, golden_bundled, orc, knobs, form):
    """The bundled plant over 3 horizon blocks (n_dual 84, path 3)."""
    from oracle import block_diag_problem

    knobs("mid_v1", form[0])
    knobs("mid2_pair", form[1])
    knobs("mid2_min_n", 0)
    Q = block_diag_problem(_bundled(golden_bundled), 3)
    gpu_lib.poison_lds(float("nan"))
    pb = _batch(gpu_lib, [Q] * 3).solve(max_updates=CAP)
    h, Y, U = orc.solve(Q, max_updates=CAP)
    assert h == 313
    for b in (0, 2):
        assert int(pb.h[b]) == 313
        assert_bitwise(pb.Y[b].cpu().numpy(), Y, f"copy {b} Y")
        assert_bitwise(pb.U[b].cpu().numpy(), U, f"copy {b} U")


@pytest.mark.parametrize("H", [2, 4])
def test_horizon_single_after_poison(gpu_lib, golden_bundled, orc, H):
    """One horizon problem (the persistent converge launch and its fallbacks)."""
    from oracle import block_diag_problem

    Q = block_diag_problem(_bundled(golden_bundled), H)
    gpu_lib.poison_lds(float("nan"))
    r = gpu_lib.solve_dual(Q, max_updates=CAP)
    h, Y, U = orc.solve(Q, max_updates=CAP)
    assert r["h"] == h == 313
    assert_bitwise(r["Y"], Y, "Y")
    assert_bitwise(r["U"], U, "U")


def test_converge_fixtures_after_poison(gpu_lib, golden_converge, orc):
    """The reference's converging synthetic cases (default routes: one
    workgroup, the persistent converge launch, the graph chain by size)."""
    cases, Ys, Us = golden_converge["cases"], golden_converge["Y"], golden_converge["U"]
    yo = uo = 0
    for (N, M, seed, h_ref) in cases:
        N, M = int(N), int(M)
        P = orc.synth_problem(int(seed), 0, N, M)
        gpu_lib.poison_lds(float("nan"))
        r = gpu_lib.solve_dual(P, max_updates=CAP)
        assert r["converged"] and r["h"] == int(h_ref), (N, M, seed, r["h"])
        assert_bitwise(r["Y"], Ys[yo:yo + N], f"Y {N}/{M}/{seed}")
        assert_bitwise(r["U"], Us[uo:uo + M], f"U {N}/{M}/{seed}")
        yo += N
        uo += M


@pytest.mark.parametrize("N,M", [(33, 9), (300, 70), (1024, 512), (2050, 100)])
def test_fixed_mode_after_poison(gpu_lib, orc, N, M):
    """Fixed mode of one problem (persistent / relay updates by size)."""
    P = orc.synth_problem(43, 1, N, M)
    gpu_lib.poison_lds(float("nan"))
    f = gpu_lib.solve_dual(P, mode=gpu_lib.MODE_FIXED, num_iter=9)
    _, Y, _ = orc.solve(P, mode=1, num_iter=9)
    assert_bitwise(f["Y"], Y, f"{N}/{M} fixed 9")


@pytest.mark.parametrize("tag", ["n1024_m512_s1_i0", "n1000_m500_s2_i7"])
def test_batched_updates_after_poison(gpu_lib, golden_large, tag):
    """The headline batched update (k_batch_stream / the iterate kernels)."""
    N, M, seed, inst, ups = (int(v) for v in golden_large[f"{tag}_meta"])
    b = gpu_lib.Batch(1, N).generate(seed, inst0=inst, M=M)
    b.reset()
    gpu_lib.poison_lds(float("nan"))
    b.iterate(ups)
    assert_bitwise(b.result()[0], golden_large[f"{tag}_Y"], "Y via batch_iterate")
