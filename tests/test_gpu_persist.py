"""GPU parity of the persistent fixed-mode launch (pqp_persist.hip): one
problem of n_dual <= 1024, every update inside ONE kernel, the iterate handed
between workgroups as tagged granules.  Bar: bit-exact with the oracle
(PQP_CPU.c's updateY2 restated) and with the graph-replayed relay update
(pqp_tune_persist(1)), for ragged sizes around the wave slices (k of 96,
144, then 196 per wave: boundaries 96, 240, 436, 632, 828) and the
workgroup (16 rows) boundaries, update counts of both parities, repeated
solves, special values, the traced launch, and the size limit (N = 1025
falls back)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _dual(orc, N, seed=8, inst=1):
    M = max(1, N // 2)
    P = orc.synth_problem(seed, inst, N, M, with_qp=False)
    P.update(Qp=np.zeros(M * M, np.float32))
    return P


def _solve(gpu_lib, P, num_iter, persist=True, reps=1):
    L = gpu_lib.lib()
    old = L.pqp_tune_persist(0 if persist else 1)
    try:
        with gpu_lib.Problem(P) as prob:
            rs = [prob.solve(gpu_lib.MODE_FIXED, num_iter=num_iter) for _ in range(reps)]
    finally:
        L.pqp_tune_persist(old)
    return rs


@pytest.mark.parametrize("N", [1, 4, 95, 96, 97, 99, 100, 191, 192, 193, 240, 241, 257, 384, 436, 437, 575, 576,
                               577, 632, 633, 828, 829, 1000, 1023, 1024])
def test_persistent_fixed_mode_vs_oracle(gpu_lib, orc, N):
    P = _dual(orc, N)
    ups = 11
    want = orc.iterate(P["Qd"], P["Fd"], N, ups)
    (r,) = _solve(gpu_lib, P, ups + 1)
    assert r["h"] == ups + 1
    assert_bitwise(r["Y"], want, f"persistent N={N}")


@pytest.mark.parametrize("num_iter", [1, 2, 3, 4, 257, 1000])
def test_persistent_update_counts_and_replays(gpu_lib, orc, num_iter):
    """Both parities of the update count, a single update, no update at all
    (num_iter = 1: Y stays 1000), three solves on one handle (the granules'
    tags are reset before every launch); equal to the relay path."""
    N = 1024
    P = _dual(orc, N, seed=3, inst=5)
    rs = _solve(gpu_lib, P, num_iter, persist=True, reps=3)
    (rr,) = _solve(gpu_lib, P, num_iter, persist=False)
    if num_iter <= 12:
        want = orc.iterate(P["Qd"], P["Fd"], N, num_iter - 1) if num_iter > 1 else np.full(N, 1000, np.float32)
        assert_bitwise(rr["Y"], want, "relay vs oracle")
    for i, r in enumerate(rs):
        assert r["h"] == num_iter
        assert_bitwise(r["Y"], rr["Y"], f"persistent solve {i} vs relay, num_iter={num_iter}")


def test_persistent_special_values(gpu_lib, orc):
    """inf/NaN/-0 entries of Qd and Fd propagate exactly as in the literal
    reference formula through many updates."""
    N = 300
    rng = np.random.default_rng(17)
    Qd = rng.standard_normal((N, N)).astype(np.float32)
    Qd[rng.random((N, N)) < 0.1] = 0.0
    Qd[rng.random((N, N)) < 0.05] = -0.0
    Qd[rng.random((N, N)) < 0.0005] = np.inf
    Qd[rng.random((N, N)) < 0.0005] = np.nan
    Qd = Qd.reshape(-1)
    Fd = rng.standard_normal(N).astype(np.float32)
    Fd[::7] = -0.0
    M = 4
    P = dict(Qd=Qd, Fd=Fd, Md=np.zeros(1, np.float32), Qp=np.zeros(M * M, np.float32),
             Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32), Mp=np.zeros(1, np.float32),
             Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32), N=N, M=M)
    ups = 6
    want = orc.iterate(Qd, Fd, N, ups)
    (r,) = _solve(gpu_lib, P, ups + 1)
    (rr,) = _solve(gpu_lib, P, ups + 1, persist=False)
    a, b, c = (np.asarray(x, np.float32) for x in (r["Y"], want, rr["Y"]))
    nan = np.isnan(a) & np.isnan(b)
    assert np.all(nan | (a.view(np.uint32) == b.view(np.uint32))), "persistent vs oracle"
    assert np.array_equal(np.isnan(a), np.isnan(c)) and np.all(np.isnan(a) | (a.view(np.uint32) == c.view(np.uint32)))


def test_beyond_persistent_limit_falls_back(gpu_lib, orc):
    N = 1025
    P = _dual(orc, N, seed=2, inst=2)
    want = orc.iterate(P["Qd"], P["Fd"], N, 5)
    (r,) = _solve(gpu_lib, P, 6)
    assert_bitwise(r["Y"], want, "N=1025 (relay)")


def test_persistent_traced_launch_same_bits(gpu_lib, orc):
    """The traced launch (pqp_tune_persist_trace: clock marks per wave and per
    seventh of each later wave's chain, a separate code path for the adds)
    gives the untraced launch's bits, and its marks are ordered."""
    import ctypes as C

    import torch

    N, ups, n_tr = 1024, 40, 20
    P = _dual(orc, N, seed=4, inst=2)
    (plain,) = _solve(gpu_lib, P, ups + 1)
    L = gpu_lib.lib()
    W = 6
    tr = torch.zeros(n_tr * W * 12, dtype=torch.int64, device="cuda")
    assert L.pqp_tune_persist_trace(C.c_void_p(tr.data_ptr()), n_tr) == 0
    try:
        (traced,) = _solve(gpu_lib, P, ups + 1)
    finally:
        L.pqp_tune_persist_trace(None, 0)
    assert_bitwise(traced["Y"], plain["Y"], "traced vs untraced")
    t = tr.cpu().numpy()
    coarse = t[: n_tr * W * 4].reshape(n_tr, W, 4)
    fine = t[n_tr * W * 4:].reshape(n_tr, W, 8)
    assert np.all(coarse[1:] > 0) and np.all(np.diff(coarse[1:], axis=2) >= 0)
    assert np.all(fine[1:, 1:] > 0) and np.all(np.diff(fine[1:, 1:], axis=2) >= 0)


@pytest.mark.parametrize("xcds", [2, 3, 8])
def test_persistent_packed_on_fewer_xcds(gpu_lib, orc, xcds):
    """persist_xcds: the workgroups of the persistent launch packed onto 2 or 3
    XCDs, or spread over all 8 (the default packs them onto 4, which every
    other test takes; the rest of a padded grid leaves at once) -- the same
    bits as the oracle at n_dual 1024 and at a ragged size."""
    for N in (1024, 437):
        P = _dual(orc, N)
        old = gpu_lib.tune("persist_xcds", xcds)
        try:
            r = _solve(gpu_lib, P, 257)[0]
            assert gpu_lib.tune_get("last_path") == 1, "not the persistent launch"
        finally:
            gpu_lib.tune("persist_xcds", old)
        assert_bitwise(r["Y"], orc.iterate(P["Qd"], P["Fd"], N, 256), f"N={N} on {xcds} XCDs")
