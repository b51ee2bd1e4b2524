"""GPU parity of the one-XCD form of the persistent fixed-mode launch
(k_split_persist<false, true>, pqp_persist.hip "lean"): 32 rows per workgroup
over Qd itself, the split entries formed on the fly (max(0, q * y) for den,
min(0, q * y) for num, whose sum is the exact negation of the reference's),
the diagonal entries put in place per lane, granules stored plain when every
workgroup is on one XCD (persist_lean 1; measured slower than the split
form, so not the default: profiles/r06/persist_lean_ab_r06c.json).  Bar: bit-exact with the oracle (PQP_CPU.c's
updateY2, :603-618, restated) and with the split form (the default), at
ragged sizes around the 32-row workgroups and the 24 / 40 / 48-packet slices
(k boundaries 96, 256, 448, 640, 832), with -0 / +0 entries and zero rows;
a Qd with a non-finite entry takes the split form (last_path 1), a run whose
y overflows re-runs on the split form (last_path 7) with the oracle's bits."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu

LEAN, LEAN_RERUN, SPLIT = 6, 7, 1


def _dual(orc, N, seed=8, inst=1):
    M = max(1, N // 2)
    P = orc.synth_problem(seed, inst, N, M, with_qp=False)
    P.update(Qp=np.zeros(M * M, np.float32))
    return P


def _raw(Qd, Fd, N, M=4):
    return dict(Qd=np.ascontiguousarray(Qd, np.float32).reshape(-1), Fd=np.asarray(Fd, np.float32),
                Md=np.zeros(1, np.float32), Qp=np.zeros(M * M, np.float32), Qp_inv=np.zeros(M * M, np.float32),
                Fp=np.zeros(M, np.float32), Mp=np.zeros(1, np.float32), Gp=np.zeros(N * M, np.float32),
                Kp=np.zeros(N, np.float32), N=N, M=M)


def _fixed(gpu_lib, P, num_iter, split=False):
    old = gpu_lib.tune("persist_lean", 0 if split else 1)
    try:
        with gpu_lib.Problem(P) as prob:
            r = prob.solve(gpu_lib.MODE_FIXED, num_iter=num_iter)
            path = gpu_lib.tune_get("last_path")
    finally:
        gpu_lib.tune("persist_lean", old)
    return r, path


def _same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(nan | (a.view(np.uint32) == b.view(np.uint32))))


ONE_WG = 5  # problems small enough for one workgroup's LDS never reach the persistent launch


@pytest.mark.parametrize("N", [161, 192, 193, 224, 255, 256, 257, 447, 448, 449, 639, 640, 641, 831, 832, 833, 993,
                               1000, 1023, 1024])
def test_lean_vs_oracle_and_split(gpu_lib, orc, N):
    P = _dual(orc, N, seed=11, inst=N)
    ups = 9
    want = orc.iterate(P["Qd"], P["Fd"], N, ups)
    r, path = _fixed(gpu_lib, P, ups + 1)
    assert path in (LEAN, ONE_WG), path
    if N >= 256:
        assert path == LEAN, path
    assert_bitwise(r["Y"], want, f"lean N={N}")
    rs, path_s = _fixed(gpu_lib, P, ups + 1, split=True)
    assert path_s == (SPLIT if path == LEAN else ONE_WG)
    assert_bitwise(r["Y"], rs["Y"], f"lean vs split N={N}")


@pytest.mark.parametrize("num_iter", [2, 3, 1000])
def test_lean_long_runs_vs_split(gpu_lib, orc, num_iter):
    N = 1024
    P = _dual(orc, N, seed=3, inst=5)
    r, path = _fixed(gpu_lib, P, num_iter)
    rs, _ = _fixed(gpu_lib, P, num_iter, split=True)
    assert path == LEAN
    assert_bitwise(r["Y"], rs["Y"], f"lean vs split, num_iter={num_iter}")


def test_lean_signed_zeros_and_zero_rows(gpu_lib, orc):
    """+0 / -0 entries everywhere (incl. the diagonal), a zero row, Fd with
    -0 and +0: the sums whose every term is a zero of some sign and the
    negated num chain's zero class give the reference's bits."""
    N = 300
    rng = np.random.default_rng(5)
    Qd = rng.standard_normal((N, N)).astype(np.float32)
    Qd[rng.random((N, N)) < 0.3] = 0.0
    Qd[rng.random((N, N)) < 0.3] = -0.0
    Qd[7, :] = 0.0
    Qd[9, :] = -0.0
    np.fill_diagonal(Qd[:50, :50], -0.0)
    Fd = rng.standard_normal(N).astype(np.float32)
    Fd[::5] = -0.0
    Fd[1::5] = 0.0
    P = _raw(Qd, Fd, N)
    ups = 12
    want = orc.iterate(P["Qd"], Fd, N, ups)
    r, path = _fixed(gpu_lib, P, ups + 1)
    assert path == LEAN
    assert_bitwise(r["Y"], want, "signed zeros")


def test_lean_nonfinite_qd_takes_split(gpu_lib, orc):
    N = 300
    rng = np.random.default_rng(17)
    Qd = rng.standard_normal((N, N)).astype(np.float32)
    Qd[3, 5] = np.inf
    Qd[100, 7] = np.nan
    Fd = rng.standard_normal(N).astype(np.float32)
    P = _raw(Qd, Fd, N)
    ups = 6
    r, path = _fixed(gpu_lib, P, ups + 1)
    assert path == SPLIT
    assert _same(r["Y"], orc.iterate(P["Qd"], Fd, N, ups))


@pytest.mark.parametrize("scale", [1e36, 2e35])
def test_lean_overflowing_y_reruns_on_split(gpu_lib, orc, scale):
    """Finite Qd and Theta (sum of |q| below the float range) whose products
    q * y overflow in the first update: the lean launch reports a non-finite
    y and the chunk is run again on the split form, with the oracle's bits
    (NaN where the oracle has NaN)."""
    N = 256
    rng = np.random.default_rng(23)
    Qd = (rng.standard_normal((N, N)) * scale).astype(np.float32)
    Fd = (rng.standard_normal(N) * scale).astype(np.float32)
    P = _raw(Qd, Fd, N)
    ups = 8
    reruns = gpu_lib.tune_get("lean_reruns")
    r, path = _fixed(gpu_lib, P, ups + 1)
    want = orc.iterate(P["Qd"], Fd, N, ups)
    assert _same(r["Y"], want)
    if not np.all(np.isfinite(want)):
        assert path == LEAN_RERUN and gpu_lib.tune_get("lean_reruns") == reruns + 1
    rs, _ = _fixed(gpu_lib, P, ups + 1, split=True)
    assert _same(r["Y"], rs["Y"])


def test_lean_repeated_solves_one_handle(gpu_lib, orc):
    """Granules, census words and error words are reset per launch: five
    solves on one handle give the same bits."""
    N = 1024
    P = _dual(orc, N, seed=9, inst=2)
    want = orc.iterate(P["Qd"], P["Fd"], N, 20)
    old = gpu_lib.tune("persist_lean", 1)
    try:
        with gpu_lib.Problem(P) as prob:
            for i in range(5):
                r = prob.solve(gpu_lib.MODE_FIXED, num_iter=21)
                assert gpu_lib.tune_get("last_path") == LEAN
                assert_bitwise(r["Y"], want, f"solve {i}")
    finally:
        gpu_lib.tune("persist_lean", old)
