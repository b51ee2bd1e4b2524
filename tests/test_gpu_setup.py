"""GPU parity of the setup GEMMs: convertToDual
(PQP_CPU.c:440-498) with a DENSE Qp_inv through the LDS-tiled k_matmul_tiled,
against digests of the reference's own Qd / Fd / Md (tests/golden/
dense_dual.npz); the tiled and one-thread-per-output products bit-identical on
ragged shapes and all four transpose modes (matrixMultiply, :84-147)."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import GOLDEN, assert_bitwise

pytestmark = pytest.mark.gpu

from pqp_amd import dense_qinv  # noqa: E402


@pytest.fixture(scope="module")
def dense():
    return np.load(GOLDEN / "dense_dual.npz")


@pytest.mark.parametrize("tag", ["n1024_m512_s3_i0", "n300_m77_s4_i2"])
def test_batch_convert_to_dual_dense_qinv(gpu_lib, orc, dense, tag):
    import torch

    N, M, seed, inst = (int(v) for v in dense[f"{tag}_meta"])
    P = orc.synth_primal(seed, inst, N, M)
    B = 2
    pb = gpu_lib.ProblemBatch(B, N, M)
    pb.set("Qp_inv", np.stack([dense_qinv(seed, M)] * B))
    for k in ("Gp", "Kp", "Fp", "Mp"):
        pb.set(k, np.stack([np.asarray(P[k], np.float32).reshape(-1)] * B))
    pb.convert_to_dual()
    torch.cuda.synchronize()
    for b in range(B):
        Qd = pb.Qd[b].cpu().numpy()
        assert hashlib.sha256(Qd.tobytes()).digest() == dense[f"{tag}_Qd_sha256"].tobytes(), f"Qd of problem {b}"
        assert_bitwise(pb.Fd[b].cpu().numpy(), dense[f"{tag}_Fd"], "Fd")
        assert_bitwise(pb.Md[b:b + 1].cpu().numpy(), dense[f"{tag}_Md"], "Md")


def test_dropin_convert_to_dual_dense_qinv(gpu_lib, orc, dense):
    tag = "n300_m77_s4_i2"
    N, M, seed, inst = (int(v) for v in dense[f"{tag}_meta"])
    P = orc.synth_primal(seed, inst, N, M)
    Qd, Fd, Md = np.zeros(N * N, np.float32), np.zeros(N, np.float32), np.zeros(1, np.float32)
    gpu_lib.convertToDual(Qd, Fd, Md, dense_qinv(seed, M), P["Gp"].copy(), P["Kp"].copy(), P["Fp"].copy(),
                          P["Mp"].copy(), N, M)
    assert hashlib.sha256(Qd.tobytes()).digest() == dense[f"{tag}_Qd_sha256"].tobytes()
    assert_bitwise(Fd, dense[f"{tag}_Fd"], "Fd")
    assert_bitwise(Md, dense[f"{tag}_Md"], "Md")


@pytest.mark.parametrize("a,b,c", [(32, 1, 32), (33, 70, 65), (64, 48, 40), (100, 37, 129), (257, 33, 31),
                                   (128, 512, 128)])
def test_tiled_matmul_vs_oracle_and_seq(gpu_lib, orc, a, b, c):
    L = gpu_lib.lib()
    rng = np.random.default_rng(a * 1000 + b * 10 + c)
    for tA in (0, 1):
        for tB in (0, 1):
            A = rng.standard_normal(a * b).astype(np.float32)
            Bm = rng.standard_normal(b * c).astype(np.float32)
            A[::7] = 0.0  # exact zeros / -0 mixed in
            Bm[::11] = -0.0
            out = np.zeros(a * c, np.float32)
            gpu_lib.matrixMultiply(out, A, tA, Bm, tB, a, b, c)
            assert_bitwise(out, orc.matmul(A, tA, Bm, tB, a, b, c), f"tiled {a}x{b}x{c} t{tA}{tB}")
            prev = L.pqp_tune_matmul_tiled(1)
            try:
                seq = np.zeros(a * c, np.float32)
                gpu_lib.matrixMultiply(seq, A, tA, Bm, tB, a, b, c)
            finally:
                L.pqp_tune_matmul_tiled(prev)
            assert_bitwise(out, seq, f"tiled vs seq {a}x{b}x{c} t{tA}{tB}")


@pytest.mark.parametrize("a,b,c", [(64, 4, 64), (128, 32, 128), (132, 100, 260), (260, 36, 68), (200, 516, 72),
                                   (1024, 512, 128)])
def test_packed_matmul_vs_oracle_and_tiled(gpu_lib, orc, a, b, c):
    """k_matmul_pk (128 x 128 tiles, 8 x 8 outputs per thread on packed fp32,
    the k range zero-padded to the 32-deep slab) in all four transpose modes:
    bit-identical to the oracle and to the 64 x 64 k_matmul_tiled
    (pqp_tune("matmul_pk_off", 1)); ragged tiles in i, j and k, exact +-0,
    and inf / NaN operands (matrixMultiply, PQP_CPU.c:84-147)."""
    import pqp_amd

    rng = np.random.default_rng(a * 7 + b * 3 + c)
    for tA in (0, 1):
        for tB in (0, 1):
            A = rng.standard_normal(a * b).astype(np.float32)
            Bm = rng.standard_normal(b * c).astype(np.float32)
            A[::7] = 0.0
            Bm[::11] = -0.0
            A[5], Bm[9] = np.inf, np.nan
            out = np.zeros(a * c, np.float32)
            gpu_lib.matrixMultiply(out, A, tA, Bm, tB, a, b, c)
            _same_up_to_nan_payload(out, orc.matmul(A, tA, Bm, tB, a, b, c), f"pk {a}x{b}x{c} t{tA}{tB}")
            prev = pqp_amd.tune("matmul_pk_off", 1)
            try:
                ref = np.zeros(a * c, np.float32)
                gpu_lib.matrixMultiply(ref, A, tA, Bm, tB, a, b, c)
            finally:
                pqp_amd.tune("matmul_pk_off", prev)
            _same_up_to_nan_payload(out, ref, f"pk vs tiled {a}x{b}x{c} t{tA}{tB}")


def _same_up_to_nan_payload(got, want, what):
    """Bit for bit, except that a NaN result only has to be a NaN: a NaN
    operand's payload and sign are not carried the same way by the host's and
    the GPU's multiply (the solver's own kernels are compared on NaN bits in
    test_gpu_parity / test_gpu_mid)."""
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan), what
    assert_bitwise(got[~nan], want[~nan], what)


@pytest.mark.parametrize("a,b", [(64, 32), (300, 77), (1024, 512), (257, 1000)])
def test_matvec_rows_vs_oracle_and_seq(gpu_lib, orc, a, b):
    """k_matvec_rows (out = A x, one lane per row, rows staged through LDS with
    coalesced loads, k zero-padded to the 32-deep slab): bit-identical to the
    oracle and to the one-thread-per-output k_matmul_seq, either transpose
    flag on the vector (matrixMultiply :84-147 with c = 1)."""
    rng = np.random.default_rng(a + 17 * b)
    A = rng.standard_normal(a * b).astype(np.float32)
    x = rng.standard_normal(b).astype(np.float32)
    A[::13] = -0.0
    x[3] = np.inf
    for tB in (0, 1):
        out = np.zeros(a, np.float32)
        gpu_lib.matrixMultiply(out, A, 0, x, tB, a, b, 1)
        assert_bitwise(out, orc.matmul(A, 0, x, tB, a, b, 1), f"matvec {a}x{b} tB={tB}")
        prev = gpu_lib.tune("matmul_tiled_off", 1)
        try:
            seq = np.zeros(a, np.float32)
            gpu_lib.matrixMultiply(seq, A, 0, x, tB, a, b, 1)
        finally:
            gpu_lib.tune("matmul_tiled_off", prev)
        assert_bitwise(out, seq, f"matvec vs seq {a}x{b}")


@pytest.mark.parametrize("b,c", [(32, 1), (512, 512), (77, 300), (1000, 1), (513, 65)])
def test_vecmat_vs_oracle_and_seq(gpu_lib, orc, b, c):
    """k_vecmat (a = 1: out[j] = sum_k x[k] B(k, j), one lane per j, eight
    loads ahead of the adds): bit-identical to the oracle and to k_matmul_seq
    for either transpose flag of B (and of the one-row A)."""
    rng = np.random.default_rng(b * 31 + c)
    x = rng.standard_normal(b).astype(np.float32)
    Bm = rng.standard_normal(b * c).astype(np.float32)
    Bm[::9] = -0.0
    for tA in (0, 1):
        for tB in (0, 1):
            out = np.zeros(c, np.float32)
            gpu_lib.matrixMultiply(out, x, tA, Bm, tB, 1, b, c)
            assert_bitwise(out, orc.matmul(x, tA, Bm, tB, 1, b, c), f"vecmat {b}x{c} t{tA}{tB}")
            prev = gpu_lib.tune("matmul_tiled_off", 1)
            try:
                seq = np.zeros(c, np.float32)
                gpu_lib.matrixMultiply(seq, x, tA, Bm, tB, 1, b, c)
            finally:
                gpu_lib.tune("matmul_tiled_off", prev)
            assert_bitwise(out, seq, f"vecmat vs seq {b}x{c}")
