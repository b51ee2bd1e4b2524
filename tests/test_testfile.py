"""testing/ sample-test format: the product's reader
against the reference's own reader (testing/CPU version/PQP_CPU_test.c
input(), compiled into oracle/_ref) and the committed fixture.  Host-only."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np
import pytest

from conftest import GOLDEN, assert_bitwise

from oracle import REF_TEST_SO, ReferenceTesting

TEST2 = GOLDEN / "testing" / "test2.txt"
SAMPLE_DIR = Path("/root/reference/testing/sample test")


def test_glibc_rand_emulation_matches_libc():
    import pqp_amd

    n = 5000
    out = (C.c_int * n)()
    assert pqp_amd.lib().pqp_tune_glibc_rand(n, out) == 0
    libc = C.CDLL(None)
    libc.srand(1)
    assert list(out) == [libc.rand() for _ in range(n)]


def test_reader_matches_golden_fixture():
    import pqp_amd

    g = dict(np.load(GOLDEN / "testing_test2.npz"))
    P = pqp_amd.read_testfile(TEST2)
    assert (P["M"], P["N"]) == (int(g["M"]), int(g["N"])) == (100, 400)
    for k in ("Qp_inv", "Fp", "Mp", "Gp", "Kp"):
        assert_bitwise(P[k], g[k], k)


@pytest.mark.skipif(not REF_TEST_SO.exists() or not SAMPLE_DIR.exists(), reason="needs /root/reference")
@pytest.mark.parametrize("name", ["test1.txt", "test2.txt", "test3.txt"])
def test_reader_matches_reference_reader(name):
    import pqp_amd

    exp = ReferenceTesting().read_testfile(SAMPLE_DIR / name)
    got = pqp_amd.read_testfile(SAMPLE_DIR / name)
    assert (got["M"], got["N"]) == (exp["M"], exp["N"])
    for k in ("Qp_inv", "Fp", "Mp", "Gp", "Kp"):
        assert_bitwise(got[k], exp[k], f"{name} {k}")


def test_gp_mapping_quirk_and_kp_option(tmp_path):
    """-1 in the file becomes +1 (C's -1 % 3 == -1), 2 becomes -1; glibc_kp=0
    keeps the file's Kp."""
    import pqp_amd

    f = tmp_path / "t.txt"
    f.write_text("2 3\n1.5 2.5\n0.5 -0.5\n7.0\n1 2 3\n0 1\n-1 2\n5 -3\n")
    P = pqp_amd.read_testfile(f, glibc_kp=False)
    assert P["Gp"].tolist() == [0, 1, 1, -1, -1, 0]
    assert P["Kp"].tolist() == [1, 2, 3]
    assert P["Qp_inv"].tolist() == [1.5, 0, 0, 2.5] and float(P["Mp"][0]) == 7.0
    Q = pqp_amd.read_testfile(f)
    assert np.allclose(Q["Kp"], [8.401877, 3.9438293, 7.830992])  # glibc rand() from seed 1


def test_reader_errors(tmp_path):
    import pqp_amd

    with pytest.raises(pqp_amd.PQPError) as e:
        pqp_amd.read_testfile(tmp_path / "missing.txt")
    assert e.value.code == pqp_amd.PQP_ERR_IO
    f = tmp_path / "short.txt"
    f.write_text("2 3\n1.5 2.5\n0.5\n")
    with pytest.raises(pqp_amd.PQPError) as e:
        pqp_amd.read_testfile(f)
    assert "malformed" in str(e.value)
