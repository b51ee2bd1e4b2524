"""CPU AddressSanitizer / UBSan runs of libpqp's host code:
the file readers (pqp_read_example, pqp_read_testfile: missing, short,
malformed, oversized and changed-between-calls files) and the C-ABI
argument / handle paths of the shim, built with host-side sanitizers
(tests/asan/Makefile).  No GPU: the shim's calls end in PQP_ERR_ARG or
PQP_ERR_NO_DEVICE.  References: PQP_CPU.c:757-930 (input()), testing/CPU
version/PQP_CPU_test.c:936-978."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

from conftest import ROOT

ASAN = ROOT / "tests" / "asan"


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    kobj = ROOT / "pqp-for-mpc_amd" / "build" / "pqp_tiny.o"
    if not kobj.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "pqp-for-mpc_amd")], check=True)
    out = tmp_path_factory.mktemp("asan_build")
    subprocess.run(["make", "-s", "-j4", "-C", str(ASAN), f"OUT={out}"], check=True, timeout=600)
    return out


def _run(exe, *args, leaks=True):
    env = dict(os.environ, ASAN_OPTIONS=f"detect_leaks={int(leaks)}:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    return subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300, env=env)


def test_readers_under_asan(built, tmp_path):
    r = _run(built / "asan_readers", str(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    assert "all cases passed" in r.stdout


def test_capi_argument_paths_under_asan(built):
    # the HIP runtime's own allocations are not ours to leak-check
    r = _run(built / "asan_capi", leaks=False)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    assert "all cases passed" in r.stdout
