"""Shared test setup.

Markers: ``gpu`` tests need an MI355X (run on the GPU box with -m gpu); all
other tests run on CPU.  ``oracle/`` is imported here strictly as the checker.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
EXAMPLE_DIR = GOLDEN / "example"
for p in (ROOT / "pqp-for-mpc_amd", ROOT / "oracle", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


# A broken converge-mode solve must fail, not hang the GPU box: cap the
# drop-in solveQuadraticDual (and the CLI / reference-main subprocesses, which
# inherit the environment).  Correct runs need <= 4524 updates here.
os.environ.setdefault("PQP_MAX_UPDATES", "200000")
CAP = 200000


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")


@pytest.fixture(scope="session")
def orc():
    from oracle import Oracle

    return Oracle()


@pytest.fixture(scope="session")
def golden_bundled():
    return dict(np.load(GOLDEN / "bundled.npz"))


@pytest.fixture(scope="session")
def golden_converge():
    return dict(np.load(GOLDEN / "synth_converge.npz"))


@pytest.fixture(scope="session")
def golden_large():
    return dict(np.load(GOLDEN / "synth_large.npz"))


def bits(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32)).view(np.uint32)


def assert_bitwise(actual, expected, what=""):
    a, e = bits(actual), bits(expected)
    assert a.shape == e.shape, f"{what}: shape {a.shape} != {e.shape}"
    bad = np.nonzero(a != e)[0]
    if bad.size:
        i = bad[0]
        raise AssertionError(f"{what}: {bad.size} of {a.size} values differ; first at {i}: "
                             f"{np.float32(a[i:i+1].view(np.float32)[0])!r} vs {np.float32(e[i:i+1].view(np.float32)[0])!r}")


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a GPU; fails loudly (no fallback) without one."""
    import pqp_amd

    L = pqp_amd.lib()
    return pqp_amd
