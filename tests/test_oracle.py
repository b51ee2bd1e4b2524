"""The oracle (CPU restatement of PQP_CPU.c) pinned against the reference.

Two anchors:
  * the committed golden fixtures (tests/golden/*.npz, produced by the
    reference itself via tests/golden/make_golden.py) -- always run;
  * the compiled reference oracle/_ref/libpqp_ref.so -- run where it exists.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import EXAMPLE_DIR, GOLDEN, assert_bitwise

from oracle import REF_SO, Reference


def test_bundled_setup_matches_golden(orc, golden_bundled):
    P = orc.bundled_problem(EXAMPLE_DIR)
    g = golden_bundled
    for k in ("Qp_inv", "Gp", "Kp", "Fp", "Mp", "Qp", "Qd", "Fd", "Md"):
        assert_bitwise(P[k], g[k], k)
    assert_bitwise(orc.theta(P["Qd"], P["N"]), g["theta"], "theta")


def test_bundled_iterates_match_golden(orc, golden_bundled):
    g = golden_bundled
    N = int(g["N"])
    th = orc.theta(g["Qd"], N)
    Y = np.full(N, 1000.0, np.float32)
    snaps = {}
    for h in range(1, 313):
        if h in (1, 2, 10, 100, 312):
            snaps[h] = Y
        Y = orc.update(Y, g["Qd"], th, g["Fd"], N)
    for h, y in snaps.items():
        assert_bitwise(y, g[f"Y_h{h}"], f"Y_h{h}")
    assert_bitwise(Y, g["Ystar"], "Y after 312 updates")


def test_bundled_solve_matches_golden(orc, golden_bundled):
    g = golden_bundled
    P = {k: g[k] for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
    P.update(N=int(g["N"]), M=int(g["M"]))
    h, Y, U = orc.solve(P)
    assert h == int(g["h"]) == 313
    assert_bitwise(Y, g["Ystar"], "Ystar")
    U = orc.u_from_y(Y, P["Fp"], P["Gp"], P["Qp_inv"], P["N"], P["M"])
    assert_bitwise(U, g["Ustar"], "Ustar")
    assert np.float32(orc.cost(U, P["Qp"], P["Fp"], P["Mp"], P["M"])) == g["Jp"]
    assert np.float32(orc.cost(Y, P["Qd"], P["Fd"], P["Md"], P["N"])) == g["Jd"]
    # the FMA-contracted reference build is a result we must NOT reproduce
    assert not np.array_equal(Y.view(np.uint32), g["Ystar_fma_contracted"].view(np.uint32))


def test_bundled_fixed_mode(orc, golden_bundled):
    g = golden_bundled
    P = {k: g[k] for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
    P.update(N=int(g["N"]), M=int(g["M"]))
    h, Y, _ = orc.solve(P, mode=1, num_iter=1000)
    assert h == 1000
    assert_bitwise(Y, g["Y_fixed999"], "fixed-999 Y")


def test_bundled_per_iteration_costs(orc, golden_bundled):
    g = golden_bundled
    N, M = int(g["N"]), int(g["M"])
    th = orc.theta(g["Qd"], N)
    Y = np.full(N, 1000.0, np.float32)
    for h in range(313):
        flag, U, jp, jd = orc.terminate(Y, g["Qd"], g["Fd"], g["Md"], g["Qp"], g["Qp_inv"], g["Fp"], g["Mp"],
                                        g["Gp"], g["Kp"], N, M)
        assert int(g["iter_feasible"][h]) == 1
        assert np.float32(jp) == g["iter_Jp"][h] and np.float32(jd) == g["iter_Jd"][h], h
        assert flag == (1 if h == 312 else 0), h
        Y = orc.update(Y, g["Qd"], th, g["Fd"], N)


def test_synthetic_converge_cases(orc, golden_converge):
    cases, Ys, Us = golden_converge["cases"], golden_converge["Y"], golden_converge["U"]
    yo = uo = 0
    for (N, M, seed, h_ref) in cases:
        N, M = int(N), int(M)
        P = orc.synth_problem(int(seed), 0, N, M)
        h, Y, U = orc.solve(P, max_updates=100000)
        assert h == int(h_ref), (N, M, seed)
        assert_bitwise(Y, Ys[yo:yo + N], f"Y {N}/{M}/{seed}")
        U = orc.u_from_y(Y, P["Fp"], P["Gp"], P["Qp_inv"], N, M)
        assert_bitwise(U, Us[uo:uo + M], f"U {N}/{M}/{seed}")
        yo += N
        uo += M


@pytest.mark.parametrize("tag", ["n1024_m512_s1_i0", "n1000_m500_s2_i7"])
def test_synthetic_large_duals(orc, golden_large, tag):
    N, M, seed, inst, ups = (int(v) for v in golden_large[f"{tag}_meta"])
    P = orc.synth_problem(seed, inst, N, M, with_qp=False)
    assert hashlib.sha256(P["Qd"].tobytes()).digest() == golden_large[f"{tag}_Qd_sha256"].tobytes()
    assert_bitwise(P["Fd"], golden_large[f"{tag}_Fd"], "Fd")
    assert_bitwise(P["Md"], golden_large[f"{tag}_Md"], "Md")
    th = orc.theta(P["Qd"], N)
    assert_bitwise(th, golden_large[f"{tag}_theta"], "theta")
    Y = orc.iterate(P["Qd"], P["Fd"], N, ups)
    assert_bitwise(Y, golden_large[f"{tag}_Y"], "Y")


def test_split_update_equals_fused_update(orc):
    """orc_update (split entries derived on the fly) == orc_update_split (stored)."""
    rng = np.random.default_rng(0)
    for N in (1, 5, 28, 64):
        Qd = rng.standard_normal(N * N).astype(np.float32)
        Qd[rng.random(N * N) < 0.2] = 0.0
        Qd[rng.random(N * N) < 0.05] = -0.0
        Fd = rng.standard_normal(N).astype(np.float32)
        Y = rng.random(N).astype(np.float32) * 100
        th = orc.theta(Qd, N)
        qp, qn = orc.split_theta(Qd, th, N)
        fdp, fdn = np.maximum(Fd, 0).astype(np.float32), np.maximum(-Fd, 0).astype(np.float32)
        assert_bitwise(orc.update(Y, Qd, th, Fd, N), orc.update_split(Y, qp, qn, fdp, fdn, N), f"N={N}")


# -- against the compiled reference (only where /root/reference was built) --
needs_ref = pytest.mark.skipif(not REF_SO.exists(), reason="oracle/_ref not built (no /root/reference)")


@needs_ref
def test_matmul_all_transposes_vs_reference(orc):
    ref = Reference()
    rng = np.random.default_rng(1)
    import ctypes as C

    fp = C.POINTER(C.c_float)
    for (a, b, c) in [(1, 1, 1), (3, 7, 5), (17, 9, 1), (1, 33, 20), (40, 40, 40)]:
        for tA in (0, 1):
            for tB in (0, 1):
                A = rng.standard_normal(a * b).astype(np.float32)
                B = rng.standard_normal(b * c).astype(np.float32)
                out = np.zeros(a * c, np.float32)
                ref.lib.matrixMultiply(out.ctypes.data_as(fp), A.copy().ctypes.data_as(fp), tA,
                                       B.copy().ctypes.data_as(fp), tB, a, b, c)
                assert_bitwise(orc.matmul(A, tA, B, tB, a, b, c), out, f"{a}x{b}x{c} t{tA}{tB}")


@needs_ref
def test_gauss_jordan_vs_reference(orc):
    ref = Reference()
    rng = np.random.default_rng(2)
    for n in (1, 2, 7, 16, 33):
        A = (rng.standard_normal((n, n)) + n * np.eye(n)).astype(np.float32).reshape(-1)
        assert_bitwise(orc.gauss_jordan(A, n), ref.gauss_jordan(A, n), f"n={n}")
    # a matrix whose column 0 triggers the bubble-pass swaps
    A = np.array([[1, 2, 0], [3, 1, 1], [5, 0, 2]], np.float32).reshape(-1)
    assert_bitwise(orc.gauss_jordan(A, 3), ref.gauss_jordan(A, 3), "swap case")


@needs_ref
def test_random_dense_duals_vs_reference(orc):
    """Dense random primal data (not the generator's structure)."""
    ref = Reference()
    rng = np.random.default_rng(3)
    for (N, M) in [(6, 3), (20, 11), (50, 25)]:
        Qinv = rng.random((M, M)).astype(np.float32)
        Qinv = ((Qinv + Qinv.T) / 2 + M * np.eye(M)).astype(np.float32).reshape(-1)
        Gp = rng.standard_normal(N * M).astype(np.float32)
        Kp = rng.random(N).astype(np.float32) * 5
        Fp = rng.standard_normal(M).astype(np.float32)
        Mp = np.ones(1, np.float32)
        got = orc.convert_to_dual(Qinv, Gp, Kp, Fp, Mp, N, M)
        exp = ref.convert_to_dual(Qinv, Gp, Kp, Fp, Mp, N, M)
        for g_, e_, k in zip(got, exp, ("Qd", "Fd", "Md")):
            assert_bitwise(g_, e_, k)
        S = ref.split(exp[0], exp[1], N)
        th = orc.theta(exp[0], N)
        Y = np.full(N, 1000.0, np.float32)
        Yr = Y.copy()
        for _ in range(25):
            Y = orc.update(Y, exp[0], th, exp[1], N)
            Yr = ref.update(Yr, S, exp[1], N)
        assert_bitwise(Y, Yr, f"updates N={N}")
        P = dict(Qd=exp[0], Fd=exp[1], Md=exp[2], Qp=orc.gauss_jordan(Qinv, M), Qp_inv=Qinv, Fp=Fp, Mp=Mp, Gp=Gp,
                 Kp=Kp, N=N, M=M)
        flag_o, U_o, _, _ = orc.terminate(Y, P["Qd"], P["Fd"], P["Md"], P["Qp"], Qinv, Fp, Mp, Gp, Kp, N, M)
        flag_r, U_r = ref.terminate(Y, P)
        assert flag_o == flag_r
        assert_bitwise(U_o, U_r, "U")


@pytest.mark.parametrize("tag", ["n1024_m512_s3_i0", "n300_m77_s4_i2"])
def test_dense_qinv_duals_match_reference(orc, tag):
    """convertToDual with a dense Qp_inv (tests/golden/dense_dual.npz, from
    PQP_CPU.c): pins the oracle for the general setup GEMM's parity case."""
    from conftest import GOLDEN
    from pqp_amd import dense_qinv

    g = np.load(GOLDEN / "dense_dual.npz")
    N, M, seed, inst = (int(v) for v in g[f"{tag}_meta"])
    P = orc.synth_primal(seed, inst, N, M)
    Qinv = dense_qinv(seed, M)
    assert hashlib.sha256(Qinv.tobytes()).digest() == g[f"{tag}_Qinv_sha256"].tobytes()
    Qd, Fd, Md = orc.convert_to_dual(Qinv, P["Gp"], P["Kp"], P["Fp"], P["Mp"], N, M)
    assert hashlib.sha256(Qd.tobytes()).digest() == g[f"{tag}_Qd_sha256"].tobytes()
    assert_bitwise(Fd, g[f"{tag}_Fd"], "Fd")
    assert_bitwise(Md, g[f"{tag}_Md"], "Md")


@needs_ref
def test_reference_fixed_driver_matches_golden(golden_bundled):
    """oracle/ref_fixed.c (bench.py's configs[0] fixed-1000 CPU baseline) runs
    the reference's own functions: its Y after 999 updates is the golden
    fixed-999 Y* (made by make_golden.py from the reference), bit for bit."""
    from oracle import REF_FIXED_SO

    if not REF_FIXED_SO.exists():
        pytest.skip("oracle/_ref/libref_fixed.so not built")
    ref = Reference()
    P = {k: golden_bundled[k] for k in ("Qd", "Fd")}
    P["N"] = int(golden_bundled["N"])
    Y, total, loop = ref.fixed_solve(P, 1000)
    assert np.array_equal(Y.view(np.uint32), golden_bundled["Y_fixed999"].astype(np.float32).view(np.uint32))
    assert 0 < loop <= total


@pytest.mark.parametrize("k", [9, 36])
def test_block_problems_match_reference_golden(orc, golden_bundled, k):
    """The restatement on the bundled example as k diagonal blocks (a large
    problem that stops, every iterate feasible): the reference's h, Y*, U*,
    Jp, Jd (tests/golden/blocks.npz, made by the reference)."""
    from oracle import block_diag_problem

    g = np.load(GOLDEN / "blocks.npz")
    P = {kk: golden_bundled[kk] for kk in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
    P.update(N=int(golden_bundled["N"]), M=int(golden_bundled["M"]))
    Q = block_diag_problem(P, k)
    h, Y, U = orc.solve(Q, max_updates=5000)
    assert h == int(g[f"h{k}"]) == 313
    assert np.array_equal(Y.view(np.uint32), g[f"Y{k}"].view(np.uint32))
    assert np.array_equal(U.view(np.uint32), g[f"U{k}"].view(np.uint32))
    flag, _, Jp, Jd = orc.terminate(Y, Q["Qd"], Q["Fd"], Q["Md"], Q["Qp"], Q["Qp_inv"], Q["Fp"], Q["Mp"], Q["Gp"],
                                    Q["Kp"], Q["N"], Q["M"])
    assert flag == 1 and np.float32(Jp) == g[f"Jp{k}"] and np.float32(Jd) == g[f"Jd{k}"]


def test_mpc_population_sample_matches_reference_golden(orc):
    """The restatement pinned on the bench's mpc_batch population
    (tests/golden/mpc_states.npz, made by the reference itself): the states
    kept in full (every h = 314 one among them) and every 64th state give the
    reference's h and the same (Y*, U*) digest."""
    import sys

    from conftest import ROOT

    sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
    from pqp_amd import perturbed_states

    G = np.load(GOLDEN / "mpc_states.npz")
    E = orc.load_example(EXAMPLE_DIR)
    xs = perturbed_states(E["x"], len(G["h"]), seed=5)
    assert hashlib.sha256(xs.tobytes()).digest() == G["xs_sha256"].tobytes()
    assert sorted(set(G["h"].tolist())) == [313, 314] and int((G["h"] == 314).sum()) == 3
    for b in sorted(set(G["kept"].tolist()) | set(range(0, len(xs), 64))):
        P = orc.example_at_state(EXAMPLE_DIR, xs[b])
        h, Y, U = orc.solve(P)
        assert h == G["h"][b], (b, h, G["h"][b])
        d = np.frombuffer(hashlib.sha256(Y.tobytes() + U.tobytes()).digest()[:8], np.uint64)[0]
        assert d == G["digest"][b], f"state {b}: (Y*, U*) differ from the reference"


def test_horizon_population_sample_matches_reference_golden(orc):
    """The restatement pinned on the bench's horizon leg population
    (tests/golden/horizon_states.npz, made by the reference itself: its setup
    of each stacked problem and its converge solve capped at 999 updates): the
    problems kept in full (the capped H = 2 one and every h = 314 among them)
    and every 512th give the reference's h and (Y*, U*) digest."""
    import sys

    from conftest import ROOT

    sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
    from pqp_amd import perturbed_states

    G = np.load(GOLDEN / "horizon_states.npz")
    E = orc.load_example(EXAMPLE_DIR)
    cap = int(G["cap"])
    for H in G["H"].tolist():
        hg = G[f"h{H}"].astype(np.int64)
        xs = perturbed_states(E["x"], len(hg) * H, seed=7).reshape(len(hg), H, -1)
        assert hashlib.sha256(xs.tobytes()).digest() == G[f"xs_sha256_{H}"].tobytes()
        for b in sorted(set(G[f"kept{H}"].tolist()) | set(range(0, len(hg), 512))):
            h, Y, U = orc.solve(orc.horizon_problem(EXAMPLE_DIR, xs[b]), max_updates=cap)
            assert h == hg[b], (H, b, h, hg[b])
            d = np.frombuffer(hashlib.sha256(Y.tobytes() + U.tobytes()).digest()[:8], np.uint64)[0]
            assert d == G[f"digest{H}"][b], f"H={H} problem {b}: (Y*, U*) differ from the reference"
