"""GPU parity of converge mode as ONE persistent pipelined launch
(pqp_converge.hip): the update and the stages of terminate() run as
concurrent roles, terminate(Y_u) beside the update to Y_{u+1}, exchanging
tagged granules.  Bar: the reference's h, and Y*, U*, Jp, Jd bit for bit
(golden fixtures from the compiled reference, and the oracle); the same
results as the graph-replayed launch chain of pqp_wide.hip."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import CAP, GOLDEN, assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture
def persistent(gpu_lib):
    """Every converge-mode solve over the persistent launch (LDS-sized
    problems too)."""
    L = gpu_lib.lib()
    prev_min = L.pqp_tune_wide_min_n(0)
    prev_off = L.pqp_tune_converge_persist(0)
    yield L
    L.pqp_tune_wide_min_n(prev_min)
    L.pqp_tune_converge_persist(prev_off)
    L.pqp_tune_converge_chunk(0)


def _same(r, h, Y, U, what):
    assert r["h"] == abs(h) and r["converged"] == (h > 0), (what, r["h"], h)
    assert_bitwise(r["Y"], Y, f"{what} Y")
    assert_bitwise(r["U"], U, f"{what} U")


def test_persistent_bundled_converge(gpu_lib, golden_bundled, persistent):
    """The bundled example (n_dual 28, M 7): h = 313, Y*, U*, Jp, Jd of the
    compiled reference."""
    g = golden_bundled
    P = {k: np.ascontiguousarray(g[k], dtype=np.float32) for k in
         ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
    P.update(N=int(g["N"]), M=int(g["M"]))
    r = gpu_lib.solve_dual(P, max_updates=CAP)
    assert r["converged"] and r["h"] == 313
    assert_bitwise(r["Y"], g["Ystar"], "Y*")
    assert_bitwise(r["U"], g["Ustar"], "U*")
    assert np.float32(r["Jp"]) == g["iter_Jp"][-1] and np.float32(r["Jd"]) == g["iter_Jd"][-1]


def test_persistent_converge_fixtures(gpu_lib, golden_converge, orc, persistent):
    """The converging synthetic cases (h from 3 to several thousand) against
    the reference's h, Y* and U*."""
    cases, Ys, Us = golden_converge["cases"], golden_converge["Y"], golden_converge["U"]
    yo = uo = 0
    for (N, M, seed, h_ref) in cases:
        N, M = int(N), int(M)
        P = orc.synth_problem(int(seed), 0, N, M)
        r = gpu_lib.solve_dual(P, max_updates=CAP)
        assert r["converged"] and r["h"] == int(h_ref), (N, M, seed, r["h"])
        assert_bitwise(r["Y"], Ys[yo:yo + N], f"Y {N}/{M}/{seed}")
        assert_bitwise(r["U"], Us[uo:uo + M], f"U {N}/{M}/{seed}")
        yo += N
        uo += M


@pytest.mark.parametrize("chunk", [1, 2, 3, 8, 9, 100])
def test_persistent_chunked_launches(gpu_lib, golden_converge, orc, persistent, chunk):
    """Launches that decide only `chunk` iterates each, chained through the
    iterate they leave behind (chunks shorter than, equal to and longer than
    the ring depth of 8): same h, Y*, U*, Jp, Jd as one launch."""
    persistent.pqp_tune_converge_chunk(chunk)
    N, M, seed, h_ref = (int(v) for v in golden_converge["cases"][1])
    P = orc.synth_problem(seed, 0, N, M)
    r = gpu_lib.solve_dual(P, max_updates=CAP)
    persistent.pqp_tune_converge_chunk(0)
    one = gpu_lib.solve_dual(P, max_updates=CAP)
    assert r["h"] == one["h"] == h_ref and r["converged"]
    assert_bitwise(r["Y"], one["Y"], "Y")
    assert_bitwise(r["U"], one["U"], "U")
    assert np.float32(r["Jp"]) == np.float32(one["Jp"]) and np.float32(r["Jd"]) == np.float32(one["Jd"])


@pytest.mark.parametrize("N,M,cap", [(1, 1, 5), (28, 7, 0), (33, 16, 9), (97, 40, 12), (100, 160, 10),
                                     (383, 191, 6), (385, 200, 7), (513, 512, 5), (1024, 512, 25),
                                     (1024, 1024, 4), (640, 1024, 3)])
def test_persistent_capped_vs_oracle(gpu_lib, orc, persistent, N, M, cap):
    """Ragged sizes around the 32-column workgroups and the wave slices (M > N
    too), capped: h = cap + 1 (or the reference's h when it stops first), Y
    and U bit-identical to the oracle; cap 0 runs to convergence."""
    P = orc.synth_problem(7, N % 5, N, M)
    c = cap if cap else CAP
    r = gpu_lib.solve_dual(P, max_updates=c)
    h, Y, U = orc.solve(P, max_updates=c)
    _same(r, h, Y, U, f"N={N} M={M}")


def test_persistent_matches_graph_chain(gpu_lib, orc, persistent):
    """The persistent launch and the graph-replayed chain (pqp_wide.hip) on a
    capped n_dual = 1024 problem: same h, Y, U, Jp, Jd."""
    N, M, cap = 1024, 512, 40
    P = orc.synth_problem(3, 1, N, M)
    with gpu_lib.Problem(P) as prob:
        a = prob.solve(max_updates=cap)
        persistent.pqp_tune_converge_persist(1)
        b = prob.solve(max_updates=cap)
        persistent.pqp_tune_converge_persist(0)
        c = prob.solve(max_updates=cap)  # the persistent launch again on the same handle
    for r in (b, c):
        assert r["h"] == a["h"] == cap + 1
        assert_bitwise(r["Y"], a["Y"], "Y")
        assert_bitwise(r["U"], a["U"], "U")
        same = lambda x, y: (np.isnan(x) and np.isnan(y)) or np.float32(x) == np.float32(y)
        assert same(r["Jp"], a["Jp"]) and same(r["Jd"], a["Jd"])


def test_persistent_testfile_vs_oracle(gpu_lib, orc, tmp_path):
    """testing/ test2.txt (n_dual 400, M 100) on the default routing, which
    sends it to the persistent launch: the reference's h = 3, Y, U."""
    from test_gpu_wide import _testing_file

    P = gpu_lib.testfile_problem(_testing_file("test2.txt", tmp_path))
    r = gpu_lib.solve_dual(P, max_updates=CAP)
    h, Y, U = orc.solve(P, max_updates=CAP)
    _same(r, h, Y, U, "test2")


def _terminate_costs(orc, P, Y):
    """(flag, Jp, Jd) of the reference's terminate() on iterate Y (oracle)."""
    flag, _, Jp, Jd = orc.terminate(Y, P["Qd"], P["Fd"], P["Md"], P["Qp"], P["Qp_inv"], P["Fp"], P["Mp"], P["Gp"],
                                    P["Kp"], P["N"], P["M"])
    return flag, Jp, Jd


# caps of both parities: DEC sums the N-long dots of even and odd iterates on
# different waves (pqp_converge.hip)
@pytest.mark.parametrize("N,M,cap", [(100, 50, 20), (100, 100, 21), (385, 192, 30), (385, 385, 31),
                                     (1024, 512, 40), (1024, 512, 39), (1024, 1024, 22)])
def test_persistent_feasible_iterates_vs_oracle(gpu_lib, orc, persistent, N, M, cap):
    """every iterate feasible (Kp = 1e30 seen by checkFeas only;
    Fd keeps the generator's Kp), so terminate() runs all of computeCost on
    every iterate (PQP_CPU.c:648-666, :679-684): DEC's four dots, the M-long
    ones included.  h, Y, U bit for bit, and the last terminate()'s Jp, Jd."""
    P = orc.synth_problem(8, N % 3, N, M)
    P["Kp"] = np.full(N, 1e30, np.float32)
    r = gpu_lib.solve_dual(P, max_updates=cap)
    assert gpu_lib.lib().pqp_tune_last_path(None) == 3, "not the persistent converge launch"
    h, Y, U = orc.solve(P, max_updates=cap)
    _same(r, h, Y, U, f"feasible N={N} M={M}")
    flag, Jp, Jd = _terminate_costs(orc, P, Y)
    assert flag == 0 and np.isfinite(Jp) and np.isfinite(Jd)
    assert np.float32(r["Jp"]) == np.float32(Jp), (r["Jp"], Jp)
    assert np.float32(r["Jd"]) == np.float32(Jd), (r["Jd"], Jd)


@pytest.mark.parametrize("chunk", [0, 50, 7])
@pytest.mark.parametrize("k", [9, 36])
def test_persistent_large_problem_stops_like_reference(gpu_lib, golden_bundled, persistent, chunk, k):
    """The bundled example as k diagonal blocks (n_dual 252 / 1008, every
    iterate feasible) STOPS under the exact-float test at the reference's
    h = 313 (tests/golden/blocks.npz, made by oracle/_ref): one launch, and
    launches of 50 / 7 decided iterates, so the stop lands inside a chained
    launch.  Y*, U*, Jp, Jd bit for bit."""
    from oracle import block_diag_problem

    g = np.load(GOLDEN / "blocks.npz")
    P = {kk: np.ascontiguousarray(golden_bundled[kk], dtype=np.float32) for kk in
         ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
    P.update(N=int(golden_bundled["N"]), M=int(golden_bundled["M"]))
    Q = block_diag_problem(P, k)
    persistent.pqp_tune_converge_chunk(chunk)
    r = gpu_lib.solve_dual(Q, max_updates=CAP)
    assert gpu_lib.lib().pqp_tune_last_path(None) == 3, "not the persistent converge launch"
    assert r["converged"] and r["h"] == int(g[f"h{k}"]) == 313
    assert_bitwise(r["Y"], g[f"Y{k}"], "Y*")
    assert_bitwise(r["U"], g[f"U{k}"], "U*")
    assert np.float32(r["Jp"]) == g[f"Jp{k}"] and np.float32(r["Jd"]) == g[f"Jd{k}"]


@pytest.mark.parametrize("chunk", [5, 8])
def test_persistent_feasible_chunked(gpu_lib, orc, persistent, chunk):
    """Feasible iterates at n_dual 1024 across chained launches of `chunk`
    decided iterates: same h, Y, U, Jp, Jd as the oracle."""
    N, M, cap = 1024, 512, 23
    P = orc.synth_problem(8, 2, N, M)
    P["Kp"] = np.full(N, 1e30, np.float32)
    persistent.pqp_tune_converge_chunk(chunk)
    r = gpu_lib.solve_dual(P, max_updates=cap)
    h, Y, U = orc.solve(P, max_updates=cap)
    _same(r, h, Y, U, f"feasible chunk={chunk}")
    _, Jp, Jd = _terminate_costs(orc, P, Y)
    assert np.float32(r["Jp"]) == np.float32(Jp) and np.float32(r["Jd"]) == np.float32(Jd)


@pytest.mark.parametrize("xcds", [7, 8])
def test_persistent_converge_packed_on_fewer_xcds(gpu_lib, golden_converge, orc, persistent, xcds):
    """converge_xcds: the roles' workgroups packed onto 7 XCDs or spread over
    all 8 (the default packs them onto 6, which every other test takes; the
    rest of a padded grid leaves at once) -- the reference's h, Y*, U* on the
    converging fixtures, and a capped n_dual 1024 solve equal to the default
    launch's."""
    old = gpu_lib.tune("converge_xcds", xcds)
    try:
        cases, Ys, Us = golden_converge["cases"], golden_converge["Y"], golden_converge["U"]
        yo = uo = 0
        for (N, M, seed, h_ref) in cases:
            N, M = int(N), int(M)
            P = orc.synth_problem(int(seed), 0, N, M)
            r = gpu_lib.solve_dual(P, max_updates=CAP)
            assert r["converged"] and r["h"] == int(h_ref), (N, M, seed, r["h"])
            assert_bitwise(r["Y"], Ys[yo:yo + N], f"Y {N}/{M}/{seed} on {xcds} XCDs")
            assert_bitwise(r["U"], Us[uo:uo + M], f"U {N}/{M}/{seed} on {xcds} XCDs")
            yo += N
            uo += M
        P = orc.synth_problem(3, 0, 1024, 512)
        packed = gpu_lib.solve_dual(P, max_updates=40)
        assert gpu_lib.tune_get("last_path") == 3
    finally:
        gpu_lib.tune("converge_xcds", old)
    spread = gpu_lib.solve_dual(P, max_updates=40)
    assert packed["h"] == spread["h"] == 41
    assert_bitwise(packed["Y"], spread["Y"], "n_dual 1024 Y, this placement vs the default")
    assert_bitwise(packed["U"], spread["U"], "n_dual 1024 U, this placement vs the default")
