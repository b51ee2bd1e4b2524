"""GPU parity: the HIP path (through the C ABI) against the reference's golden
fixtures and the oracle.  Bar: bit-exact fp32 (the north star's 1e-6 relative
tolerance on y* is met with zero error), iterations-to-convergence identical.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import CAP, EXAMPLE_DIR, GOLDEN, assert_bitwise

pytestmark = pytest.mark.gpu

KEYS = ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")


def bundled_problem(g):
    P = {k: np.ascontiguousarray(g[k], dtype=np.float32) for k in KEYS}
    P.update(N=int(g["N"]), M=int(g["M"]))
    return P


# ---------------------------------------------------------------------------
# bundled example (configs 1/2)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("solver", ["quintet", "wave_pipelined", "wave_plain", "tiny"])
def test_bundled_converge_bit_exact(gpu_lib, golden_bundled, solver):
    """One problem in converge mode: k_solve_quintet (default), and with the
    tiny_old knob the round-4 kernels -- the one-wave solver (pipelined and
    plain forms) and the four-wave k_solve_tiny."""
    g = golden_bundled
    L = gpu_lib.lib()
    old_t = gpu_lib.tune("tiny_old", 0 if solver == "quintet" else 1)
    old_b = L.pqp_tune_wave_min_b(1 << 30 if solver == "tiny" else 1)
    old_p = L.pqp_tune_wave_pipe_max_b(0 if solver == "wave_plain" else 1 << 30)
    try:
        r = gpu_lib.solve_dual(bundled_problem(g), max_updates=CAP)
    finally:
        L.pqp_tune_wave_min_b(old_b)
        L.pqp_tune_wave_pipe_max_b(old_p)
        gpu_lib.tune("tiny_old", old_t)
    assert r["converged"]
    assert r["h"] == int(g["h"]) == 313, (r["h"], r["Jp"], r["Jd"], gpu_lib.tune_get("last_path"))
    assert_bitwise(r["Y"], g["Ystar"], "Y*")
    assert_bitwise(r["U"], g["Ustar"], "U from the final terminate()")
    assert np.float32(r["Jp"]) == g["iter_Jp"][-1] and np.float32(r["Jd"]) == g["iter_Jd"][-1]
    assert not np.array_equal(r["Y"].view(np.uint32), g["Ystar_fma_contracted"].view(np.uint32))


def test_bundled_fixed_1000_bit_exact(gpu_lib, golden_bundled):
    g = golden_bundled
    r = gpu_lib.solve_dual(bundled_problem(g), mode=gpu_lib.MODE_FIXED, num_iter=1000)
    assert r["h"] == 1000
    assert_bitwise(r["Y"], g["Y_fixed999"], "fixed-999 Y")


@pytest.mark.parametrize("k", [1, 2, 10, 100, 312])
def test_bundled_fixed_k_updates(gpu_lib, golden_bundled, k):
    g = golden_bundled
    r = gpu_lib.solve_dual(bundled_problem(g), mode=gpu_lib.MODE_FIXED, num_iter=k)
    want = g["Ystar"] if k == 313 else (g[f"Y_h{k}"])
    assert_bitwise(r["Y"], want, f"Y after {k - 1} updates")


def test_problem_handle_repeated_solves(gpu_lib, golden_bundled):
    g = golden_bundled
    with gpu_lib.Problem(bundled_problem(g)) as prob:
        for _ in range(3):
            r = prob.solve(max_updates=CAP)
            assert r["h"] == 313
            assert_bitwise(r["Y"], g["Ystar"], "Y*")
            f = prob.solve(gpu_lib.MODE_FIXED, num_iter=1000)
            assert_bitwise(f["Y"], g["Y_fixed999"], "fixed-999 Y")


def test_lds_staged_solver_on_bundled(gpu_lib, golden_bundled):
    """Route the bundled problem through k_solve_small (instead of the
    register-resident k_solve_tiny): same bits, same h."""
    L = gpu_lib.lib()
    old = L.pqp_tune_set_variant(0x100)
    try:
        r = gpu_lib.solve_dual(bundled_problem(golden_bundled), max_updates=CAP)
        f = gpu_lib.solve_dual(bundled_problem(golden_bundled), mode=gpu_lib.MODE_FIXED, num_iter=1000)
    finally:
        L.pqp_tune_set_variant(old)
    assert r["h"] == 313
    assert_bitwise(r["Y"], golden_bundled["Ystar"], "Y*")
    assert_bitwise(r["U"], golden_bundled["Ustar"], "U")
    assert_bitwise(f["Y"], golden_bundled["Y_fixed999"], "fixed-999")


@pytest.mark.parametrize("N,M", [(5, 3), (16, 16), (17, 9), (32, 32), (40, 20), (64, 32), (97, 13), (100, 50),
                                 (128, 64), (300, 150)])
def test_single_problem_paths(gpu_lib, orc, N, M):
    """N, M <= 32: register-resident k_solve_tiny (16- and 32-wide builds);
    N <= ~98: LDS-staged k_solve_small (several lane passes per role from
    N > 32); larger problems: k_solve_single."""
    P = orc.synth_problem(5, 3, N, M)
    with gpu_lib.Problem(P) as prob:
        r = prob.solve(gpu_lib.MODE_FIXED, num_iter=41)
        h, Y, _ = orc.solve(P, mode=1, num_iter=41)
        assert r["h"] == h == 41
        assert_bitwise(r["Y"], Y, f"fixed N={N}")
        c = prob.solve(max_updates=60)
    h2, Y2, U2 = orc.solve(P, max_updates=60)
    assert c["h"] == abs(h2)
    assert_bitwise(c["Y"], Y2, f"converge-capped N={N}")
    assert_bitwise(c["U"], U2, f"U N={N}")


@pytest.mark.parametrize("N", [99, 257, 1000])
def test_large_fixed_split_vs_single_workgroup(gpu_lib, orc, N):
    """Fixed mode of a large problem: the multi-workgroup split-matrix path
    (default) and the one-workgroup solver (tuning bit 0x200) give the same
    bits as the oracle."""
    M = N // 2
    P = orc.synth_problem(8, 1, N, M, with_qp=False)
    P.update(Qp=np.zeros(M * M, np.float32))
    _, Yr, _ = orc.solve(P, mode=1, num_iter=12)
    L = gpu_lib.lib()
    with gpu_lib.Problem(P) as prob:
        a = prob.solve(gpu_lib.MODE_FIXED, num_iter=12)
        old = L.pqp_tune_set_variant(0x200)
        try:
            b = prob.solve(gpu_lib.MODE_FIXED, num_iter=12)
        finally:
            L.pqp_tune_set_variant(old)
    assert a["h"] == b["h"] == 12
    assert_bitwise(a["Y"], Yr, "split path")
    assert_bitwise(b["Y"], Yr, "single-workgroup path")


def test_dropin_solveQuadraticDual_prints_h(gpu_lib, golden_bundled, capfd):
    g = golden_bundled
    P = bundled_problem(g)
    Y, U = np.zeros(P["N"], np.float32), np.zeros(P["M"], np.float32)
    gpu_lib.solveQuadraticDual(Y, P["Qd"], P["Fd"], P["Md"], U, P["Qp"], P["Qp_inv"], P["Fp"], P["Mp"], P["Gp"],
                               P["Kp"], P["N"], P["M"])
    out = capfd.readouterr().out
    assert "Printing number of iterations = 313\n" in out
    assert_bitwise(Y, g["Ystar"], "Y*")


def test_cli_stdout_matches_reference_byte_for_byte(gpu_lib):
    expected = (GOLDEN / "bundled_stdout.txt").read_text()
    assert gpu_lib.run_example(EXAMPLE_DIR) == expected


def test_pqp_cli_binary(tmp_path):
    import shutil
    import subprocess

    from conftest import ROOT

    (tmp_path / "example").mkdir()
    for f in EXAMPLE_DIR.glob("*.txt"):
        shutil.copy(f, tmp_path / "example" / f.name)
    cli = ROOT / "pqp-for-mpc_amd" / "bin" / "pqp_cli"
    out = subprocess.run([str(cli)], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout == (GOLDEN / "bundled_stdout.txt").read_text()


# ---------------------------------------------------------------------------
# drop-in helpers, one by one, vs the reference's values
# ---------------------------------------------------------------------------
def test_dropin_updateY2_split_matrices(gpu_lib, golden_bundled, orc):
    g = golden_bundled
    N = int(g["N"])
    qp, qn = orc.split_theta(g["Qd"], g["theta"], N)
    for a, b in ((1, 2), (100, None)):
        Y = np.ascontiguousarray(g[f"Y_h{a}"])
        out = np.zeros(N, np.float32)
        gpu_lib.updateY2(out, Y.copy(), qp, qn, g["Fd"].copy(), g["Fdp"].copy(), g["Fdn"].copy(), N)
        want = g[f"Y_h{b}"] if b else orc.update_split(Y, qp, qn, g["Fdp"], g["Fdn"], N)
        assert_bitwise(out, want, f"updateY2 from Y_h{a}")


def test_dropin_terminate(gpu_lib, golden_bundled):
    g = golden_bundled
    P = bundled_problem(g)
    for key, flag_ref in (("Y_h1", 0), ("Y_h312", 0), ("Ystar", 1)):
        U = np.zeros(P["M"], np.float32)
        flag = gpu_lib.terminate(np.ascontiguousarray(g[key]), P["Qd"], P["Fd"], P["Md"], U, P["Qp"], P["Qp_inv"],
                                 P["Fp"], P["Mp"], P["Gp"], P["Kp"], P["N"], P["M"])
        assert flag == flag_ref, key
    assert_bitwise(U, g["Ustar"], "U")


def test_dropin_setup_functions(gpu_lib, golden_bundled, orc):
    g = golden_bundled
    ex = orc.load_example(EXAMPLE_DIR)
    N, M = int(g["N"]), int(g["M"])
    Qp = np.zeros(M * M, np.float32)
    gpu_lib.Gauss_Jordan(ex["Qp_inv"].copy(), Qp, M)
    assert_bitwise(Qp, g["Qp"], "Gauss_Jordan")
    Fp = np.zeros(M, np.float32)
    gpu_lib.computeFp(Fp, ex["Fp1"], ex["Fp2"], ex["Fp3"], ex["D"], ex["x"])
    assert_bitwise(Fp, g["Fp"], "computeFp")
    Mp = np.zeros(1, np.float32)
    gpu_lib.computeMp(Mp, ex["Mp1"], ex["Mp2"], ex["Mp3"], ex["Mp4"], ex["Mp5"], ex["Mp6"], ex["D"], ex["x"])
    assert_bitwise(Mp, g["Mp"], "computeMp")
    Qd, Fd, Md = np.zeros(N * N, np.float32), np.zeros(N, np.float32), np.zeros(1, np.float32)
    gpu_lib.convertToDual(Qd, Fd, Md, g["Qp_inv"].copy(), g["Gp"].copy(), g["Kp"].copy(), g["Fp"].copy(),
                          g["Mp"].copy(), N, M)
    assert_bitwise(Qd, g["Qd"], "Qd")
    assert_bitwise(Fd, g["Fd"], "Fd")
    assert_bitwise(Md, g["Md"], "Md")
    th = np.zeros(N * N, np.float32)
    gpu_lib.computeTheta(th, g["Qd"].copy(), N)
    assert_bitwise(th.reshape(N, N).diagonal().copy(), g["theta"], "computeTheta")
    assert np.count_nonzero(th) == N
    U = np.zeros(M, np.float32)
    gpu_lib.computeUfromY(U, g["Ystar"].copy(), g["Fp"].copy(), g["Gp"].copy(), g["Qp_inv"].copy(), N, M)
    assert_bitwise(U, g["Ustar"], "computeUfromY")
    assert gpu_lib.checkFeas(U, g["Gp"].copy(), g["Kp"].copy(), N, M) == 1
    assert gpu_lib.checkFeas((U * 100).astype(np.float32), g["Gp"].copy(), g["Kp"].copy(), N, M) == 0
    assert np.float32(gpu_lib.computeCost(U, g["Qp"].copy(), g["Fp"].copy(), g["Mp"].copy(), M)) == g["Jp"]
    assert np.float32(gpu_lib.computeCost(g["Ystar"].copy(), g["Qd"].copy(), g["Fd"].copy(), g["Md"].copy(),
                                          N)) == g["Jd"]


def test_dropin_matrixMultiply_transposes(gpu_lib, orc):
    rng = np.random.default_rng(7)
    for (a, b, c) in [(1, 1, 1), (3, 7, 5), (17, 9, 1), (1, 33, 20), (64, 48, 40)]:
        for tA in (0, 1):
            for tB in (0, 1):
                A = rng.standard_normal(a * b).astype(np.float32)
                B = rng.standard_normal(b * c).astype(np.float32)
                out = np.zeros(a * c, np.float32)
                gpu_lib.matrixMultiply(out, A, tA, B, tB, a, b, c)
                assert_bitwise(out, orc.matmul(A, tA, B, tB, a, b, c), f"{a}x{b}x{c} t{tA}{tB}")


# ---------------------------------------------------------------------------
# synthetic problems: converge mode (iterations identical) and large duals
# ---------------------------------------------------------------------------
def test_synthetic_converge_cases(gpu_lib, golden_converge, orc):
    cases, Ys, Us = golden_converge["cases"], golden_converge["Y"], golden_converge["U"]
    yo = uo = 0
    for (N, M, seed, h_ref) in cases:
        N, M = int(N), int(M)
        P = orc.synth_problem(int(seed), 0, N, M)
        r = gpu_lib.solve_dual(P, max_updates=CAP)
        assert r["converged"] and r["h"] == int(h_ref), (N, M, seed, r["h"])
        assert_bitwise(r["Y"], Ys[yo:yo + N], f"Y {N}/{M}/{seed}")
        yo += N
        uo += M


def test_converge_cap_reports_not_converged(gpu_lib, orc):
    P = orc.synth_problem(2, 0, 16, 8)  # the reference does not converge on this one
    r = gpu_lib.solve_dual(P, max_updates=500)
    assert not r["converged"] and r["h"] == 501
    h, Y, _ = orc.solve(P, mode=1, num_iter=501)
    assert_bitwise(r["Y"], Y, "Y after 500 updates")


@pytest.mark.parametrize("tag", ["n1024_m512_s1_i0", "n1000_m500_s2_i7"])
def test_batch_generator_and_updates_match_reference(gpu_lib, golden_large, tag):
    N, M, seed, inst, ups = (int(v) for v in golden_large[f"{tag}_meta"])
    b = gpu_lib.Batch(1, N).generate(seed, inst0=inst, M=M)
    Qd = b.qd_rowmajor(0)
    assert hashlib.sha256(Qd.tobytes()).digest() == golden_large[f"{tag}_Qd_sha256"].tobytes()
    assert_bitwise(b.Fd[0, :N].cpu().numpy(), golden_large[f"{tag}_Fd"], "Fd")
    assert_bitwise(b.Md[:1].cpu().numpy(), golden_large[f"{tag}_Md"], "Md")
    assert_bitwise(b.theta[0, :N].cpu().numpy(), golden_large[f"{tag}_theta"], "theta")
    b.reset()
    for _ in range(ups):
        b.update()
    assert_bitwise(b.result()[0], golden_large[f"{tag}_Y"], "Y via batch_update")
    b.iterate(ups)
    assert_bitwise(b.result()[0], golden_large[f"{tag}_Y"], "Y via batch_iterate")


@pytest.mark.parametrize("N", [1, 3, 4, 28, 64, 255, 256, 257, 300, 1023, 1025, 2050])
def test_batch_kernels_vs_oracle_edge_sizes(gpu_lib, orc, N):
    """Ragged N (not multiples of 4 / 64 / 256 / 1024), several problems."""
    B, M, ups = 3, max(1, N // 2), 4
    b = gpu_lib.Batch(B, N).generate(seed=11, inst0=5, M=M)
    b.iterate(ups)
    it = b.result()
    b.reset()
    for _ in range(ups):
        b.update()
    up = b.result()
    for j in range(B):
        P = orc.synth_problem(11, 5 + j, N, M, with_qp=False)
        want = orc.iterate(P["Qd"], P["Fd"], N, ups)
        assert_bitwise(it[j], want, f"iterate N={N} problem {j}")
        assert_bitwise(up[j], want, f"update N={N} problem {j}")


def _iterate_kind(gpu_lib, b, ups, kind):
    prev = gpu_lib.tune("iterate_kind", kind)
    try:
        b.reset()
        b.iterate(ups)
        return b.result().copy()
    finally:
        gpu_lib.tune("iterate_kind", prev)


@pytest.mark.parametrize("N,B,ups", [(1024, 5, 23), (1024, 3, 1), (1024, 2, 2), (1024, 3, 3), (2048, 3, 11),
                                     (3072, 2, 4)])
def test_stream_kernels_vs_oracle_and_iterate(gpu_lib, orc, N, B, ups):
    """pqp_batch_iterate where N is a multiple of 1024 -- k_batch_resident
    (N = 1024: Qd's first blocks in LDS / L2 across the launch's iterations,
    incl. launches of 1, 2 and 3 updates, where the LDS copy is written and
    read once or not at all) and k_batch_stream: ragged batches, the first and
    last problem against the oracle and every problem bit for bit against
    k_batch_iterate (iterate_kind 1) and k_batch_stream (iterate_kind 2)."""
    M = N // 2
    b = gpu_lib.Batch(B, N).generate(seed=21, inst0=3, M=M)
    b.iterate(ups)
    first = b.result().copy()
    assert_bitwise(first, _iterate_kind(gpu_lib, b, ups, 1), f"default vs k_batch_iterate N={N}")
    assert_bitwise(first, _iterate_kind(gpu_lib, b, ups, 2), f"default vs k_batch_stream N={N}")
    assert_bitwise(first, _iterate_kind(gpu_lib, b, ups, 3), f"default vs k_batch_resident LDS + L2 N={N}")
    for j in (0, B - 1):
        P = orc.synth_problem(21, 3 + j, N, M, with_qp=False)
        assert_bitwise(first[j], orc.iterate(P["Qd"], P["Fd"], N, ups), f"N={N} problem {j}")


def test_resident_kernel_chained_launches(gpu_lib, orc):
    """Updates beyond one launch (pqp_batch_iterate splits runs into launches
    of 256): every launch starts from the previous one's Y and refills its LDS
    copy of Qd's first blocks."""
    N, B, ups = 1024, 2, 300
    b = gpu_lib.Batch(B, N).generate(seed=4, inst0=9, M=N // 2)
    b.iterate(ups)
    res = b.result().copy()
    assert_bitwise(res, _iterate_kind(gpu_lib, b, ups, 1), "resident vs k_batch_iterate, 300 updates")
    P = orc.synth_problem(4, 9, N, N // 2, with_qp=False)
    assert_bitwise(res[0], orc.iterate(P["Qd"], P["Fd"], N, ups), "300 updates vs oracle")


def test_batch_load_bundled_fixed_999(gpu_lib, golden_bundled):
    g = golden_bundled
    N = int(g["N"])
    b = gpu_lib.Batch(2, N).load(np.stack([g["Qd"], g["Qd"]]), np.stack([g["Fd"], g["Fd"]]))
    assert_bitwise(b.theta[0, :N].cpu().numpy(), g["theta"], "theta")
    b.iterate(999)
    assert_bitwise(b.result()[0], g["Y_fixed999"], "iterate 999")
    assert_bitwise(b.result()[1], g["Y_fixed999"], "iterate 999 (2nd copy)")


def test_batch_problems_are_independent(gpu_lib):
    """Problem inst0+j of a batch == the same problem generated alone."""
    N, B = 512, 16
    big = gpu_lib.Batch(B, N).generate(seed=3, inst0=100).iterate(7).result()
    for j in (0, 5, 15):
        one = gpu_lib.Batch(1, N).generate(seed=3, inst0=100 + j).iterate(7).result()[0]
        assert_bitwise(big[j], one, f"problem {j}")


def test_iterate_equals_repeated_update_large_batch(gpu_lib):
    N, B, ups = 1024, 96, 12
    b = gpu_lib.Batch(B, N).generate(seed=9)
    b.iterate(ups)
    a = b.result()
    b.reset()
    for _ in range(ups):
        b.update()
    assert_bitwise(b.result(), a, "iterate vs update")
    assert np.all(np.isfinite(a)) and np.all(a >= 0)


def test_full_size_batch_properties(gpu_lib, orc):
    """BASELINE config 4 (N=1024, B=4096, 16 GiB of Qd): sampled problems
    bit-exact against the oracle, all iterates finite and non-negative."""
    import torch

    N, B, ups = 1024, 4096, 3
    b = gpu_lib.Batch(B, N).generate(seed=1)
    b.iterate(ups)
    Y = b.result()
    assert np.all(np.isfinite(Y)) and np.all(Y >= 0)
    for j in (0, 1777, 4095):
        P = orc.synth_problem(1, j, N, N // 2, with_qp=False)
        assert_bitwise(Y[j], orc.iterate(P["Qd"], P["Fd"], N, ups), f"problem {j}")
    del b
    torch.cuda.empty_cache()


def test_batch_argument_validation(gpu_lib):
    import ctypes as C

    import torch

    L = gpu_lib.lib()
    q = torch.zeros(64, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = C.c_void_p(q.data_ptr())
    assert L.pqp_batch_update(1, 4, p, 3, 16, p, p, 4, p, p, s) == gpu_lib.PQP_ERR_ARG  # ldq < N
    assert "ldq" in gpu_lib.last_error()
    assert L.pqp_batch_update(1, 4, p, 4, 16, p, p, 4, p, p, s) == gpu_lib.PQP_ERR_ARG  # Y aliases Ynext
    assert L.pqp_batch_iterate(1, 4, p, 4, 16, p, p, 4, None, p, -1, s) == gpu_lib.PQP_ERR_ARG


def test_reference_main_linked_against_libpqp(tmp_path):
    """PQP_CPU.c's own main() (oracle/_ref, built from /root/reference) with
    libpqp.so first in the symbol search order: the reference driver calls the
    GPU drop-ins and must print exactly what the reference prints."""
    import shutil
    import subprocess

    from conftest import ROOT

    exe = ROOT / "oracle" / "_ref" / "ref_main_on_libpqp"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_main_on_libpqp not built (needs /root/reference at build time)")
    (tmp_path / "example").mkdir()
    for f in EXAMPLE_DIR.glob("*.txt"):
        shutil.copy(f, tmp_path / "example" / f.name)
    out = subprocess.run([str(exe)], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout == (GOLDEN / "bundled_stdout.txt").read_text()


# ---------------------------------------------------------------------------
# batched small problems (one workgroup per problem): F1 setup + F2 solve
# ---------------------------------------------------------------------------
def test_problem_batch_replicated_bundled(gpu_lib, golden_bundled):
    g = golden_bundled
    pb = gpu_lib.ProblemBatch.replicate(bundled_problem(g), 300)
    pb.solve(max_updates=CAP)
    h = pb.h.cpu().numpy()
    assert np.all(h == 313) and np.all(pb.status.cpu().numpy() == 1)
    Y, U = pb.Y.cpu().numpy(), pb.U.cpu().numpy()
    for b in (0, 1, 150, 299):
        assert_bitwise(Y[b], g["Ystar"], f"Y* problem {b}")
        assert_bitwise(U[b], g["Ustar"], f"U problem {b}")
    pb.solve(gpu_lib.MODE_FIXED, num_iter=1000)
    assert np.all(pb.h.cpu().numpy() == 1000)
    assert_bitwise(pb.Y.cpu().numpy()[299], g["Y_fixed999"], "fixed-999")


def test_batched_setup_from_primal(gpu_lib, golden_bundled):
    """Batched Gauss_Jordan + convertToDual on device reproduce the reference's
    dual of the bundled problem."""
    g = golden_bundled
    pb = gpu_lib.ProblemBatch.replicate({k: g[k] for k in ("Qp_inv", "Gp", "Kp", "Fp", "Mp")} |
                                        dict(N=int(g["N"]), M=int(g["M"])), 5)
    pb.gauss_jordan().convert_to_dual()
    for name in ("Qd", "Fd", "Qp"):
        assert_bitwise(getattr(pb, name).cpu().numpy()[4], g[name], name)
    assert_bitwise(pb.Md.cpu().numpy()[4:5], g["Md"], "Md")


def _oracle_example_at_state(orc, x):
    """main()'s setup (PQP_CPU.c:988-994) with the state x replaced."""
    return orc.example_at_state(EXAMPLE_DIR, x)


def test_mpc_batch_of_states_vs_oracle(gpu_lib, orc):
    """The bundled plant at 64 different states x: per-problem computeFp /
    computeMp / convertToDual / solve on the GPU == the oracle, including h."""
    E = orc.load_example(EXAMPLE_DIR)
    rng = np.random.default_rng(5)
    xs = (E["x"][None, :] * (1.0 + 0.05 * rng.standard_normal((64, E["ns"])))).astype(np.float32)
    pb = gpu_lib.mpc_batch(EXAMPLE_DIR, xs)
    pb.solve(max_updates=CAP)
    h, st = pb.h.cpu().numpy(), pb.status.cpu().numpy()
    Y, Fp, Mp = pb.Y.cpu().numpy(), pb.Fp.cpu().numpy(), pb.Mp.cpu().numpy()
    for b in (0, 7, 33, 63):
        P = _oracle_example_at_state(orc, xs[b])
        assert_bitwise(Fp[b], P["Fp"], f"Fp {b}")
        assert_bitwise(Mp[b:b + 1], P["Mp"], f"Mp {b}")
        hr, Yr, _ = orc.solve(P, max_updates=CAP)
        assert st[b] == (1 if hr > 0 else 2) and h[b] == abs(hr), (b, h[b], hr)
        assert_bitwise(Y[b], Yr, f"Y {b}")


def test_mpc_population_vs_reference(gpu_lib):
    """the bench's whole mpc_batch population -- the bundled plant
    at 16384 perturbed states (pqp_amd.perturbed_states, seed 5) -- solved on
    the GPU (setup and converge mode on device, as the bench leg runs it)
    against the REFERENCE's own solve of every state (tests/golden/
    mpc_states.npz, made by make_golden.py from oracle/_ref): every h
    (16381 x 313 and 3 x 314) and a digest of every (Y*, U*)
    (PQP_CPU.c:694-750; the stop test at :718, :683-684)."""
    import hashlib

    G = np.load(GOLDEN / "mpc_states.npz")
    E = gpu_lib.read_example(EXAMPLE_DIR)
    xs = gpu_lib.perturbed_states(E["x"], len(G["h"]), seed=5)
    assert hashlib.sha256(xs.tobytes()).digest() == G["xs_sha256"].tobytes(), "the state generator moved"
    pb = gpu_lib.mpc_batch(EXAMPLE_DIR, xs)
    pb.solve(max_updates=CAP)
    h, st = pb.h.cpu().numpy(), pb.status.cpu().numpy()
    Y, U = pb.Y.cpu().numpy(), pb.U.cpu().numpy()
    for j, b in enumerate(G["kept"]):  # readable first failures: the h = 314 states and a few more, in full
        assert h[b] == G["h"][b], (b, h[b], G["h"][b])
        assert_bitwise(Y[b], G["kept_Y"][j], f"Y* of state {b}")
        assert_bitwise(U[b], G["kept_U"][j], f"U* of state {b}")
    bad_h = np.nonzero(h != G["h"].astype(np.int64))[0]
    assert bad_h.size == 0, f"{bad_h.size} states stop at another h than the reference; first {bad_h[:8]}"
    assert (st == 1).all()
    dig = np.array([np.frombuffer(hashlib.sha256(Y[b].tobytes() + U[b].tobytes()).digest()[:8], np.uint64)[0]
                    for b in range(len(h))], np.uint64)
    bad = np.nonzero(dig != G["digest"])[0]
    assert bad.size == 0, f"{bad.size} of {len(h)} states differ from the reference in Y* or U*; first {bad[:8]}"


def test_batched_synthetic_converge_groups(gpu_lib, golden_converge, orc):
    cases, Ys = golden_converge["cases"], golden_converge["Y"]
    offs = np.concatenate([[0], np.cumsum(cases[:, 0])])
    groups = {}
    for idx, (N, M, seed, h) in enumerate(cases):
        groups.setdefault((int(N), int(M)), []).append((idx, int(seed), int(h)))
    for (N, M), items in groups.items():
        pb = gpu_lib.ProblemBatch(len(items), N, M)
        for j, (idx, seed, _) in enumerate(items):
            P = orc.synth_problem(seed, 0, N, M)
            for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp"):
                getattr(pb, k)[j] = pb.torch.as_tensor(P[k].reshape(-1), device=pb.device)
        pb.solve(max_updates=CAP)
        for j, (idx, seed, h) in enumerate(items):
            assert int(pb.h[j]) == h, (N, M, seed)
            assert_bitwise(pb.Y[j].cpu().numpy(), Ys[offs[idx]:offs[idx] + N], f"{N}/{M}/{seed}")


@pytest.mark.parametrize("N,M", [(48, 24), (120, 60)])
def test_batched_larger_paths(gpu_lib, orc, N, M):
    """LDS-staged (N=48) and global-memory (N=120) batched paths, fixed and
    capped-converge modes, vs the oracle."""
    B = 6
    pb = gpu_lib.ProblemBatch(B, N, M)
    Ps = [orc.synth_problem(21, j, N, M) for j in range(B)]
    for j, P in enumerate(Ps):
        for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp"):
            getattr(pb, k)[j] = pb.torch.as_tensor(P[k].reshape(-1), device=pb.device)
    pb.solve(gpu_lib.MODE_FIXED, num_iter=30)
    for j in (0, B - 1):
        _, Yr, _ = orc.solve(Ps[j], mode=1, num_iter=30)
        assert_bitwise(pb.Y[j].cpu().numpy(), Yr, f"fixed {j}")
    pb.solve(max_updates=40)
    for j in (0, B - 1):
        hr, Yr, Ur = orc.solve(Ps[j], max_updates=40)
        assert int(pb.h[j]) == abs(hr)
        assert_bitwise(pb.Y[j].cpu().numpy(), Yr, f"capped {j}")
        assert_bitwise(pb.U[j].cpu().numpy(), Ur, f"U {j}")


# ---------------------------------------------------------------------------
# testing/ sample file (F3): reader -> GPU setup -> GPU iterations
# ---------------------------------------------------------------------------
def test_testfile_problem_vs_reference(gpu_lib, orc):
    g = dict(np.load(GOLDEN / "testing_test2.npz"))
    P = gpu_lib.testfile_problem(GOLDEN / "testing" / "test2.txt")
    N, M = P["N"], P["M"]
    assert hashlib.sha256(P["Qd"].tobytes()).digest() == g["Qd_sha256"].tobytes()
    for k in ("Fd", "Md", "Qp"):
        assert_bitwise(P[k], g[k], k)
    with gpu_lib.Problem(P) as prob:
        r = prob.solve(gpu_lib.MODE_FIXED, num_iter=21)
        assert_bitwise(r["Y"], g["Y20"], "Y after 20 updates (solver)")
        c = prob.solve(max_updates=150)
    b = gpu_lib.Batch(1, N).load(P["Qd"][None, :], P["Fd"][None, :])
    assert_bitwise(b.theta[0, :N].cpu().numpy(), g["theta"], "theta")
    assert_bitwise(b.iterate(20).result()[0], g["Y20"], "Y after 20 updates (batched kernel)")
    hr, Yr, Ur = orc.solve(P, max_updates=150)
    assert c["h"] == abs(hr)
    assert_bitwise(c["Y"], Yr, "converge-capped Y")
    assert_bitwise(c["U"], Ur, "converge-capped U")


# ---------------------------------------------------------------------------
# non-finite and signed-zero propagation: the lean form must match the
# reference's literal (max(0,+-q)+0.0f)*y arithmetic bit for bit
# ---------------------------------------------------------------------------
def _same_bits_or_both_nan(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(nan | (a.view(np.uint32) == b.view(np.uint32))))


@pytest.mark.parametrize("N", [7, 300, 1024, 1030, 2048])
def test_update_special_values_vs_oracle(gpu_lib, orc, N):
    rng = np.random.default_rng(N)
    Qd = rng.standard_normal((N, N)).astype(np.float32)
    Qd[rng.random((N, N)) < 0.1] = 0.0
    Qd[rng.random((N, N)) < 0.05] = -0.0
    Qd[rng.random((N, N)) < 0.002] = np.nan
    Qd = Qd.reshape(-1)
    Fd = rng.standard_normal(N).astype(np.float32)
    Fd[::7] = -0.0
    th = orc.theta(Qd, N)
    for trial in range(3):
        Y = (rng.random(N) * 100).astype(np.float32)
        if trial >= 1:
            Y[rng.integers(0, N, 3)] = np.inf
            Y[rng.integers(0, N, 2)] = 0.0
        if trial == 2:
            Y[rng.integers(0, N, 2)] = np.nan
        want = orc.update(Y, Qd, th, Fd, N)
        got = gpu_lib.update(Qd, th, Fd, Y, N)  # k_batch_update (lean + literal window)
        assert _same_bits_or_both_nan(got, want), f"N={N} trial={trial}"
        b = gpu_lib.Batch(1, N).load(Qd[None, :], Fd[None, :])
        b.Y[0, :N] = b.torch.as_tensor(Y, device=b.device)
        b.iterate(1, from_start=False)
        assert _same_bits_or_both_nan(b.result()[0], want), f"iterate N={N} trial={trial}"


def test_pqp_update_host_vs_golden(gpu_lib, golden_bundled):
    g = golden_bundled
    N = int(g["N"])
    Y = g["Y_h1"]
    for h in range(1, 10):
        Y = gpu_lib.update(g["Qd"], g["theta"], g["Fd"], Y, N)
    assert_bitwise(Y, g["Y_h10"], "9 updates via pqp_update_host")


def test_oneshot_tiny_problems_back_to_back(gpu_lib, orc, golden_bundled):
    """pqp_solve_dual on tiny problems re-fills one cached handle: solves of
    different problems and sizes in a row (growing and shrinking N and M)
    each give the reference's h, Y and U."""
    g = golden_bundled
    bundled = {k: np.ascontiguousarray(g[k], dtype=np.float32) for k in
               ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
    bundled.update(N=int(g["N"]), M=int(g["M"]))
    cases = [bundled, orc.synth_problem(3, 0, 8, 4), orc.synth_problem(4, 1, 32, 16), bundled,
             orc.synth_problem(5, 2, 16, 8)]
    for j, P in enumerate(cases):
        for mode in (gpu_lib.MODE_CONVERGE, gpu_lib.MODE_FIXED):
            r = gpu_lib.solve_dual(P, mode=mode, num_iter=50, max_updates=3000)
            if mode == gpu_lib.MODE_CONVERGE:
                h, Y, U = orc.solve(P, max_updates=3000)
                assert r["h"] == abs(h), (j, r["h"], h)
                assert_bitwise(r["U"], U, f"case {j} U")
            else:
                Y = orc.iterate(P["Qd"], P["Fd"], int(P["N"]), 49)
                assert r["h"] == 50
            assert_bitwise(r["Y"], Y, f"case {j} mode {mode} Y")
