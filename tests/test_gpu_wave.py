"""GPU parity of the one-wave converge-mode solver (k_solve_wave): many
N, M <= 32 problems per launch, terminate()'s mat-vecs packed beside the
update's.  Forced on for every batch size here (pqp_tune_wave_min_b(1)); bar:
bit-exact Y, U and identical h / status against the oracle (PQP_CPU.c
restated) and against the four-wave k_solve_tiny."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import CAP, EXAMPLE_DIR, assert_bitwise

pytestmark = pytest.mark.gpu

KEYS = ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")


@pytest.fixture(params=[1 << 30, 0], ids=["pipelined", "plain"])
def wave_on(gpu_lib, request):
    """k_solve_wave for every batch size, in its software-pipelined form and
    in its plain form."""
    L = gpu_lib.lib()
    old = L.pqp_tune_wave_min_b(1)
    old_pipe = L.pqp_tune_wave_pipe_max_b(request.param)
    yield
    L.pqp_tune_wave_min_b(old)
    L.pqp_tune_wave_pipe_max_b(old_pipe)


def _batch_of(gpu_lib, probs, N, M):
    pb = gpu_lib.ProblemBatch(len(probs), N, M)
    for j, P in enumerate(probs):
        for k in KEYS:
            getattr(pb, k)[j] = pb.torch.as_tensor(np.asarray(P[k], np.float32).reshape(-1), device=pb.device)
    return pb


@pytest.mark.parametrize("N,M", [(1, 1), (5, 3), (8, 8), (9, 2), (16, 16), (17, 9), (24, 12), (28, 7), (29, 30),
                                 (32, 8), (32, 32)])
def test_wave_solver_vs_oracle(gpu_lib, orc, wave_on, N, M):
    probs = [orc.synth_problem(11, j, N, M) for j in range(3)]
    pb = _batch_of(gpu_lib, probs, N, M)
    cap = 300
    pb.solve(max_updates=cap)
    for j, P in enumerate(probs):
        h, Y, U = orc.solve(P, max_updates=cap)
        assert int(pb.h[j]) == abs(h), (N, M, j)
        assert int(pb.status[j]) == (1 if h > 0 else 2)
        assert_bitwise(pb.Y[j].cpu().numpy(), Y, f"Y N={N} M={M} j={j}")
        assert_bitwise(pb.U[j].cpu().numpy(), U, f"U N={N} M={M} j={j}")


def test_wave_converge_fixtures(gpu_lib, golden_converge, orc, wave_on):
    cases, Ys = golden_converge["cases"], golden_converge["Y"]
    offs = np.concatenate([[0], np.cumsum(cases[:, 0])])
    done = 0
    for idx, (N, M, seed, h) in enumerate(cases):
        N, M = int(N), int(M)
        if N > 32 or M > 32:
            continue
        pb = _batch_of(gpu_lib, [orc.synth_problem(int(seed), 0, N, M)], N, M)
        pb.solve(max_updates=CAP)
        assert int(pb.h[0]) == int(h) and int(pb.status[0]) == 1, (N, M, seed)
        assert_bitwise(pb.Y[0].cpu().numpy(), Ys[offs[idx]:offs[idx] + N], f"{N}/{M}/{seed}")
        done += 1
    assert done >= 2


def test_wave_mpc_states_vs_tiny(gpu_lib, wave_on):
    """The bundled plant at 300 perturbed states: the one-wave solver and the
    four-wave solver give the same h, Y and U for every problem (bundled
    fixtures pin the four-wave solver to the reference)."""
    L = gpu_lib.lib()
    ex = gpu_lib.read_example(EXAMPLE_DIR)
    rng = np.random.default_rng(9)
    xs = (ex["x"][None, :] * (1.0 + 0.05 * rng.standard_normal((300, ex["ns"])))).astype(np.float32)
    a = gpu_lib.mpc_batch(EXAMPLE_DIR, xs)
    a.solve(max_updates=CAP)
    cur = L.pqp_tune_wave_min_b(1 << 30)
    b = gpu_lib.mpc_batch(EXAMPLE_DIR, xs)
    b.solve(max_updates=CAP)
    L.pqp_tune_wave_min_b(cur)
    assert np.array_equal(a.h.cpu().numpy(), b.h.cpu().numpy())
    assert np.array_equal(a.status.cpu().numpy(), b.status.cpu().numpy())
    assert_bitwise(a.Y.cpu().numpy(), b.Y.cpu().numpy(), "Y")
    assert_bitwise(a.U.cpu().numpy(), b.U.cpu().numpy(), "U")
    assert int(a.h.cpu().numpy().min()) >= 313


def test_wave_resumes_across_launches(gpu_lib, orc, wave_on):
    """A capped solve longer than one launch's chunk (the solver stops and
    resumes from its saved state): equal to the oracle's capped solve."""
    N, M = 32, 32
    P = orc.synth_problem(3, 1, N, M)
    pb = _batch_of(gpu_lib, [P], N, M)
    cap = 30000  # > the per-launch chunk at this size
    pb.solve(max_updates=cap)
    h, Y, U = orc.solve(P, max_updates=cap)
    assert int(pb.h[0]) == abs(h)
    assert_bitwise(pb.Y[0].cpu().numpy(), Y, "Y")
    assert_bitwise(pb.U[0].cpu().numpy(), U, "U")
