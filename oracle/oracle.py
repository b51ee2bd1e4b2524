"""ctypes front-end for the TEST-ONLY checkers built by ``oracle/Makefile``.

* :class:`Oracle` wraps ``oracle/_build/liboracle.so``: the CPU restatement of
  PQP_CPU.c (``oracle/pqp_oracle.c``; every function there cites the
  reference file:line it follows).
* :class:`Reference` wraps ``oracle/_ref/libpqp_ref.so``: the reference
  PQP_CPU.c itself, compiled unmodified from /root/reference (``main`` renamed).
  It only exists where the reference sources exist (this container) or where
  the prebuilt file travelled with the repo snapshot.

Only ``tests/``, ``bench.py``'s ``cpu_baseline`` leg and
``__graft_entry__.smoke()`` import this module, and only as a checker.  The
product package (``pqp-for-mpc_amd/pqp_amd``) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ORACLE_SO = HERE / "_build" / "liboracle.so"
REF_SO = HERE / "_ref" / "libpqp_ref.so"
REF_BIN = HERE / "_ref" / "pqp_cpu_ref"
REF_TEST_SO = HERE / "_ref" / "libpqp_ref_test.so"
REF_FIXED_SO = HERE / "_ref" / "libref_fixed.so"
REF_CONVERGE_SO = HERE / "_ref" / "libref_converge.so"

# Bundled-example dimensions: PQP_CPU.c:13-17 (pHorizon=1, nState=29, nInput=7,
# nOutput=7, nDis=1) -> M = 7 primal, N = 28 dual (PQP_CPU.c:940-941).
EX_M, EX_ND, EX_NS = 7, 1, 29
EX_N = 4 * EX_M

_fp = C.POINTER(C.c_float)


def build():
    """Build the oracle (and, where /root/reference exists, oracle/_ref)."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _p(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_fp)


def block_diag_problem(P: dict, k: int) -> dict:
    """k copies of dual problem P on the diagonal (test data, numpy only):
    Qd, Gp, Qp, Qp_inv block-diagonal, the vectors tiled, Md and Mp times k.
    Rows of different blocks never meet in a product (the zero entries add
    +0.0 to a sum that is never -0.0), so every block's iterate is P's own,
    bit for bit, while terminate()'s dots run over all k*N (k*M) entries.
    From the bundled example this gives large problems that STOP under the
    reference's exact-float test (h = 313 up to n_dual 1008, 36 copies)."""
    N, M = int(P["N"]), int(P["M"])

    def bd(a, r, c):
        out = np.zeros((k * r, k * c), np.float32)
        a = np.asarray(a, np.float32).reshape(r, c)
        for b in range(k):
            out[b * r:(b + 1) * r, b * c:(b + 1) * c] = a
        return out.reshape(-1)

    tile = lambda a: np.tile(np.asarray(a, np.float32).reshape(-1), k)  # noqa: E731
    return dict(Qd=bd(P["Qd"], N, N), Gp=bd(P["Gp"], N, M), Qp=bd(P["Qp"], M, M), Qp_inv=bd(P["Qp_inv"], M, M),
                Fd=tile(P["Fd"]), Kp=tile(P["Kp"]), Fp=tile(P["Fp"]),
                Md=(np.asarray(P["Md"], np.float32) * np.float32(k)).reshape(1),
                Mp=(np.asarray(P["Mp"], np.float32) * np.float32(k)).reshape(1), N=k * N, M=k * M)


class Oracle:
    """The CPU restatement (test infrastructure)."""

    def __init__(self, path: Path = ORACLE_SO):
        if not Path(path).exists():
            build()
        self.lib = L = C.CDLL(str(path))
        L.orc_matmul.argtypes = [_fp, _fp, C.c_int, _fp, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_gauss_jordan.argtypes = [_fp, _fp, C.c_int]
        L.orc_compute_fp.argtypes = [_fp] * 6 + [C.c_int] * 3
        L.orc_compute_mp.argtypes = [_fp] * 9 + [C.c_int] * 2
        L.orc_convert_to_dual.argtypes = [_fp] * 8 + [C.c_int] * 2
        L.orc_theta_diag.argtypes = [_fp, _fp, C.c_int]
        L.orc_split_theta.argtypes = [_fp] * 4 + [C.c_int]
        L.orc_update_split.argtypes = [_fp] * 6 + [C.c_int]
        L.orc_update.argtypes = [_fp] * 5 + [C.c_int]
        L.orc_u_from_y.argtypes = [_fp] * 5 + [C.c_int] * 2
        L.orc_feasible.argtypes = [_fp] * 3 + [C.c_int] * 2
        L.orc_feasible.restype = C.c_int
        L.orc_cost.argtypes = [_fp] * 4 + [C.c_int]
        L.orc_cost.restype = C.c_float
        L.orc_terminate.argtypes = [_fp] * 11 + [C.c_int] * 2 + [_fp, _fp]
        L.orc_terminate.restype = C.c_int
        L.orc_solve.argtypes = [_fp] * 11 + [C.c_int] * 3 + [C.c_long] * 2
        L.orc_solve.restype = C.c_long
        L.orc_load_example.argtypes = [C.c_char_p] + [C.c_int] * 3 + [_fp] * 14
        L.orc_load_example.restype = C.c_int
        L.orc_synth_key.argtypes = [C.c_uint32] * 3
        L.orc_synth_key.restype = C.c_uint32
        L.orc_synth_primal.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.c_int] + [_fp] * 5
        L.orc_time_updates.argtypes = [_fp, _fp, _fp, C.c_int, C.c_long]
        L.orc_time_updates.restype = C.c_double
        L.orc_time_updates_batch.argtypes = [C.c_int] + [_fp] * 5 + [C.c_int, C.c_long, C.c_int]
        L.orc_time_updates_batch.restype = C.c_double

    # -- primitives -------------------------------------------------------
    def matmul(self, A, tA, B, tB, a, b, c):
        A, B = f32(A), f32(B)
        out = np.zeros(a * c, np.float32)
        self.lib.orc_matmul(_p(out), _p(A), tA, _p(B), tB, a, b, c)
        return out

    def gauss_jordan(self, A, n):
        A = f32(A)
        out = np.zeros(n * n, np.float32)
        self.lib.orc_gauss_jordan(_p(A), _p(out), n)
        return out

    def convert_to_dual(self, Qp_inv, Gp, Kp, Fp, Mp, N, M):
        Qd, Fd, Md = np.zeros(N * N, np.float32), np.zeros(N, np.float32), np.zeros(1, np.float32)
        args = [f32(x) for x in (Qp_inv, Gp, Kp, Fp, Mp)]
        self.lib.orc_convert_to_dual(_p(Qd), _p(Fd), _p(Md), *[_p(x) for x in args], N, M)
        return Qd, Fd, Md

    def theta(self, Qd, N):
        Qd = f32(Qd)
        th = np.zeros(N, np.float32)
        self.lib.orc_theta_diag(_p(th), _p(Qd), N)
        return th

    def split_theta(self, Qd, theta, N):
        Qd, theta = f32(Qd), f32(theta)
        qp, qn = np.zeros(N * N, np.float32), np.zeros(N * N, np.float32)
        self.lib.orc_split_theta(_p(qp), _p(qn), _p(Qd), _p(theta), N)
        return qp, qn

    def update(self, Y, Qd, theta, Fd, N):
        Y, Qd, theta, Fd = f32(Y), f32(Qd), f32(theta), f32(Fd)
        out = np.zeros(N, np.float32)
        self.lib.orc_update(_p(out), _p(Y), _p(Qd), _p(theta), _p(Fd), N)
        return out

    def update_split(self, Y, Qdp, Qdn, Fdp, Fdn, N):
        args = [f32(x) for x in (Y, Qdp, Qdn, Fdp, Fdn)]
        out = np.zeros(N, np.float32)
        self.lib.orc_update_split(_p(out), *[_p(x) for x in args], N)
        return out

    def iterate(self, Qd, Fd, N, updates, Y0=None):
        """`updates` fixed-mode updates from Y0 (default all 1000)."""
        th = self.theta(Qd, N)
        Y = np.full(N, 1000.0, np.float32) if Y0 is None else f32(Y0).copy()
        for _ in range(updates):
            Y = self.update(Y, Qd, th, Fd, N)
        return Y

    def u_from_y(self, Y, Fp, Gp, Qp_inv, N, M):
        args = [f32(x) for x in (Y, Fp, Gp, Qp_inv)]
        U = np.zeros(M, np.float32)
        self.lib.orc_u_from_y(_p(U), *[_p(x) for x in args], N, M)
        return U

    def feasible(self, U, Gp, Kp, N, M):
        return int(self.lib.orc_feasible(_p(f32(U)), _p(f32(Gp)), _p(f32(Kp)), N, M))

    def cost(self, Z, Q, F, Mc, n):
        return float(self.lib.orc_cost(_p(f32(Z)), _p(f32(Q)), _p(f32(F)), _p(f32(Mc)), n))

    def terminate(self, Y, Qd, Fd, Md, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M):
        """Returns (flag, U, Jp, Jd); Jp/Jd are NaN when the feasibility test failed."""
        U = np.zeros(M, np.float32)
        jp = np.full(1, np.nan, np.float32)
        jd = np.full(1, np.nan, np.float32)
        args = [f32(x) for x in (Y, Qd, Fd, Md)]
        rest = [f32(x) for x in (Qp, Qp_inv, Fp, Mp, Gp, Kp)]
        flag = self.lib.orc_terminate(*[_p(x) for x in args], _p(U), *[_p(x) for x in rest], N, M, _p(jp), _p(jd))
        return int(flag), U, float(jp[0]), float(jd[0])

    def solve(self, P: dict, mode: int = 0, num_iter: int = 1000, max_updates: int = 1 << 40):
        """solveQuadraticDual on a problem dict (keys: Qd Fd Md Qp Qp_inv Fp Mp Gp Kp N M).
        Returns (h, Y, U)."""
        N, M = P["N"], P["M"]
        Y, U = np.zeros(N, np.float32), np.zeros(M, np.float32)
        a = {k: f32(P[k]) for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
        h = self.lib.orc_solve(_p(Y), _p(a["Qd"]), _p(a["Fd"]), _p(a["Md"]), _p(U), _p(a["Qp"]),
                               _p(a["Qp_inv"]), _p(a["Fp"]), _p(a["Mp"]), _p(a["Gp"]), _p(a["Kp"]),
                               N, M, mode, num_iter, max_updates)
        return int(h), Y, U

    # -- problem construction ---------------------------------------------
    def load_example(self, directory, m=EX_M, nd=EX_ND, ns=EX_NS) -> dict:
        N = 4 * m
        shapes = dict(Qp_inv=m * m, Fp1=m * nd, Fp2=m * ns, Fp3=m, Mp1=ns * ns, Mp2=nd * ns,
                      Mp3=nd * nd, Mp4=ns, Mp5=nd, Mp6=1, Gp=N * m, Kp=N, x=ns, D=nd)
        arr = {k: np.zeros(v, np.float32) for k, v in shapes.items()}
        order = ["Qp_inv", "Fp1", "Fp2", "Fp3", "Mp1", "Mp2", "Mp3", "Mp4", "Mp5", "Mp6", "Gp", "Kp", "x", "D"]
        rc = self.lib.orc_load_example(str(directory).encode(), m, nd, ns, *[_p(arr[k]) for k in order])
        if rc != 0:
            raise IOError(f"could not read example files under {directory}")
        arr.update(N=N, M=m, nd=nd, ns=ns)
        return arr

    def bundled_problem(self, directory) -> dict:
        """main() of PQP_CPU.c:935-996 up to (not including) the solve."""
        P = self.load_example(directory)
        N, M, nd, ns = P["N"], P["M"], P["nd"], P["ns"]
        Qp = self.gauss_jordan(P["Qp_inv"], M)
        Fp, Mp = np.zeros(M, np.float32), np.zeros(1, np.float32)
        self.lib.orc_compute_fp(_p(Fp), _p(P["Fp1"]), _p(P["Fp2"]), _p(P["Fp3"]), _p(P["D"]), _p(P["x"]), M, nd, ns)
        self.lib.orc_compute_mp(_p(Mp), _p(P["Mp1"]), _p(P["Mp2"]), _p(P["Mp3"]), _p(P["Mp4"]), _p(P["Mp5"]),
                                _p(P["Mp6"]), _p(P["D"]), _p(P["x"]), nd, ns)
        Qd, Fd, Md = self.convert_to_dual(P["Qp_inv"], P["Gp"], P["Kp"], Fp, Mp, N, M)
        P.update(Qp=Qp, Fp=Fp, Mp=Mp, Qd=Qd, Fd=Fd, Md=Md)
        return P

    def example_at_state(self, directory, x) -> dict:
        """main()'s setup (PQP_CPU.c:988-994) with the plant state x replaced:
        computeFp (:373), computeMp (:395), Gauss_Jordan (:251), convertToDual
        (:489) on the example's plant."""
        E = self.load_example(directory)
        N, M, nd, ns = E["N"], E["M"], E["nd"], E["ns"]
        x = f32(x)
        Fp, Mp = np.zeros(M, np.float32), np.zeros(1, np.float32)
        self.lib.orc_compute_fp(_p(Fp), _p(E["Fp1"]), _p(E["Fp2"]), _p(E["Fp3"]), _p(E["D"]), _p(x), M, nd, ns)
        self.lib.orc_compute_mp(_p(Mp), *[_p(E[k]) for k in ("Mp1", "Mp2", "Mp3", "Mp4", "Mp5", "Mp6", "D")], _p(x),
                                nd, ns)
        Qd, Fd, Md = self.convert_to_dual(E["Qp_inv"], E["Gp"], E["Kp"], Fp, Mp, N, M)
        return dict(Qd=Qd, Fd=Fd, Md=Md, Qp=self.gauss_jordan(E["Qp_inv"], M), Qp_inv=E["Qp_inv"], Fp=Fp, Mp=Mp,
                    Gp=E["Gp"], Kp=E["Kp"], N=N, M=M)

    def horizon_problem(self, directory, states) -> dict:
        """One stacked-horizon problem (bench.py's horizon leg, pqp_amd.
        horizon_batch): the example's plant once per stage, stage h at state
        states[h] -- computeFp / computeMp per stage (:373, :395), the
        block-diagonal primal, Mp summed in stage order, then Gauss_Jordan
        (:251) and convertToDual (:489) of the whole."""
        stages = [self.example_at_state(directory, x) for x in states]
        H = len(stages)
        N, M = stages[0]["N"], stages[0]["M"]

        def bd(k, r, c):
            out = np.zeros((H * r, H * c), np.float32)
            for h, S in enumerate(stages):
                out[h * r:(h + 1) * r, h * c:(h + 1) * c] = np.asarray(S[k], np.float32).reshape(r, c)
            return out.reshape(-1)

        Mp = np.float32(stages[0]["Mp"][0])
        for S in stages[1:]:
            Mp = np.float32(Mp + np.float32(S["Mp"][0]))
        Q = dict(Qp_inv=bd("Qp_inv", M, M), Gp=bd("Gp", N, M), Kp=np.concatenate([S["Kp"] for S in stages]),
                 Fp=np.concatenate([S["Fp"] for S in stages]), Mp=np.array([Mp], np.float32), N=H * N, M=H * M)
        Q["Qd"], Q["Fd"], Q["Md"] = self.convert_to_dual(Q["Qp_inv"], Q["Gp"], Q["Kp"], Q["Fp"], Q["Mp"], H * N, H * M)
        Q["Qp"] = self.gauss_jordan(Q["Qp_inv"], H * M)
        return Q

    def synth_primal(self, seed, inst, N, M) -> dict:
        P = dict(Qp_inv=np.zeros(M * M, np.float32), Gp=np.zeros(N * M, np.float32),
                 Kp=np.zeros(N, np.float32), Fp=np.zeros(M, np.float32), Mp=np.zeros(1, np.float32))
        self.lib.orc_synth_primal(seed, inst, N, M, _p(P["Qp_inv"]), _p(P["Gp"]), _p(P["Kp"]),
                                  _p(P["Fp"]), _p(P["Mp"]))
        P.update(N=N, M=M)
        return P

    def synth_problem(self, seed, inst, N, M, with_qp=True) -> dict:
        P = self.synth_primal(seed, inst, N, M)
        P["Qd"], P["Fd"], P["Md"] = self.convert_to_dual(P["Qp_inv"], P["Gp"], P["Kp"], P["Fp"], P["Mp"], N, M)
        if with_qp:
            P["Qp"] = self.gauss_jordan(P["Qp_inv"], M)
        return P

    def time_updates_batch(self, Y, Qp, Qn, Fp, Fn, N, rounds, threads):
        """Seconds for `rounds` updates of each of the B problems of the
        stacked split matrices (B x N x N), spread over OpenMP threads."""
        B = Y.size // N
        return float(self.lib.orc_time_updates_batch(B, _p(Y), _p(Qp), _p(Qn), _p(Fp), _p(Fn), N, rounds, threads))

    def time_updates(self, Qd, Fd, N, updates):
        """Seconds for `updates` reference-style updateY2 calls (split matrices stored)."""
        Y = np.zeros(N, np.float32)
        t = self.lib.orc_time_updates(_p(Y), _p(f32(Qd)), _p(f32(Fd)), N, updates)
        return float(t), Y


class Reference:
    """The reference PQP_CPU.c compiled as a shared library (oracle/_ref)."""

    def __init__(self, path: Path = REF_SO):
        if not Path(path).exists():
            raise FileNotFoundError(f"{path} not built (needs /root/reference; run make -C oracle)")
        self.lib = L = C.CDLL(str(path))
        L.matrixMultiply.argtypes = [_fp, _fp, C.c_int, _fp, C.c_int, C.c_int, C.c_int, C.c_int]
        L.Gauss_Jordan.argtypes = [_fp, _fp, C.c_int]
        L.computeFp.argtypes = [_fp] * 6
        L.computeMp.argtypes = [_fp] * 9
        L.convertToDual.argtypes = [_fp] * 8 + [C.c_int] * 2
        L.computeTheta.argtypes = [_fp, _fp, C.c_int]
        L.computeQdp_theta.argtypes = [_fp] * 3 + [C.c_int]
        L.computeQdn_theta.argtypes = [_fp] * 3 + [C.c_int]
        L.matrixPos.argtypes = [_fp, _fp, C.c_int, C.c_int]
        L.matrixNeg.argtypes = [_fp, _fp, C.c_int, C.c_int]
        L.updateY2.argtypes = [_fp] * 7 + [C.c_int]
        L.computeUfromY.argtypes = [_fp] * 5 + [C.c_int] * 2
        L.checkFeas.argtypes = [_fp] * 3 + [C.c_int] * 2
        L.checkFeas.restype = C.c_int
        L.computeCost.argtypes = [_fp] * 4 + [C.c_int]
        L.computeCost.restype = C.c_float
        L.terminate.argtypes = [_fp] * 11 + [C.c_int] * 2
        L.terminate.restype = C.c_int
        L.solveQuadraticDual.argtypes = [_fp] * 11 + [C.c_int] * 2
        L.input.argtypes = [_fp] * 16
        self.libc = C.CDLL(None)

    def bundled_problem(self, example_parent) -> dict:
        """Run the reference's own input()/setup with CWD = example_parent (it
        fopen()s ./example/*.txt, PQP_CPU.c:764)."""
        m, nd, ns, N = EX_M, EX_ND, EX_NS, EX_N
        z = lambda n: np.zeros(n, np.float32)  # noqa: E731
        P = dict(Qp_inv=z(m * m), Fp1=z(m * nd), Fp2=z(m * ns), Fp3=z(m), Mp1=z(ns * ns), Mp2=z(nd * ns),
                 Mp3=z(nd * nd), Mp4=z(ns), Mp5=z(nd), Mp6=z(1), Gp=z(N * m), Kp=z(N), x=z(ns), D=z(nd),
                 theta7=z(7 * nd), Z=z(7 * ns))
        cwd = os.getcwd()
        os.chdir(example_parent)
        try:
            self.lib.input(*[_p(P[k]) for k in ("Qp_inv", "Fp1", "Fp2", "Fp3", "Mp1", "Mp2", "Mp3", "Mp4",
                                                "Mp5", "Mp6", "Gp", "Kp", "x", "D", "theta7", "Z")])
        finally:
            os.chdir(cwd)
        Qp, Fp, Mp = z(m * m), z(m), z(1)
        self.lib.Gauss_Jordan(_p(P["Qp_inv"]), _p(Qp), m)
        self.lib.computeFp(_p(Fp), _p(P["Fp1"]), _p(P["Fp2"]), _p(P["Fp3"]), _p(P["D"]), _p(P["x"]))
        self.lib.computeMp(_p(Mp), *[_p(P[k]) for k in ("Mp1", "Mp2", "Mp3", "Mp4", "Mp5", "Mp6", "D", "x")])
        Qd, Fd, Md = self.convert_to_dual(P["Qp_inv"], P["Gp"], P["Kp"], Fp, Mp, N, m)
        P.update(N=N, M=m, Qp=Qp, Fp=Fp, Mp=Mp, Qd=Qd, Fd=Fd, Md=Md)
        return P

    def convert_to_dual(self, Qp_inv, Gp, Kp, Fp, Mp, N, M):
        Qd, Fd, Md = np.zeros(N * N, np.float32), np.zeros(N, np.float32), np.zeros(1, np.float32)
        a = [f32(x).copy() for x in (Qp_inv, Gp, Kp, Fp, Mp)]
        self.lib.convertToDual(_p(Qd), _p(Fd), _p(Md), *[_p(x) for x in a], N, M)
        return Qd, Fd, Md

    def split(self, Qd, Fd, N):
        """Setup section of solveQuadraticDual (PQP_CPU.c:696-708)."""
        Qd, Fd = f32(Qd).copy(), f32(Fd).copy()
        theta = np.zeros(N * N, np.float32)
        qp, qn = np.zeros(N * N, np.float32), np.zeros(N * N, np.float32)
        fdp, fdn = np.zeros(N, np.float32), np.zeros(N, np.float32)
        self.lib.matrixPos(_p(fdp), _p(Fd), N, 1)
        self.lib.matrixNeg(_p(fdn), _p(Fd), N, 1)
        self.lib.computeTheta(_p(theta), _p(Qd), N)
        self.lib.computeQdp_theta(_p(qp), _p(Qd), _p(theta), N)
        self.lib.computeQdn_theta(_p(qn), _p(Qd), _p(theta), N)
        return dict(theta=theta, Qdp_theta=qp, Qdn_theta=qn, Fdp=fdp, Fdn=fdn)

    def update(self, Y, S, Fd, N):
        out = np.zeros(N, np.float32)
        Y = f32(Y).copy()
        self.lib.updateY2(_p(out), _p(Y), _p(S["Qdp_theta"]), _p(S["Qdn_theta"]), _p(f32(Fd).copy()),
                          _p(S["Fdp"]), _p(S["Fdn"]), N)
        return out

    def terminate(self, Y, P):
        N, M = P["N"], P["M"]
        U = np.zeros(M, np.float32)
        a = {k: f32(P[k]).copy() for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
        flag = self.lib.terminate(_p(f32(Y).copy()), _p(a["Qd"]), _p(a["Fd"]), _p(a["Md"]), _p(U), _p(a["Qp"]),
                                  _p(a["Qp_inv"]), _p(a["Fp"]), _p(a["Mp"]), _p(a["Gp"]), _p(a["Kp"]), N, M)
        return int(flag), U

    def cost(self, Z, Q, F, Mc, n):
        return float(self.lib.computeCost(_p(f32(Z).copy()), _p(f32(Q).copy()), _p(f32(F).copy()),
                                          _p(f32(Mc).copy()), n))

    def feasible(self, U, P):
        return int(self.lib.checkFeas(_p(f32(U).copy()), _p(f32(P["Gp"]).copy()), _p(f32(P["Kp"]).copy()),
                                      P["N"], P["M"]))

    def gauss_jordan(self, A, n):
        out = np.zeros(n * n, np.float32)
        self.lib.Gauss_Jordan(_p(f32(A).copy()), _p(out), n)
        return out

    def u_from_y(self, Y, P):
        U = np.zeros(P["M"], np.float32)
        self.lib.computeUfromY(_p(U), _p(f32(Y).copy()), _p(f32(P["Fp"]).copy()), _p(f32(P["Gp"]).copy()),
                               _p(f32(P["Qp_inv"]).copy()), P["N"], P["M"])
        return U

    def fixed_solve(self, P, num_iter: int = 1000):
        """The reference's fixed-iteration solve (oracle/ref_fixed.c over this
        library's own setup/updateY2/copyMatrix; the testing/ harness loop,
        PQP_CPU_test.c:714-744): Y after num_iter - 1 updates from Y = 1000.
        Returns (Y, seconds of the whole call, seconds of the update loop)."""
        if not hasattr(self, "_fixed"):
            if not REF_FIXED_SO.exists():
                raise FileNotFoundError(f"{REF_FIXED_SO} not built (needs /root/reference; run make -C oracle)")
            self._fixed = C.CDLL(str(REF_FIXED_SO))
            self._fixed.ref_fixed_solve.argtypes = [_fp, _fp, _fp, C.c_int, C.c_long, C.POINTER(C.c_double)]
            self._fixed.ref_fixed_solve.restype = C.c_double
        N = P["N"]
        Y = np.zeros(N, np.float32)
        loop = C.c_double(0.0)
        total = self._fixed.ref_fixed_solve(_p(Y), _p(f32(P["Qd"]).copy()), _p(f32(P["Fd"]).copy()), N, num_iter,
                                            C.byref(loop))
        return Y, float(total), float(loop.value)

    def converge_solve(self, P, cap: int):
        """The reference's converge-mode solve stopped after `cap` updates
        (oracle/ref_converge.c over this library's own setup, terminate and
        updateY2: PQP_CPU.c:696-740 plus the cap test).  Returns (h, Y, U), h < 0
        when capped -- the Oracle.solve(max_updates=cap) convention."""
        if not hasattr(self, "_conv"):
            if not REF_CONVERGE_SO.exists():
                raise FileNotFoundError(f"{REF_CONVERGE_SO} not built (needs /root/reference; run make -C oracle)")
            self._conv = C.CDLL(str(REF_CONVERGE_SO))
            self._conv.ref_converge_solve.argtypes = [_fp] * 11 + [C.c_int, C.c_int, C.c_long]
            self._conv.ref_converge_solve.restype = C.c_long
        N, M = P["N"], P["M"]
        Y, U = np.zeros(N, np.float32), np.zeros(M, np.float32)
        a = {k: f32(P[k]).copy() for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
        h = self._conv.ref_converge_solve(_p(Y), _p(a["Qd"]), _p(a["Fd"]), _p(a["Md"]), _p(U), _p(a["Qp"]),
                                          _p(a["Qp_inv"]), _p(a["Fp"]), _p(a["Mp"]), _p(a["Gp"]), _p(a["Kp"]),
                                          N, M, cap)
        return int(h), Y, U

    def solve(self, P):
        """The reference solveQuadraticDual; returns (h, Y, U) with h parsed from
        its own printf (PQP_CPU.c:741)."""
        N, M = P["N"], P["M"]
        Y, U = np.zeros(N, np.float32), np.zeros(M, np.float32)
        a = {k: f32(P[k]).copy() for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
        with tempfile.TemporaryFile(mode="w+b") as tf:
            self.libc.fflush(None)
            saved = os.dup(1)
            os.dup2(tf.fileno(), 1)
            try:
                self.lib.solveQuadraticDual(_p(Y), _p(a["Qd"]), _p(a["Fd"]), _p(a["Md"]), _p(U), _p(a["Qp"]),
                                            _p(a["Qp_inv"]), _p(a["Fp"]), _p(a["Mp"]), _p(a["Gp"]), _p(a["Kp"]),
                                            N, M)
                self.libc.fflush(None)
            finally:
                os.dup2(saved, 1)
                os.close(saved)
            tf.seek(0)
            text = tf.read().decode()
        h = int(text.strip().split("=")[-1])
        return h, Y, U


class ReferenceTesting:
    """testing/CPU version/PQP_CPU_test.c compiled unmodified (main renamed):
    its input() is the reference reader of the testing/ sample files
    (PQP_CPU_test.c:936-978), including the glibc-rand Kp overwrite."""

    def __init__(self, path: Path = REF_TEST_SO):
        if not Path(path).exists():
            raise FileNotFoundError(f"{path} not built (needs /root/reference)")
        self.lib = C.CDLL(str(path))
        self.lib.input.argtypes = [_fp] * 9 + [C.c_int, C.c_int, C.c_void_p]
        self.libc = C.CDLL(None)
        self.libc.fopen.restype = C.c_void_p
        self.libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
        self.libc.fclose.argtypes = [C.c_void_p]

    def read_testfile(self, path) -> dict:
        fp = self.libc.fopen(str(path).encode(), b"r")
        if not fp:
            raise FileNotFoundError(path)
        try:
            M, N = C.c_int(0), C.c_int(0)
            self.libc.fscanf(C.c_void_p(fp), b"%d%d", C.byref(M), C.byref(N))  # the commented-out main's header read
            M, N = M.value, N.value
            z = lambda n: np.zeros(n, np.float32)  # noqa: E731
            P = dict(Qp_inv=z(M * M), Fp=z(M), Mp=z(1), Gp=z(N * M), Kp=z(N))
            dummy = [z(64) for _ in range(4)]
            self.libc.srand(1)  # a fresh process's rand() state (the harness never seeds)
            self.lib.input(_p(P["Qp_inv"]), _p(P["Fp"]), _p(P["Mp"]), _p(P["Gp"]), _p(P["Kp"]),
                           *[_p(d) for d in dummy], N, M, C.c_void_p(fp))
        finally:
            self.libc.fclose(fp)
        P.update(N=N, M=M)
        return P
