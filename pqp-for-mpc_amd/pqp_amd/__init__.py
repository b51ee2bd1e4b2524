"""pqp_amd -- Python mirror of the reference's solver interface over libpqp.

The functions below keep the reference's names, argument order and meaning
(PQP_CPU.c; see include/pqp.h for the C ABI they call): numpy float32 arrays
stand in for the caller-owned ``float*`` buffers, outputs are written in place.
Every call runs on the GPU through ``libpqp.so`` (built in-tree by
``make -C pqp-for-mpc_amd``).  There is no CPU fallback: if the library or a
gfx950 device is missing, calls raise :class:`PQPError`.

Layers
  * drop-in:  solveQuadraticDual, updateY2, terminate, convertToDual,
    computeUfromY, computeCost, checkFeas, computeTheta, matrixMultiply,
    Gauss_Jordan, computeFp, computeMp
  * status API: solve_dual, update, read_example, run_example
  * batched device API (torch tensors as device memory): :class:`Batch`,
    :class:`ProblemBatch`, :func:`mpc_batch`, :func:`horizon_batch`
  * row blocks of one large problem (row-sharded solve): :class:`RowBlock`
    (driver in :mod:`pqp_amd.rowshard`)
"""
from __future__ import annotations

import ctypes as C
import os
import tempfile
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
# PQP_LIB: another build of the library (A/B timing scripts only)
LIB_PATH = Path(os.environ["PQP_LIB"]) if os.environ.get("PQP_LIB") else PKG / "libpqp.so"

PQP_OK = 0
PQP_ERR_ARG, PQP_ERR_HIP, PQP_ERR_ALLOC, PQP_ERR_IO, PQP_ERR_NOT_CONVERGED, PQP_ERR_NO_DEVICE = -1, -2, -3, -4, -5, -6
PQP_ERR_NEEDS_QDT = -7
MODE_CONVERGE, MODE_FIXED = 0, 1

# The reference's compile-time problem dimensions (PQP_CPU.c:13-17).
P_HORIZON, N_STATE, N_INPUT, N_OUTPUT, N_DIS = 1, 29, 7, 7, 1

_fp = C.POINTER(C.c_float)
_vp = C.c_void_p

# name -> (restype, argtypes) for every symbol of include/pqp.h
SIGNATURES = {
    "pqp_last_error": (C.c_char_p, []),
    "pqp_version": (C.c_int, []),
    "solveQuadraticDual": (None, [_fp] * 11 + [C.c_int] * 2),
    "updateY2": (None, [_fp] * 7 + [C.c_int]),
    "terminate": (C.c_int, [_fp] * 11 + [C.c_int] * 2),
    "convertToDual": (None, [_fp] * 8 + [C.c_int] * 2),
    "computeUfromY": (None, [_fp] * 5 + [C.c_int] * 2),
    "computeCost": (C.c_float, [_fp] * 4 + [C.c_int]),
    "checkFeas": (C.c_int, [_fp] * 3 + [C.c_int] * 2),
    "computeTheta": (None, [_fp, _fp, C.c_int]),
    "matrixMultiply": (None, [_fp, _fp, C.c_int, _fp, C.c_int, C.c_int, C.c_int, C.c_int]),
    "Gauss_Jordan": (None, [_fp, _fp, C.c_int]),
    "computeFp": (None, [_fp] * 6),
    "computeMp": (None, [_fp] * 9),
    "input": (None, [_fp] * 16),
    "pqp_solve_dual": (C.c_int, [_fp] * 9 + [C.c_int] * 3 + [C.c_longlong] * 2 + [_fp, _fp,
                                                                                   C.POINTER(C.c_longlong), _fp, _fp]),
    "pqp_problem_create": (C.c_int, [_fp] * 9 + [C.c_int] * 2 + [C.POINTER(C.c_void_p)]),
    "pqp_problem_create_on": (C.c_int, [C.c_int, _vp] + [_fp] * 9 + [C.c_int] * 2 + [C.POINTER(C.c_void_p)]),
    "pqp_problem_device": (C.c_int, [_vp]),
    "pqp_problem_solve": (C.c_int, [_vp, C.c_int, C.c_longlong, C.c_longlong, _fp, _fp, C.POINTER(C.c_longlong), _fp,
                                    _fp]),
    "pqp_problem_destroy": (C.c_int, [_vp]),
    "pqp_update_host": (C.c_int, [_fp] * 5 + [C.c_int]),
    "pqp_read_example": (C.c_int, [C.c_char_p] + [C.c_int] * 3 + [_fp] * 14),
    "pqp_run_example": (C.c_int, [C.c_char_p, _vp]),
    "pqp_read_testfile": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)] + [_fp] * 5),
    "pqp_batch_generate": (C.c_int, [C.c_uint32, C.c_longlong, C.c_int, C.c_int, C.c_int, _vp, C.c_int, C.c_longlong,
                                     _vp, _vp, _vp, C.c_int, _vp]),
    "pqp_batch_synth_primal": (C.c_int, [C.c_uint32, C.c_longlong] + [C.c_int] * 3 + [_vp] * 5 + [_vp]),
    "pqp_batch_pack": (C.c_int, [C.c_int, C.c_int, _vp, _vp, C.c_int, C.c_longlong, _vp]),
    "pqp_batch_theta": (C.c_int, [C.c_int, C.c_int, _vp, C.c_int, C.c_longlong, _vp, C.c_int, _vp]),
    "pqp_batch_update": (C.c_int, [C.c_int, C.c_int, _vp, C.c_int, C.c_longlong, _vp, _vp, C.c_int, _vp, _vp, _vp]),
    "pqp_batch_iterate": (C.c_int, [C.c_int, C.c_int, _vp, C.c_int, C.c_longlong, _vp, _vp, C.c_int, _vp, _vp,
                                    C.c_int, _vp]),
    "pqp_batch_gauss_jordan": (C.c_int, [C.c_int, C.c_int, _vp, _vp, _vp]),
    "pqp_batch_convert_to_dual": (C.c_int, [C.c_int] * 3 + [_vp] * 8 + [_vp]),
    "pqp_release_workspaces": (C.c_int, []),
    "pqp_batch_compute_fp": (C.c_int, [C.c_int] * 4 + [_vp] * 6 + [_vp]),
    "pqp_batch_compute_mp": (C.c_int, [C.c_int] * 3 + [_vp] * 9 + [_vp]),
    "pqp_batch_solve": (C.c_int, [C.c_int] * 3 + [_vp] * 9 + [C.c_int, C.c_longlong, C.c_longlong] + [_vp] * 4
                        + [_vp]),
    "pqp_batch_solve_path": (C.c_int, [C.c_int, C.c_int]),
    "pqp_batch_solve_kernel": (C.c_int, [C.c_int, C.c_int]),
    "pqp_batch_prepare": (C.c_int, [C.c_int] * 3 + [_vp] * 8 + [C.POINTER(C.c_int), _vp]),
    "pqp_batch_solve_prepared": (C.c_int, [C.c_int] * 3 + [_vp] * 14 + [C.c_int, C.c_longlong, C.c_longlong]
                                 + [_vp] * 4 + [_vp]),
    "pqp_rowblock_create": (C.c_int, [_vp, C.c_int, _vp, C.c_int, C.c_int, C.c_int, _vp, C.POINTER(C.c_void_p)]),
    "pqp_rowblock_update": (C.c_int, [_vp, _vp, _vp, _vp]),
    "pqp_rowblock_check": (C.c_int, [_vp, _vp]),
    "pqp_rowblock_destroy": (C.c_int, [_vp]),
    "pqp_synth_rows": (C.c_int, [C.c_uint32, C.c_longlong] + [C.c_int] * 4 + [_vp, C.c_int, _vp, _vp, _vp]),
    # include/pqp_tuning.h
    "pqp_tune": (C.c_int, [C.c_char_p, C.c_longlong, C.POINTER(C.c_longlong)]),
    "pqp_tune_get": (C.c_int, [C.c_char_p, C.POINTER(C.c_longlong)]),
    "pqp_tune_trace": (C.c_int, [C.c_char_p, _vp, C.c_int]),
    "pqp_tune_glibc_rand": (C.c_int, [C.c_int, C.POINTER(C.c_int)]),
    "pqp_tune_poison_lds": (C.c_int, [C.c_float]),
}


class PQPError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libpqp error {code}: {msg}")
        self.code = code


_LIB = None


def lib() -> C.CDLL:
    """Load the in-tree libpqp.so (raises if it was not built)."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise PQPError(PQP_ERR_NO_DEVICE, f"{LIB_PATH} is missing: run `make -C pqp-for-mpc_amd` "
                                              "(or __graft_entry__.build())")
        # One HIP runtime per process: PyTorch-ROCm ships its own
        # libamdhip64.so.7.  Loading torch first makes libpqp's DT_NEEDED
        # libamdhip64.so.7 bind to that copy, so torch streams/pointers and
        # libpqp share a runtime (and a second runtime never starts).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("PQP_LIB") and not hasattr(L, name):
                continue  # an older build under A/B: entry points it lacks stay unbound
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
        if hasattr(L, "pqp_tune"):
            _attach_knobs(L)
    return _LIB


# ---------------------------------------------------------------------------
# tuning knobs (include/pqp_tuning.h): one keyed C entry point; Python names
# ---------------------------------------------------------------------------
def tune(key: str, value: int) -> int:
    """pqp_tune: set knob `key`, return its previous value."""
    old = C.c_longlong(0)
    _check(lib().pqp_tune(key.encode(), int(value), C.byref(old)))
    return int(old.value)


def tune_get(key: str, arg: int = 0) -> int:
    """pqp_tune_get: a knob's value or a diagnostic (last_path,
    persist_fallbacks, converge_grid with arg = N << 32 | M)."""
    v = C.c_longlong(int(arg))
    _check(lib().pqp_tune_get(key.encode(), C.byref(v)))
    return int(v.value)


def poison_lds(value: float = float("nan")) -> None:
    """pqp_tune_poison_lds (test hook): fill every CU's LDS with `value`, so a
    kernel that reads LDS it never wrote reads that value."""
    _check(lib().pqp_tune_poison_lds(float(value)))


def batch_chunk_for(N: int, M: int) -> int:
    """Iterates per problem that one pqp_batch_solve launch runs for (N, M):
    the library's own sizing (or the batch_chunk knob when set)."""
    return tune_get("batch_chunk_for", (int(N) << 32) | int(M))


# L.pqp_tune_<name>(value) -> previous value, for the knobs the tests and
# scripts set (one C entry point behind them all)
_KNOB_NAMES = {"persist": "persist_off", "converge_persist": "converge_persist_off", "wide_min_n": "wide_min_n",
               "lean_min_n": "lean_min_n", "relay_spin_max": "relay_spin_max", "matmul_tiled": "matmul_tiled_off",
               "gj_blocked": "gj_blocked_off", "persist_fit_cus": "persist_fit_cus",
               "persist_stall": "persist_stall_wg", "converge_chunk": "converge_chunk", "wave_min_b": "wave_min_b",
               "fixed_rl_max_b": "fixed_rl_max_b", "wave_pipe_max_b": "wave_pipe_max_b"}


def _set_variant(variant: int) -> int:
    """The packed kernel-variant word of the round-1 tuning API: 0x100
    force_small, 0x200 force_single, bits 17-19 split_lw (1: 8 ... 4: 64)."""
    known = 0x100 | 0x200 | (7 << 17)
    if variant & ~known:  # the retired arms' bits (split_kind, split_u, ...): refused, not dropped
        raise PQPError(PQP_ERR_ARG, f"pqp_tune_set_variant: retired variant bits {variant & ~known:#x}")
    lw_old = tune_get("split_lw")
    old = ((0x100 if tune_get("force_small") else 0) | (0x200 if tune_get("force_single") else 0)
           | (((lw_old.bit_length() - 3) if lw_old else 0) << 17))
    sel = (variant >> 17) & 7
    tune("split_lw", 4 << sel if 1 <= sel <= 4 else 0)
    tune("force_small", 1 if variant & 0x100 else 0)
    tune("force_single", 1 if variant & 0x200 else 0)
    return old


def _batch_converge(opts: int) -> int:
    """batch_opts plus the k_solve_single build bit (2: 4-byte loads) in one
    word."""
    return tune("batch_opts", opts & 19) | (4 if tune("single_scalar", 1 if opts & 4 else 0) else 0)


def _last_path(fallbacks=None) -> int:
    """Solver path of this thread's last solve; the fallback count goes to
    `fallbacks` (a c_longlong or byref() of one) when given."""
    if fallbacks is not None:
        getattr(fallbacks, "_obj", fallbacks).value = tune_get("persist_fallbacks")
    return tune_get("last_path")


def _attach_knobs(L):
    for name, key in _KNOB_NAMES.items():
        setattr(L, f"pqp_tune_{name}", lambda v, key=key: tune(key, v))
    L.pqp_tune_set_variant = _set_variant
    L.pqp_tune_batch_converge = _batch_converge
    L.pqp_tune_last_path = _last_path
    L.pqp_tune_converge_grid = lambda N, M: tune_get("converge_grid", (int(N) << 32) | int(M))
    L.pqp_tune_persist_trace = lambda buf, n: L.pqp_tune_trace(b"persist", buf, n)
    L.pqp_tune_converge_trace = lambda buf, n: L.pqp_tune_trace(b"converge", buf, n)


def last_error() -> str:
    return (lib().pqp_last_error() or b"").decode()


def _check(rc: int):
    if rc != PQP_OK:
        raise PQPError(rc, last_error())


def _f32(a) -> np.ndarray:
    a = np.asarray(a, dtype=np.float32)
    return np.ascontiguousarray(a)


def _buf(a: np.ndarray):
    if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]):
        raise TypeError("buffers must be C-contiguous float32 numpy arrays")
    return a.ctypes.data_as(_fp)


# ---------------------------------------------------------------------------
# drop-in entry points (reference names; outputs written in place)
# ---------------------------------------------------------------------------
def solveQuadraticDual(Y, Qd, Fd, Md, U, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M):
    """PQP_CPU.c:694 -- prints 'Printing number of iterations = h'."""
    lib().solveQuadraticDual(*[_buf(a) for a in (Y, Qd, Fd, Md, U, Qp, Qp_inv, Fp, Mp, Gp, Kp)], N, M)


def updateY2(Y_next, Y, Qdp_theta, Qdn_theta, Fd, Fdp, Fdn, N):
    """PQP_CPU.c:603."""
    lib().updateY2(*[_buf(a) for a in (Y_next, Y, Qdp_theta, Qdn_theta, Fd, Fdp, Fdn)], N)


def terminate(Y, Qd, Fd, Md, U, Qp, Qp_inv, Fp, Mp, Gp, Kp, N, M) -> int:
    """PQP_CPU.c:673."""
    return int(lib().terminate(*[_buf(a) for a in (Y, Qd, Fd, Md, U, Qp, Qp_inv, Fp, Mp, Gp, Kp)], N, M))


def convertToDual(Qd, Fd, Md, Qp_inv, Gp, Kp, Fp, Mp, N, M):
    """PQP_CPU.c:489."""
    lib().convertToDual(*[_buf(a) for a in (Qd, Fd, Md, Qp_inv, Gp, Kp, Fp, Mp)], N, M)


def computeUfromY(U, Y, Fp, Gp, Qp_inv, N, M):
    """PQP_CPU.c:352."""
    lib().computeUfromY(*[_buf(a) for a in (U, Y, Fp, Gp, Qp_inv)], N, M)


def computeCost(Z, Q, F, Mc, N) -> float:
    """PQP_CPU.c:648."""
    return float(lib().computeCost(*[_buf(a) for a in (Z, Q, F, Mc)], N))


def checkFeas(U, Gp, Kp, N, M) -> int:
    """PQP_CPU.c:632."""
    return int(lib().checkFeas(*[_buf(a) for a in (U, Gp, Kp)], N, M))


def computeTheta(theta, Qd, N):
    """PQP_CPU.c:503."""
    lib().computeTheta(_buf(theta), _buf(Qd), N)


def matrixMultiply(output, mat1, transpose1, mat2, transpose2, a, b, c):
    """PQP_CPU.c:84."""
    lib().matrixMultiply(_buf(output), _buf(mat1), transpose1, _buf(mat2), transpose2, a, b, c)


def Gauss_Jordan(A, res, N):
    """PQP_CPU.c:251."""
    lib().Gauss_Jordan(_buf(A), _buf(res), N)


def computeFp(Fp, Fp1, Fp2, Fp3, D, x):
    """PQP_CPU.c:373 (bundled dimensions)."""
    lib().computeFp(*[_buf(a) for a in (Fp, Fp1, Fp2, Fp3, D, x)])


def computeMp(Mp, Mp1, Mp2, Mp3, Mp4, Mp5, Mp6, D, x):
    """PQP_CPU.c:395 (bundled dimensions)."""
    lib().computeMp(*[_buf(a) for a in (Mp, Mp1, Mp2, Mp3, Mp4, Mp5, Mp6, D, x)])


# ---------------------------------------------------------------------------
# status API
# ---------------------------------------------------------------------------
def solve_dual(P: dict, mode: int = MODE_CONVERGE, num_iter: int = 1000, max_updates: int = 0):
    """pqp_solve_dual on a problem dict with keys Qd Fd Md Qp Qp_inv Fp Mp Gp Kp N M.

    Returns dict(h, Y, U, Jp, Jd, converged).  Raises on any error other than
    hitting the update cap in converge mode (then converged=False)."""
    N, M = int(P["N"]), int(P["M"])
    a = {k: _f32(P[k]) for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")}
    Y, U = np.zeros(N, np.float32), np.zeros(M, np.float32)
    h = C.c_longlong(0)
    jp, jd = np.zeros(1, np.float32), np.zeros(1, np.float32)
    rc = lib().pqp_solve_dual(*[_buf(a[k]) for k in ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")],
                              N, M, mode, num_iter, max_updates, _buf(Y), _buf(U), C.byref(h), _buf(jp), _buf(jd))
    if rc not in (PQP_OK, PQP_ERR_NOT_CONVERGED):
        _check(rc)
    return dict(h=int(h.value), Y=Y, U=U, Jp=float(jp[0]), Jd=float(jd[0]), converged=(rc == PQP_OK))


class Problem:
    """A dual problem resident in HBM (pqp_problem_*): upload/prepare once,
    solve repeatedly.  Keys of P: Qd Fd Md Qp Qp_inv Fp Mp Gp Kp N M.
    `device` (int) and `stream` (a hipStream_t of that device, as int or
    torch stream) bind the handle (pqp_problem_create_on); by default the
    current device and a stream of the handle's own.  Solves release the GIL
    (ctypes), so handles may be solved from several threads at once."""

    KEYS = ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")

    def __init__(self, P: dict, device: int | None = None, stream=None):
        import threading

        self.N, self.M = int(P["N"]), int(P["M"])
        a = [_f32(P[k]) for k in self.KEYS]
        h = C.c_void_p()
        if stream is not None and not isinstance(stream, int):
            stream = stream.cuda_stream
        _check(lib().pqp_problem_create_on(-1 if device is None else int(device), stream, *[_buf(x) for x in a],
                                           self.N, self.M, C.byref(h)))
        self._h = h
        # the outputs and their ctypes pointers are made once (building a
        # pointer per call cost ~4 us each -- a fifth of a bundled solve); a
        # lock keeps two threads solving this handle from sharing them (the
        # library serializes the solves of one handle anyway)
        self._Y, self._U = np.zeros(self.N, np.float32), np.zeros(self.M, np.float32)
        self._jp, self._jd = np.zeros(1, np.float32), np.zeros(1, np.float32)
        self._hv = C.c_longlong(0)
        self._args = (_buf(self._Y), _buf(self._U), C.byref(self._hv), _buf(self._jp), _buf(self._jd))
        self._solve = lib().pqp_problem_solve
        self._lock = threading.Lock()

    @property
    def device(self) -> int:
        return int(lib().pqp_problem_device(self._h))

    def solve(self, mode: int = MODE_CONVERGE, num_iter: int = 1000, max_updates: int = 0) -> dict:
        with self._lock:
            rc = self._solve(self._h, mode, num_iter, max_updates, *self._args)
            if rc not in (PQP_OK, PQP_ERR_NOT_CONVERGED):
                _check(rc)
            return dict(h=int(self._hv.value), Y=self._Y.copy(), U=self._U.copy(), Jp=float(self._jp[0]),
                        Jd=float(self._jd[0]), converged=(rc == PQP_OK))

    def close(self):
        if self._h:
            lib().pqp_problem_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def update(Qd, theta_diag, Fd, Y, N) -> np.ndarray:
    """One fused update (pqp_update_host)."""
    out = np.zeros(N, np.float32)
    _check(lib().pqp_update_host(_buf(_f32(Qd)), _buf(_f32(theta_diag)), _buf(_f32(Fd)), _buf(_f32(Y)),
                                 _buf(out), N))
    return out


def read_example(directory, m=N_INPUT * P_HORIZON, nd=N_DIS * P_HORIZON, ns=N_STATE) -> dict:
    """Host reader of example/*.txt (PQP_CPU.c:757-930).  No GPU work."""
    N = 4 * m
    shapes = dict(Qp_inv=m * m, Fp1=m * nd, Fp2=m * ns, Fp3=m, Mp1=ns * ns, Mp2=nd * ns, Mp3=nd * nd, Mp4=ns,
                  Mp5=nd, Mp6=1, Gp=N * m, Kp=N, x=ns, D=nd)
    arr = {k: np.zeros(v, np.float32) for k, v in shapes.items()}
    order = ["Qp_inv", "Fp1", "Fp2", "Fp3", "Mp1", "Mp2", "Mp3", "Mp4", "Mp5", "Mp6", "Gp", "Kp", "x", "D"]
    _check(lib().pqp_read_example(str(directory).encode(), m, nd, ns, *[_buf(arr[k]) for k in order]))
    arr.update(N=N, M=m, nd=nd, ns=ns)
    return arr


def read_testfile(path, glibc_kp: bool = True) -> dict:
    """testing/ sample-test file (pqp_read_testfile).  No GPU work."""
    M, N = C.c_int(0), C.c_int(0)
    _check(lib().pqp_read_testfile(str(path).encode(), int(glibc_kp), C.byref(M), C.byref(N), None, None, None, None,
                                   None))
    M, N = M.value, N.value
    arr = dict(Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32), Mp=np.zeros(1, np.float32),
               Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32))
    Mi, Ni = C.c_int(M), C.c_int(N)  # the dimensions the arrays were sized for
    _check(lib().pqp_read_testfile(str(path).encode(), int(glibc_kp), C.byref(Mi), C.byref(Ni),
                                   *[_buf(arr[k]) for k in ("Qp_inv", "Fp", "Mp", "Gp", "Kp")]))
    arr.update(N=N, M=M)
    return arr


def testfile_problem(path, glibc_kp: bool = True) -> dict:
    """A testing/ sample-test file as a dual problem, setup on the GPU
    (Gauss_Jordan, convertToDual)."""
    P = read_testfile(path, glibc_kp)
    N, M = P["N"], P["M"]
    Qp = np.zeros(M * M, np.float32)
    Gauss_Jordan(P["Qp_inv"], Qp, M)
    Qd, Fd, Md = np.zeros(N * N, np.float32), np.zeros(N, np.float32), np.zeros(1, np.float32)
    convertToDual(Qd, Fd, Md, P["Qp_inv"], P["Gp"], P["Kp"], P["Fp"], P["Mp"], N, M)
    P.update(Qp=Qp, Qd=Qd, Fd=Fd, Md=Md)
    return P


def example_problem(directory) -> dict:
    """main() of PQP_CPU.c:935-994 up to the solve, on the GPU: read the
    example files, Gauss_Jordan, computeFp, computeMp, convertToDual.  Returns
    the dual problem dict accepted by solve_dual()."""
    P = read_example(directory)
    N, M = P["N"], P["M"]
    Qp, Fp, Mp = np.zeros(M * M, np.float32), np.zeros(M, np.float32), np.zeros(1, np.float32)
    Gauss_Jordan(P["Qp_inv"], Qp, M)
    computeFp(Fp, P["Fp1"], P["Fp2"], P["Fp3"], P["D"], P["x"])
    computeMp(Mp, P["Mp1"], P["Mp2"], P["Mp3"], P["Mp4"], P["Mp5"], P["Mp6"], P["D"], P["x"])
    Qd, Fd, Md = np.zeros(N * N, np.float32), np.zeros(N, np.float32), np.zeros(1, np.float32)
    convertToDual(Qd, Fd, Md, P["Qp_inv"], P["Gp"], P["Kp"], Fp, Mp, N, M)
    P.update(Qp=Qp, Fp=Fp, Mp=Mp, Qd=Qd, Fd=Fd, Md=Md)
    return P


def run_example(directory) -> str:
    """main() of PQP_CPU.c on the GPU; returns what it prints."""
    libc = C.CDLL(None)
    libc.fopen.restype = C.c_void_p
    libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
    libc.fclose.argtypes = [C.c_void_p]
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "out.txt")
        fh = libc.fopen(path.encode(), b"w")
        try:
            rc = lib().pqp_run_example(str(directory).encode(), fh)
        finally:
            libc.fclose(fh)
        _check(rc)
        return Path(path).read_text()


# ---------------------------------------------------------------------------
# batched device API (torch provides the HBM buffers and the stream)
# ---------------------------------------------------------------------------
def dense_qinv(seed: int, M: int) -> np.ndarray:
    """A dense symmetric Qp_inv (M x M row-major, fp32) from numpy's seeded
    generator: diagonal in [1, 2), off-diagonal in [-0.05, 0.05).  The general
    (non-diagonal) setup case: its convertToDual Qd is not bit-symmetric.  The
    golden fixture tests/golden/dense_dual.npz was made by the reference from it."""
    rng = np.random.default_rng(1000 + seed)
    A = rng.uniform(-0.05, 0.05, (M, M)).astype(np.float32)
    Q = np.triu(A) + np.triu(A, 1).T
    Q[np.diag_indices(M)] = rng.uniform(1.0, 2.0, M).astype(np.float32)
    return np.ascontiguousarray(Q, np.float32).reshape(-1)


def round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


class Batch:
    """B independent dual problems of size N resident in HBM.

    QdT is [B][N][ldq] fp32 with Qd stored column-major per problem (element
    (i,k) at k*ldq + i); theta/Fd/Y are [B][ldv].  All launches go to torch's
    current HIP stream of ``device``.
    """

    def __init__(self, B: int, N: int, device=None, ldq: int | None = None, ldv: int | None = None):
        import torch

        self.torch = torch
        self.B, self.N = int(B), int(N)
        self.ldq = int(ldq) if ldq else round_up(self.N, 4)
        self.ldv = int(ldv) if ldv else round_up(self.N, 4)
        self.qstride = self.N * self.ldq
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        kw = dict(dtype=torch.float32, device=self.device)
        self.QdT = torch.empty(self.B * self.qstride, **kw)
        self.theta = torch.zeros(self.B, self.ldv, **kw)
        self.Fd = torch.zeros(self.B, self.ldv, **kw)
        self.Md = torch.zeros(self.B, **kw)
        self.Y = torch.zeros(self.B, self.ldv, **kw)
        self.Y2 = torch.zeros(self.B, self.ldv, **kw)

    def _stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def _p(t):
        return C.c_void_p(t.data_ptr())

    def generate(self, seed: int, inst0: int = 0, M: int | None = None):
        """Synthetic problems inst0..inst0+B-1 of `seed` (M defaults to N/2)."""
        M = int(M) if M else max(1, self.N // 2)
        self.M = M
        _check(lib().pqp_batch_generate(seed, inst0, self.B, self.N, M, self._p(self.QdT), self.ldq, self.qstride,
                                        self._p(self.Fd), self._p(self.Md), self._p(self.theta), self.ldv,
                                        self._stream()))
        return self

    def load(self, Qd, Fd):
        """Load row-major Qd ([B][N*N] or [B][N][N]) and Fd ([B][N]) given as
        numpy/torch; packs to QdT on the GPU and computes theta."""
        torch = self.torch
        Qd = torch.as_tensor(np.asarray(Qd, np.float32) if not torch.is_tensor(Qd) else Qd, dtype=torch.float32)
        Qd = Qd.reshape(self.B, self.N * self.N).to(self.device).contiguous()
        Fd = torch.as_tensor(np.asarray(Fd, np.float32) if not torch.is_tensor(Fd) else Fd, dtype=torch.float32)
        self.Fd.zero_()
        self.Fd[:, : self.N] = Fd.reshape(self.B, self.N).to(self.device)
        self.QdT.zero_()
        _check(lib().pqp_batch_pack(self.B, self.N, self._p(Qd), self._p(self.QdT), self.ldq, self.qstride,
                                    self._stream()))
        _check(lib().pqp_batch_theta(self.B, self.N, self._p(self.QdT), self.ldq, self.qstride, self._p(self.theta),
                                     self.ldv, self._stream()))
        torch.cuda.current_stream(self.device).synchronize()  # Qd staging buffer goes out of scope
        return self

    def reset(self, value: float = 1000.0):
        self.Y.fill_(value)
        return self

    def update(self):
        """One updateY2 for every problem: Y <- Y_next (pqp_batch_update)."""
        _check(lib().pqp_batch_update(self.B, self.N, self._p(self.QdT), self.ldq, self.qstride, self._p(self.theta),
                                      self._p(self.Fd), self.ldv, self._p(self.Y), self._p(self.Y2), self._stream()))
        self.Y, self.Y2 = self.Y2, self.Y
        return self

    def iterate(self, updates: int, from_start: bool = True):
        """`updates` fused updates per problem in one launch (pqp_batch_iterate);
        from_start=True begins at the reference's Y = 1000."""
        y0 = None if from_start else self._p(self.Y)
        _check(lib().pqp_batch_iterate(self.B, self.N, self._p(self.QdT), self.ldq, self.qstride, self._p(self.theta),
                                       self._p(self.Fd), self.ldv, y0, self._p(self.Y2), int(updates),
                                       self._stream()))
        self.Y, self.Y2 = self.Y2, self.Y
        return self

    def result(self) -> np.ndarray:
        return self.Y[:, : self.N].cpu().numpy()

    def qd_rowmajor(self, b: int) -> np.ndarray:
        """Problem b's Qd back in the reference's row-major layout (host)."""
        qt = self.QdT[b * self.qstride:(b + 1) * self.qstride].reshape(self.N, self.ldq)[:, : self.N]
        return qt.t().contiguous().cpu().numpy().reshape(-1)


class ProblemBatch:
    """B independent dual problems of sizes (N, M) resident in HBM, solved one
    workgroup per problem (pqp_batch_* of include/pqp.h).  Arrays follow the
    reference's row-major layout per problem, stacked: Qd [B, N*N], Fd [B, N],
    Md [B], Qp / Qp_inv [B, M*M], Fp [B, M], Mp [B], Gp [B, N*M], Kp [B, N]."""

    PRIMAL = ("Qp_inv", "Gp", "Kp", "Fp", "Mp")
    DUAL = ("Qd", "Fd", "Md")

    def __init__(self, B: int, N: int, M: int, device=None, transposes: bool = True):
        import torch

        self.torch = torch
        self.B, self.N, self.M = int(B), int(N), int(M)
        self.transposes = bool(transposes)  # prepare() keeps Gp', Qp_inv' for coalesced row walks (path 2)
        self._prep = None  # pqp_batch_prepare's per-problem data, until Qd / Gp / Qp_inv change
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        f = dict(dtype=torch.float32, device=self.device)
        B, N, M = self.B, self.N, self.M
        self.Qd, self.Fd, self.Md = torch.zeros(B, N * N, **f), torch.zeros(B, N, **f), torch.zeros(B, **f)
        self.Qp, self.Qp_inv = torch.zeros(B, M * M, **f), torch.zeros(B, M * M, **f)
        self.Fp, self.Mp = torch.zeros(B, M, **f), torch.zeros(B, **f)
        self.Gp, self.Kp = torch.zeros(B, N * M, **f), torch.zeros(B, N, **f)
        self.Y, self.U = torch.zeros(B, N, **f), torch.zeros(B, M, **f)
        self.h = torch.zeros(B, dtype=torch.int64, device=self.device)
        self.status = torch.zeros(B, dtype=torch.int32, device=self.device)

    def _s(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def _p(t):
        return C.c_void_p(t.data_ptr())

    @classmethod
    def replicate(cls, P: dict, B: int, device=None) -> "ProblemBatch":
        """B copies of one problem dict (keys of solve_dual)."""
        pb = cls(B, int(P["N"]), int(P["M"]), device)
        for k in cls.PRIMAL + cls.DUAL + ("Qp",):
            if k in P:
                v = pb.torch.as_tensor(np.asarray(P[k], np.float32).reshape(-1), device=pb.device)
                getattr(pb, k).copy_(v.expand(B, -1) if getattr(pb, k).dim() == 2 else v.expand(B))
        return pb

    @classmethod
    def synthetic(cls, seed: int, inst0: int, B: int, N: int, M: int | None = None, device=None,
                  transposes: bool = True) -> "ProblemBatch":
        """Synthetic problems inst0..inst0+B-1 of `seed` (the primal behind
        Batch.generate), with Qp and the duals built on the device."""
        M = int(M) if M else max(1, int(N) // 2)
        pb = cls(B, N, M, device, transposes=transposes)
        _check(lib().pqp_batch_synth_primal(seed, inst0, pb.B, pb.N, pb.M, *[pb._p(getattr(pb, k)) for k in
                                                                            cls.PRIMAL], pb._s()))
        return pb.gauss_jordan().convert_to_dual()

    def problem(self, b: int = 0) -> dict:
        """Problem b as a host dict (the keys of solve_dual / Problem)."""
        P = {k: getattr(self, k)[b].cpu().numpy().reshape(-1) for k in self.PRIMAL + self.DUAL + ("Qp",)}
        P.update(N=self.N, M=self.M)
        return P

    def set(self, name: str, values):
        """Per-problem values for one array ([B, ...] numpy/torch)."""
        t = getattr(self, name)
        t.copy_(self.torch.as_tensor(np.asarray(values, np.float32) if not self.torch.is_tensor(values) else values,
                                     device=self.device).reshape(t.shape))
        if name in ("Qd", "Gp", "Qp_inv"):
            self.invalidate()
        return self

    def invalidate(self):
        """Drop the prepared per-problem data.  solve() also notices in-place
        writes to Qd, Gp or Qp_inv by itself (torch's version counters), so
        this is only needed after writes torch cannot see (e.g. from C)."""
        self._prep = None
        return self

    def _source_key(self):
        """What the prepared data were derived from: the storage and torch's
        in-place version counter of Qd, Gp and Qp_inv (``pb.Qd[i] = ...`` or
        ``pb.Gp.copy_(...)`` bump the counter), and the solver the shape takes."""
        L = lib()
        return (tuple((t.data_ptr(), t._version) for t in (self.Qd, self.Gp, self.Qp_inv)),
                L.pqp_batch_solve_path(self.N, self.M), L.pqp_batch_solve_kernel(self.N, self.M))

    def prepare(self):
        """pqp_batch_prepare: what the solver derives from the problems alone
        (symmetry flags, Theta, column-major Qd if needed, Qp_inv', and Gp'
        where k_solve_single will read it), computed once and kept for every
        later solve() until Qd, Gp or Qp_inv change."""
        torch = self.torch
        key = self._source_key()
        path = key[1]
        if path < 0:
            _check(path)
        prep = {"path": path, "key": key}
        if path == 2:
            B, N, M = self.B, self.N, self.M
            f = dict(dtype=torch.float32, device=self.device)
            prep["theta"] = torch.empty(B, N, **f)
            prep["sym"] = torch.empty(B, dtype=torch.int32, device=self.device)
            prep["QdT"] = None
            # k_solve_pipe (pqp_batch_solve_kernel 1) never reads Gp': no B*N*M copy for it
            prep["GpT"] = torch.empty(B, M * N, **f) if self.transposes and key[2] == 0 else None
            prep["QinvT"] = torch.empty(B, M * M, **f) if self.transposes else None
            p = lambda t: self._p(t) if t is not None else None  # noqa: E731
            all_sym = C.c_int(0)
            args = lambda qdt: (B, N, M, self._p(self.Qd), self._p(self.Gp), self._p(self.Qp_inv), qdt,  # noqa: E731
                                self._p(prep["theta"]), self._p(prep["sym"]), p(prep["GpT"]), p(prep["QinvT"]),
                                C.byref(all_sym), self._s())
            rc = lib().pqp_batch_prepare(*args(None))
            if rc == PQP_ERR_NEEDS_QDT:  # some Qd is not bit-symmetric: its column-major copy
                prep["QdT"] = torch.empty(B, N * round_up(N, 4), **f)
                rc = lib().pqp_batch_prepare(*args(self._p(prep["QdT"])))
            _check(rc)
            prep["all_sym"] = bool(all_sym.value)
        self._prep = prep
        return self

    def gauss_jordan(self):
        """Qp = inverse(Qp_inv) per problem (Gauss_Jordan, PQP_CPU.c:251)."""
        _check(lib().pqp_batch_gauss_jordan(self.B, self.M, self._p(self.Qp_inv), self._p(self.Qp), self._s()))
        return self

    def convert_to_dual(self):
        """Qd, Fd, Md from the primal data (convertToDual, PQP_CPU.c:489)."""
        _check(lib().pqp_batch_convert_to_dual(self.B, self.N, self.M, *[self._p(getattr(self, k)) for k in
                                                                         self.PRIMAL + self.DUAL], self._s()))
        return self.invalidate()

    def solve(self, mode: int = MODE_CONVERGE, num_iter: int = 1000, max_updates: int = 0, prepared: bool = True):
        """solveQuadraticDual for every problem; fills Y, U, h, status.  The
        per-problem setup is prepared on the first call and reused
        (prepared=False: pqp_batch_solve, which redoes it every call)."""
        if not prepared:
            _check(lib().pqp_batch_solve(self.B, self.N, self.M, *[self._p(getattr(self, k)) for k in
                                                                  ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp",
                                                                   "Gp", "Kp")],
                                         mode, num_iter, max_updates, self._p(self.Y), self._p(self.U),
                                         self._p(self.h), self._p(self.status), self._s()))
            return self
        if self._prep is None or self._prep["key"] != self._source_key():
            self.prepare()  # first solve, Qd / Gp / Qp_inv written, or a knob moved the size to another solver
        P = self._prep
        p = lambda k: self._p(P[k]) if P.get(k) is not None else None  # noqa: E731
        _check(lib().pqp_batch_solve_prepared(self.B, self.N, self.M, self._p(self.Qd), p("QdT"), p("theta"), p("sym"),
                                              p("GpT"), p("QinvT"),
                                              *[self._p(getattr(self, k)) for k in
                                                ("Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")],
                                              mode, num_iter, max_updates, self._p(self.Y), self._p(self.U),
                                              self._p(self.h), self._p(self.status), self._s()))
        return self


def perturbed_states(x, B: int, seed: int = 5, rel: float = 0.05) -> np.ndarray:
    """B plant states around x ([B, nState] float32): x * (1 + rel * N(0, 1))
    per entry from numpy's seeded generator -- the MPC workload of the bench's
    mpc_batch leg (seed 5), whose every solve is pinned to the reference by
    tests/golden/mpc_states.npz.  Numpy only; no GPU work."""
    x = np.asarray(x, np.float32).reshape(1, -1)
    rng = np.random.default_rng(seed)
    return (x * (1.0 + rel * rng.standard_normal((int(B), x.shape[1])))).astype(np.float32)


def mpc_batch(directory, states, device=None) -> ProblemBatch:
    """The bundled plant (example/*.txt) at B different states x (and the
    file's disturbance D): per-problem Fp = Fp1 D + Fp2 x - Fp3 and Mp
    (computeFp / computeMp), shared Qp_inv, Gp, Kp, then Qp and the duals --
    all on the GPU.  `states` is [B, nState]."""
    import torch

    E = read_example(directory)
    xs = np.ascontiguousarray(np.asarray(states, np.float32).reshape(len(states), -1))
    B, ns = xs.shape
    if ns != E["ns"]:
        raise ValueError(f"states must have {E['ns']} columns")
    pb = ProblemBatch(B, E["N"], E["M"], device)
    dev = pb.device
    T = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=dev).contiguous()  # noqa: E731
    plant = {k: T(E[k]) for k in ("Fp1", "Fp2", "Fp3", "Mp1", "Mp2", "Mp3", "Mp4", "Mp5", "Mp6")}
    x = T(xs)
    D = T(np.tile(E["D"], (B, 1)))
    for k in ("Qp_inv", "Gp", "Kp"):
        getattr(pb, k).copy_(T(E[k]).reshape(1, -1).expand(B, -1))
    p = ProblemBatch._p
    s = pb._s()
    _check(lib().pqp_batch_compute_fp(B, E["M"], E["nd"], ns, p(plant["Fp1"]), p(plant["Fp2"]), p(plant["Fp3"]),
                                      p(D), p(x), p(pb.Fp), s))
    _check(lib().pqp_batch_compute_mp(B, E["nd"], ns, *[p(plant[k]) for k in ("Mp1", "Mp2", "Mp3", "Mp4", "Mp5",
                                                                                "Mp6")], p(D), p(x), p(pb.Mp), s))
    pb.gauss_jordan().convert_to_dual()
    return pb


def horizon_batch(directory, H: int, states, device=None) -> ProblemBatch:
    """B MPC problems over H horizon stages of the bundled plant
    (example/*.txt), each stage at its own state: problem b stacks H copies
    of the plant's constraint set, stage h of it at state states[b, h]
    (``states`` is [B, H, nState] or [B, nState] for one state per problem).
    The primal is block-diagonal -- Qp_inv = diag(Qp_inv, ..., Qp_inv), Gp =
    diag(Gp, ..., Gp), Kp stacked, Fp = the stages' computeFp (PQP_CPU.c:373)
    stacked, Mp = the stages' computeMp (:395) summed in stage order -- and
    the dual is formed on the GPU from it like any other problem: Qp =
    Gauss_Jordan(Qp_inv) (:251) and convertToDual (:489).  n_dual = 28 H,
    M = 7 H.  Setup runs on the device through the C ABI (pqp_batch_compute_fp
    / _mp, pqp_batch_gauss_jordan, pqp_batch_convert_to_dual); torch only
    places the blocks.  Every problem's setup and solve equal the reference's
    (tests/test_gpu_mid.py; the bench's 16384-problem populations at H = 2 and
    4 against tests/golden/horizon_states.npz: at H = 2 16377 stop at h = 313,
    6 at 314, and one never meets the reference's exact-float gap test)."""
    import torch

    E = read_example(directory)
    m, nd, ns, n = E["M"], E["nd"], E["ns"], E["N"]
    H = int(H)
    xs = np.asarray(states, np.float32)
    if xs.ndim == 2:
        xs = np.repeat(xs[:, None, :], H, axis=1)
    if xs.ndim != 3 or xs.shape[1] != H or xs.shape[2] != ns:
        raise ValueError(f"states must be [B, {H}, {ns}] or [B, {ns}]")
    B = xs.shape[0]
    pb = ProblemBatch(B, n * H, m * H, device)
    dev = pb.device
    T = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=dev).contiguous()  # noqa: E731
    plant = {k: T(E[k]) for k in ("Fp1", "Fp2", "Fp3", "Mp1", "Mp2", "Mp3", "Mp4", "Mp5", "Mp6")}
    x = T(xs.reshape(B * H, ns))
    D = T(np.tile(E["D"], (B * H, 1)))
    Fps = torch.empty(B * H, m, dtype=torch.float32, device=dev)
    Mps = torch.empty(B * H, dtype=torch.float32, device=dev)
    p = ProblemBatch._p
    s = pb._s()
    _check(lib().pqp_batch_compute_fp(B * H, m, nd, ns, p(plant["Fp1"]), p(plant["Fp2"]), p(plant["Fp3"]), p(D),
                                      p(x), p(Fps), s))
    _check(lib().pqp_batch_compute_mp(B * H, nd, ns, *[p(plant[k]) for k in ("Mp1", "Mp2", "Mp3", "Mp4", "Mp5",
                                                                               "Mp6")], p(D), p(x), p(Mps), s))
    Qinv, Gp = T(E["Qp_inv"]).reshape(m, m), T(E["Gp"]).reshape(n, m)
    QI = pb.Qp_inv.view(B, H * m, H * m)
    GP = pb.Gp.view(B, H * n, H * m)
    for h in range(H):  # the diagonal blocks (the rest stays +0.0)
        QI[:, h * m:(h + 1) * m, h * m:(h + 1) * m] = Qinv
        GP[:, h * n:(h + 1) * n, h * m:(h + 1) * m] = Gp
    pb.Kp.copy_(T(E["Kp"]).repeat(H).expand(B, -1))
    pb.Fp.copy_(Fps.view(B, H * m))
    Mv = Mps.view(B, H)
    pb.Mp.copy_(Mv[:, 0])
    for h in range(1, H):  # ((Mp_0 + Mp_1) + Mp_2) + ... in fp32, stage order
        pb.Mp.add_(Mv[:, h])
    torch.cuda.current_stream(dev).synchronize()  # the staging tensors go out of scope
    pb.gauss_jordan().convert_to_dual()
    return pb


class RowBlock:
    """Rows [row0, row0+rows) of one large dual problem's updateY2
    (pqp_rowblock_* of include/pqp.h).

    ``update(Y, Y_rows)`` reads the full iterate Y (N floats, device) and
    writes the block's rows of Y_next, bit-identical to the corresponding rows
    of PQP_CPU.c:603-618.  Launches go to torch's current stream of `device`.
    """

    def __init__(self, Qd_rows, Fd, N: int, row0: int, rows: int, ld: int | None = None, device=None):
        import torch

        self.torch = torch
        self.N, self.row0, self.rows = int(N), int(row0), int(rows)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ld = int(ld) if ld else self.N
        dev = lambda a: (a if torch.is_tensor(a) else torch.as_tensor(np.asarray(a, np.float32))).to(  # noqa: E731
            self.device, torch.float32).contiguous()
        Fd = dev(Fd)
        if self.rows > 0:
            Qd_rows = dev(Qd_rows)
            if Qd_rows.numel() < (self.rows - 1) * self.ld + self.N:
                raise ValueError("Qd_rows is smaller than rows x ld")
        h = C.c_void_p()
        _check(lib().pqp_rowblock_create(C.c_void_p(Qd_rows.data_ptr()) if self.rows > 0 else None, self.ld,
                                         C.c_void_p(Fd.data_ptr()), self.N, self.row0, self.rows, self._s(),
                                         C.byref(h)))
        self._h = h

    def _s(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    @classmethod
    def synthetic(cls, seed: int, inst: int, N: int, row0: int, rows: int, M: int | None = None, device=None):
        """The block of synthetic problem `inst` of `seed` (pqp_synth_rows,
        the generator of :meth:`Batch.generate`), generated on the device
        without the full N x N matrix.  Returns (block, Fd, Md) with Fd/Md
        the full problem's (device tensors)."""
        import torch

        device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        M = int(M) if M else max(1, int(N) // 2)
        ld = round_up(int(N), 4)
        kw = dict(dtype=torch.float32, device=device)
        Q = torch.empty(max(1, int(rows)) * ld, **kw)
        Fd = torch.empty(int(N), **kw)
        Md = torch.empty(1, **kw)
        s = C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
        _check(lib().pqp_synth_rows(seed, inst, int(N), M, int(row0), int(rows), C.c_void_p(Q.data_ptr()), ld,
                                    C.c_void_p(Fd.data_ptr()), C.c_void_p(Md.data_ptr()), s))
        blk = cls(Q, Fd, N, row0, rows, ld=ld, device=device)
        return blk, Fd, Md

    def update(self, Y, Y_rows):
        """Y_rows[:rows] = updateY2(Y)[row0:row0+rows] (async)."""
        _check(lib().pqp_rowblock_update(self._h, C.c_void_p(Y.data_ptr()),
                                         C.c_void_p(Y_rows.data_ptr()) if self.rows > 0 else None, self._s()))

    def check(self):
        """Synchronize and raise PQPError if an update since the last check
        hit an expired hand-off wait inside the kernel (its rows are then not
        valid; pqp_rowblock_check)."""
        _check(lib().pqp_rowblock_check(self._h, self._s()))

    def close(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.pqp_rowblock_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
