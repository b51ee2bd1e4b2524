"""The C-ABI library: loads, exports every symbol include/pqp.h declares, and
its host-only pieces (file reader, argument validation) behave like the
reference.  No GPU compute is issued here."""
from __future__ import annotations

import functools
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import EXAMPLE_DIR, ROOT, assert_bitwise

HEADERS = sorted((ROOT / "include").glob("*.h"))
LIBSO = ROOT / "pqp-for-mpc_amd" / "pqp_amd" / "libpqp.so"


def declared_functions() -> list[str]:
    text = "\n".join(h.read_text() for h in HEADERS)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*([A-Za-z_][A-Za-z0-9_]*)\s*\(", text, re.M)
    return sorted(set(names))


def test_header_lists_reference_entry_points():
    names = declared_functions()
    for ref_name in ("solveQuadraticDual", "updateY2", "terminate", "convertToDual", "computeUfromY", "computeCost",
                     "checkFeas", "computeTheta", "matrixMultiply", "Gauss_Jordan", "computeFp", "computeMp",
                     "input"):
        assert ref_name in names


def test_library_exports_every_declared_symbol():
    assert LIBSO.exists(), "libpqp.so not built (run __graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIBSO)], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing


def test_python_mirror_binds_every_symbol():
    import pqp_amd

    assert set(pqp_amd.SIGNATURES) == set(declared_functions())  # every header of include/
    L = pqp_amd.lib()
    for n in declared_functions():
        assert getattr(L, n) is not None
    assert L.pqp_version() >= 105


def declared_arity() -> dict[str, int]:
    """name -> number of parameters of every prototype in include/*.h."""
    text = "\n".join(h.read_text() for h in HEADERS)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*([A-Za-z_][A-Za-z0-9_]*)\s*\(([^)]*)\)\s*;",
                         text, re.M):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_python_mirror_arity_matches_header():
    """Every ctypes binding takes exactly the parameters its prototype declares."""
    import pqp_amd

    arity = declared_arity()
    assert set(arity) == set(pqp_amd.SIGNATURES)
    bad = {n: (len(pqp_amd.SIGNATURES[n][1]), k) for n, k in arity.items() if len(pqp_amd.SIGNATURES[n][1]) != k}
    assert not bad, bad


@functools.lru_cache(maxsize=None)
def _gfx950_asm(name: str) -> str:
    """The gfx950 assembly of one kernel TU, compiled once per session."""
    import tempfile

    hipcc = Path("/opt/rocm/bin/hipcc")
    if not hipcc.exists():
        pytest.skip("hipcc not present")
    src = ROOT / "pqp-for-mpc_amd" / "csrc" / name
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "k.s"
        subprocess.run([str(hipcc), "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fno-fast-math", "--cuda-device-only", "-S", str(src), "-o", str(out)], check=True)
        return out.read_text()


@pytest.mark.parametrize("src,pattern,min_kernels", [
    ("pqp_kernels.hip",
     r"_ZN3pqp(15k_batch_iterate|14k_batch_update|14k_solve_single|13k_split_relay|12k_fixed_tiny"
     r"|12k_solve_wave|12k_lean_relay|12k_solve_pipe|12k_solve_mid2|11k_matmul_pk|14k_matmul_tiled"
     r"|12k_gj_blocked|13k_matvec_rows|8k_vecmat)",
     40),
    ("pqp_wide.hip", r"_ZN3pqp12_GLOBAL__N_1(12k_gemv_relay|13k_wide_decide)", 2),
    ("pqp_persist.hip", r"_ZN3pqp15k_split_persist", 1),
    ("pqp_converge.hip", r"_ZN3pqp12_GLOBAL__N_118k_converge_persist", 1),
])
def test_hot_kernels_compile_for_gfx950_without_fma(src, pattern, min_kernels):
    """The update and terminate() kernels must not contract a*b+c into FMA
    (bit-parity rule): compile each kernel TU for gfx950
    exactly as the Makefile does and inspect the ISA of the hot kernels."""
    asm = _gfx950_asm(src)
    bodies = re.split(r"\n(?=_ZN3pqp[A-Za-z0-9_]*:)", asm)
    hot = [b for b in bodies if re.match(pattern, b)]
    assert len(hot) >= min_kernels, f"hot kernels of {src} not found in the gfx950 assembly ({len(hot)})"
    for body in hot:
        name = body.split(":", 1)[0]
        body = body.split(".Lfunc_end", 1)[0]
        # the only f32 FMAs allowed are the 5 inside each IEEE-correct division
        # expansion (v_div_scale .. v_div_fmas .. v_div_fixup); none may come
        # from contracting the solver's own products and sums
        n_div = len(re.findall(r"\bv_div_fixup_f32", body))
        n_fma = len(re.findall(r"\bv_(fma|fmac|mad|mac|pk_fma)_f32", body))
        assert n_fma == 5 * n_div, f"{name}: {n_fma} FMAs for {n_div} divisions"


@pytest.mark.parametrize("src,name", [
    ("pqp_persist.hip", "_ZN3pqp15k_split_persistILb0EEEvPKfS2_iiS2_PfPyPiS4_iii"),
    # the headline kernel: its register blocks pinned in AGPRs across the
    # launch (pqp_kernels.hip k_batch_resident) must stay there
    ("pqp_kernels.hip", "_ZN3pqp16k_batch_residentILi16ELi2ELi2EEEvPKfxiS2_S2_iS2_Pfi"),
    ("pqp_converge.hip", "_ZN3pqp12_GLOBAL__N_118k_converge_persistILb0EEEvNS_6CvArgsE"),
    ("pqp_kernels.hip", "_ZN3pqp12k_solve_pipeILi256ELi2ELi16ELi2ELb1EEEvNS_9SolveArgsEPNS_10SolveStateE"),
    ("pqp_kernels.hip", "_ZN3pqp12k_solve_pipeILi256ELi2ELi16ELi2ELb0EEEvNS_9SolveArgsEPNS_10SolveStateE"),
])
def test_persistent_kernels_do_not_spill(src, name):
    """The persistent launches hold a whole slice of products in registers
    (up to 196 VGPRs) at 6 waves per workgroup, i.e. 256 VGPRs per lane: a
    spill to scratch costs 0.3 us per update (measured on k_converge_persist),
    so the default instantiations must have no scratch.  k_solve_pipe's
    builds at two workgroups per CU (up to 256 VGPRs: a 128 x 96 Gp tile, or two
    64 x 64 ones, and 16 update loads per lane in flight) must not spill either,
    nor may k_batch_resident's AGPR-held Qd blocks."""
    asm = _gfx950_asm(src)
    i = asm.index("\n" + name + ":")
    m = re.search(r"; ScratchSize: (\d+)", asm[i:])
    assert m, f"{name}: no ScratchSize note"
    assert int(m.group(1)) == 0, f"{name} spills {m.group(1)} bytes per lane"


def test_read_example_matches_oracle_loader(orc):
    import pqp_amd

    got = pqp_amd.read_example(EXAMPLE_DIR)
    exp = orc.load_example(EXAMPLE_DIR)
    for k in ("Qp_inv", "Fp1", "Fp2", "Fp3", "Mp1", "Mp2", "Mp3", "Mp4", "Mp5", "Mp6", "Gp", "Kp", "x", "D"):
        assert_bitwise(got[k], exp[k], k)
    assert got["N"] == 28 and got["M"] == 7


def test_read_example_missing_file_is_an_error(tmp_path):
    import pqp_amd

    with pytest.raises(pqp_amd.PQPError) as ei:
        pqp_amd.read_example(tmp_path)
    assert ei.value.code == pqp_amd.PQP_ERR_IO
    assert "Qp_inv.txt" in str(ei.value)


def test_read_example_short_file_is_an_error(tmp_path):
    import shutil

    import pqp_amd

    for f in EXAMPLE_DIR.glob("*.txt"):
        shutil.copy(f, tmp_path / f.name)
    (tmp_path / "Kp.txt").write_text("1.0 2.0 #")
    with pytest.raises(pqp_amd.PQPError) as ei:
        pqp_amd.read_example(tmp_path)
    assert ei.value.code == pqp_amd.PQP_ERR_IO and "Kp.txt" in str(ei.value)


def test_python_buffers_are_validated():
    import pqp_amd

    with pytest.raises(TypeError):
        pqp_amd.computeTheta(np.zeros(4, np.float64), np.zeros(4, np.float32), 2)


def test_reference_main_driver_links_libpqp_first():
    """oracle/_ref/ref_main_on_libpqp resolves the reference main()'s calls to
    libpqp: libpqp.so must precede libpqp_ref.so in its DT_NEEDED order."""
    exe = ROOT / "oracle" / "_ref" / "ref_main_on_libpqp"
    if not exe.exists():
        pytest.skip("needs /root/reference at build time")
    dyn = subprocess.run(["readelf", "-d", str(exe)], capture_output=True, text=True, check=True).stdout
    needed = re.findall(r"Shared library: \[([^\]]+)\]", dyn)
    assert needed.index("libpqp.so") < needed.index("libpqp_ref.so")
    ref_syms = subprocess.run(["nm", "-D", "--defined-only", str(ROOT / "oracle/_ref/libpqp_ref.so")],
                              capture_output=True, text=True, check=True).stdout
    ours = set(declared_functions())
    called_by_main = {"input", "Gauss_Jordan", "computeFp", "computeMp", "convertToDual", "solveQuadraticDual",
                      "computeUfromY", "computeCost"}
    assert called_by_main <= ours
    assert all(f" {n}\n" in ref_syms for n in called_by_main)


def test_dropin_input_reads_example_from_cwd(tmp_path, monkeypatch, orc):
    """input() (PQP_CPU.c:757) reads ./example relative to the CWD; host I/O."""
    import shutil

    import pqp_amd

    shutil.copytree(EXAMPLE_DIR, tmp_path / "example")
    monkeypatch.chdir(tmp_path)
    m, nd, ns, no = 7, 1, 29, 7
    z = lambda n: np.zeros(n, np.float32)  # noqa: E731
    A = dict(qp_inv=z(m * m), Fp1=z(m * nd), Fp2=z(m * ns), Fp3=z(m), Mp1=z(ns * ns), Mp2=z(nd * ns), Mp3=z(nd * nd),
             Mp4=z(ns), Mp5=z(nd), Mp6=z(1), Gp=z(4 * m * m), Kp=z(4 * m), x=z(ns), D=z(nd), theta=z(no * nd),
             Z=z(no * ns))
    pqp_amd.lib().input(*[pqp_amd._buf(v) for v in A.values()])
    exp = orc.load_example(tmp_path / "example")
    assert_bitwise(A["qp_inv"], exp["Qp_inv"], "Qp_inv")
    for k in ("Fp1", "Fp2", "Fp3", "Mp1", "Mp2", "Mp3", "Mp4", "Mp5", "Mp6", "Gp", "Kp", "x", "D"):
        assert_bitwise(A[k], exp[k], k)
    assert A["Z"].any()  # read although unused by the solver (PQP_CPU.c:889-899)


def test_tuning_knobs_roundtrip():
    """The keyed tuning interface (include/pqp_tuning.h): every knob sets and
    reads back, the previous value is returned, unknown keys are errors, and
    the Python knob names map onto it.  Host-only (no GPU work)."""
    import ctypes as C

    import pqp_amd

    L = pqp_amd.lib()
    for key in ("persist_off", "lean_min_n", "batch_opts", "converge_chunk", "wide_min_n", "pipe_off",
                "pipe_variant", "pipe_force", "mid_v1", "matmul_pk_off", "iterate_kind", "tiny_chunk", "tiny_fallback",
                "tiny_np", "tiny_apoll", "tiny_ablk", "persist_xcds", "converge_xcds"):
        old = pqp_amd.tune_get(key)
        assert pqp_amd.tune(key, old + 3) == old
        assert pqp_amd.tune_get(key) == old + 3
        assert pqp_amd.tune(key, old) == old + 3
    assert pqp_amd.tune("relay_spin_max", 2**40) == 1 << 20 and pqp_amd.tune_get("relay_spin_max") == 1 << 30
    pqp_amd.tune("relay_spin_max", 0)
    assert pqp_amd.tune_get("relay_spin_max") == 1 << 20
    for gone in ("no_such_knob", "split_kind", "split_u", "fixed_tiny_old", "single_occ4", "wide_flags", "mid_split",
                 "iterate_v1", "gj_v1", "mid2_fat", "matvec_lds"):
        with pytest.raises(pqp_amd.PQPError):  # rounds 4 and 6 removed the measured-slower arms behind these
            pqp_amd.tune(gone, 1)
    prev = L.pqp_tune_set_variant((3 << 17) | 0x200)
    assert pqp_amd.tune_get("split_lw") == 32
    assert pqp_amd.tune_get("force_single") == 1
    assert L.pqp_tune_set_variant(prev) == (3 << 17) | 0x200
    with pytest.raises(pqp_amd.PQPError):  # a retired arm's bit is refused, not dropped
        L.pqp_tune_set_variant(0x1000)
    # the batched launch's chunk as the library sizes it (bench.py reads it)
    assert pqp_amd.batch_chunk_for(1024, 512) == int((1 << 28) / (3.0 * 1024 * 1024 + 2.0 * 1024 * 512 + 2.0 * 512 * 512 + 1))
    old_bc = pqp_amd.tune("batch_chunk", 7)
    try:
        assert pqp_amd.batch_chunk_for(1024, 512) == 7
    finally:
        pqp_amd.tune("batch_chunk", old_bc)
    assert L.pqp_tune_batch_converge(1 | 4 | 16) == 0 and pqp_amd.tune_get("single_scalar") == 1
    assert L.pqp_tune_batch_converge(0) == 1 | 4 | 16
    fb = C.c_longlong(-1)
    assert L.pqp_tune_last_path(C.byref(fb)) == 0 and fb.value == 0
    assert L.pqp_tune_converge_grid(1024, 512) > 0 and L.pqp_tune_converge_grid(28, 7) > 0
    assert pqp_amd.tune_get("last_batch_kernel") == 0  # no path-2 launch on this thread yet
