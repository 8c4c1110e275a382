"""The C-ABI library loads and exports every symbol include/fedagg.h declares (CPU only: no
kernel is launched; argument validation returns before any HIP call)."""

import ctypes
import re
from pathlib import Path

import pytest

from substrafl_amd import _native

HEADER = Path(__file__).resolve().parents[1] / "include" / "fedagg.h"


def declared_functions(tuning: bool = False):
    """The functions include/fedagg.h declares for the product library (``tuning``: the
    ``#if FEDAGG_TUNING`` block's instead)."""
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    blocks = re.findall(r"^#if FEDAGG_TUNING\n(.*?)^#endif", text, flags=re.S | re.M)
    text = "".join(blocks) if tuning else re.sub(r"^#if FEDAGG_TUNING\n.*?^#endif", "", text, flags=re.S | re.M)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(fedagg_[a-z0-9_]+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_abi():
    names = declared_functions()
    assert "fedagg_fedavg_f32" in names and "fedagg_scaffold_f32" in names
    assert len(names) >= 12


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(str(_native.LIB_PATH))
    for name in declared_functions():
        assert hasattr(lib, name), name
    # and the ctypes binding covers exactly the declared set
    assert sorted(_native.SIGNATURES) == declared_functions()


def test_product_library_does_not_export_tuning_entry_points():
    """Experiment-only entry points (VERDICT r04 "Next 7": the runtime copy round 3 suspected in
    the relay failure) live in the FEDAGG_TUNING build only."""
    tuning = declared_functions(tuning=True)
    assert tuning == ["fedagg_copy_async"] == sorted(_native.TUNING_SIGNATURES)
    lib = ctypes.CDLL(str(_native.LIB_PATH))
    assert lib.fedagg_tuning_build() == 0
    for name in tuning:
        assert not hasattr(lib, name), name


def test_abi_version_and_invalid_arguments():
    lib = _native.load()
    assert lib.fedagg_abi_version() == _native.ABI_VERSION == 17
    w = (ctypes.c_float * 1)(1.0)
    ptrs = _native.ptr_array([0])
    assert lib.fedagg_fedavg_f32(ptrs, w, 0, 16, None, 0, None, None, None) == -1  # K == 0
    assert b"K must be > 0" in lib.fedagg_last_error()
    assert lib.fedagg_fedavg_f32(ptrs, w, 1, 16, None, 0, None, None, None) == -1  # NULL out
    idx = (ctypes.c_uint64 * 1)(16)
    assert lib.fedagg_fedavg_f32(ptrs, w, 1, 16, idx, 1, None, 64, None) == -1  # index out of range
    assert b"out of range" in lib.fedagg_last_error()
    assert lib.fedagg_pairwise_ws_bytes(8, 3, 4) == 2 * 64 * 9 * 8
    # read-ceiling probes: arguments are checked before any launch
    assert lib.fedagg_read_probe_tile_f32(None, 4096, None, 4, None) == -1
    assert lib.fedagg_read_probe_tile_f32(256, 4096, 256, 5, None) == -1  # vpt must be 4, 8 or 16
    assert b"read_probe_tile" in lib.fedagg_last_error()
    assert lib.fedagg_tune(b"no_such_knob", 1) == -1
    assert lib.fedagg_tune(b"grid_cap", 4096) == 0
    assert lib.fedagg_tune(b"grid_cap", 0) == 0
    # Scaffold launch plan under the default tuning (no HIP call): one bucket per launch from 16
    # fp32 clients and for fp64 inputs, the fused walk below 16 fp32 clients or unaligned operands
    assert lib.fedagg_scaffold_launches(16, 4, 25_000_000, 1) == 2
    assert lib.fedagg_scaffold_launches(8, 4, 25_000_000, 1) == 1
    assert lib.fedagg_scaffold_launches(8, 8, 25_000_000, 1) == 2
    assert lib.fedagg_scaffold_launches(16, 4, 25_000_000, 0) == 1
    assert lib.fedagg_scaffold_launches(16, 2, 25_000_000, 1) == -1
    assert lib.fedagg_tune(b"sc_2l", 0) == 0
    assert lib.fedagg_scaffold_launches(16, 4, 25_000_000, 1) == 1
    assert lib.fedagg_tune(b"sc_2l", -1) == 0
    # kind-generic flat ops: operand kinds are checked before any HIP call
    numel = (ctypes.c_uint64 * 1)(4)
    kinds = (ctypes.c_int * 2)(_native.FEDAGG_F32, _native.FEDAGG_F64)
    two = _native.ptr_array([16, 32])
    c2 = (ctypes.c_double * 2)(1.0, -1.0)
    assert lib.fedagg_flat_wsum(two, kinds, 2, c2, numel, 1, 64, _native.FEDAGG_F32, None) == -1  # must be f64
    assert b"promoted kind" in lib.fedagg_last_error()
    assert lib.fedagg_flat_wsum(two, kinds, 5, c2, numel, 1, 64, _native.FEDAGG_F64, None) == -1  # > 4 lists
    assert lib.fedagg_flat_increment(two, numel, 1, 64, _native.FEDAGG_F16, 1.0, None) == -1
    assert lib.fedagg_flat_gather(two, _native.FEDAGG_F64, numel, 1, None, None) == -1
    with pytest.raises(_native.NativeLibraryError):
        _native.check(-1, "x")


def test_missing_library_is_loud(monkeypatch, tmp_path):
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", tmp_path / "nope.so")
    with pytest.raises(_native.NativeLibraryError, match="no CPU fallback"):
        _native.load()


def _build_c_demo(tmp_path, name="fedavg_abi_demo"):
    """Compile tests/c/<name>.c with gcc against include/fedagg.h and libfedagg.so: the header is
    plain C and the library links without any HIP or Python headers."""
    import shutil
    import subprocess

    root = HEADER.parents[1]
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not available")
    exe = tmp_path / name
    libdir = _native.LIB_PATH.parent
    subprocess.run([gcc, "-O2", "-ffp-contract=off", "-Wall", "-Werror", f"-I{root / 'include'}",
                    str(root / "tests" / "c" / f"{name}.c"), f"-L{libdir}", "-lfedagg",
                    f"-Wl,-rpath,{libdir}", "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(exe)], check=True)
    return exe


def test_c_demo_compiles_against_the_header(tmp_path):
    assert _build_c_demo(tmp_path).exists()
    assert _build_c_demo(tmp_path, "fedavg_multi_demo").exists()


def test_multi_entry_rejects_bad_arguments():
    """fedagg_multi_* (VERDICT r05 "Next 5"): argument checks return before any HIP call."""
    lib = _native.load()
    assert lib.fedagg_multi_create(0, None, 0) is None
    assert b"ndev" in lib.fedagg_last_error()
    devs = (ctypes.c_int * 1)(0)
    assert lib.fedagg_multi_create(1, devs, -1) is None
    assert lib.fedagg_multi_fedavg_f32(None, 1, 0, None, None, None, None, 0, None) == -1
    assert b"invalid argument" in lib.fedagg_last_error()
    assert lib.fedagg_multi_set(None, b"max_shard_bytes", 1) == -1
    assert lib.fedagg_multi_shard_info(None, 0, None, None, None, None, None, None, None) == -1


@pytest.mark.gpu
def test_c_demo_runs_bit_exact(tmp_path):
    import subprocess

    exe = _build_c_demo(tmp_path)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches=0" in r.stdout


@pytest.mark.gpu
def test_c_multi_demo_runs_bit_exact(tmp_path):
    """The one-call multi-device entry from plain C, two shards on GPU 0 (each its own session,
    several sub-ranges each): bit-identical to the single-device call and to the reference order."""
    import subprocess

    exe = _build_c_demo(tmp_path, "fedavg_multi_demo")
    r = subprocess.run([str(exe), "0", "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches=0 again=0 vs_reference_order=0 f64=0 bad_device_refused=1" in r.stdout, r.stdout
    assert "used=2" in r.stdout, r.stdout


def _declared_arity():
    """Function name -> number of parameters, from include/fedagg.h (comments stripped)."""
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = {}
    for m in re.finditer(r"(fedagg_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_ctypes_binding_matches_every_declared_arity():
    """Each ctypes binding takes as many arguments as its C declaration (a signature that drifted,
    like fedagg_push_execute's landing-tag arguments of ABI 13 or its copy table of ABI 14, would shift every argument after it)."""
    arity = _declared_arity()
    assert "fedagg_push_execute" in arity and arity["fedagg_push_execute"] == 22
    bad = {n: (arity[n], len(_native.SIGNATURES[n][1])) for n in arity
           if n in _native.SIGNATURES and arity[n] != len(_native.SIGNATURES[n][1])}
    assert not bad, bad
