"""ctypes binding of ``libfedagg.so`` (the C ABI declared in ``include/fedagg.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``hipcc --offload-arch=gfx950``).
There is deliberately no fallback: if the shared object is missing or does not load, every
aggregation call raises :class:`NativeLibraryError` -- the engine never silently computes on
the CPU or through another backend.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("FEDAGG_LIB", str(_HERE / "libfedagg.so")))

c_u64 = ctypes.c_uint64
c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_void = ctypes.c_void_p
c_dbl = ctypes.c_double
c_size = ctypes.c_size_t
P = ctypes.POINTER

# Every symbol include/fedagg.h declares, with its ctypes signature.
SIGNATURES = {
    "fedagg_abi_version": (c_int, []),
    "fedagg_last_error": (ctypes.c_char_p, []),
    "fedagg_tune": (c_int, [ctypes.c_char_p, ctypes.c_longlong]),
    "fedagg_tuning_build": (c_int, []),
    "fedagg_pairwise_ws_bytes": (c_size, [c_int, c_int, c_int]),
    "fedagg_fedavg_f32": (c_int, [P(c_void), P(ctypes.c_float), c_int, c_u64, P(c_u64), c_int, c_void, c_void, c_void]),
    "fedagg_fedavg_bf16": (c_int, [P(c_void), P(ctypes.c_float), c_int, c_u64, P(c_u64), c_int, c_void, c_void, c_void]),
    "fedagg_fedavg_tile_vectors_f32": (c_u64, [c_int, c_u64]),
    "fedagg_fedavg_tile_vectors_bf16": (c_u64, [c_int, c_u64]),
    "fedagg_fedavg_tiled_f32": (c_int, [c_void, P(ctypes.c_float), c_int, c_u64, c_u64, P(c_u64), c_int, c_void, c_void,
                                        c_void]),
    "fedagg_fedavg_tiled_bf16": (c_int, [c_void, P(ctypes.c_float), c_int, c_u64, c_u64, P(c_u64), c_int, c_void,
                                         c_void, c_void]),
    "fedagg_fedavg_f64": (c_int, [P(c_void), P(c_dbl), c_int, c_u64, P(c_u64), c_int, c_void, c_void, c_void]),
    "fedagg_fedavg_f16": (c_int, [P(c_void), P(ctypes.c_uint16), c_int, c_u64, P(c_u64), c_int, c_void, c_void, c_void]),
    "fedagg_scaffold_launches": (c_int, [c_int, c_int, c_u64, c_int]),
    "fedagg_scaffold_f32": (
        c_int,
        [P(c_void), P(c_void), c_void, P(c_dbl), c_int, c_u64, P(c_u64), c_int, c_void, c_dbl, c_void, c_void, c_void],
    ),
    "fedagg_scaffold_f64": (
        c_int,
        [P(c_void), P(c_void), c_void, P(c_dbl), c_int, c_u64, P(c_u64), c_int, c_void, c_dbl, c_void, c_void, c_void],
    ),
    "fedagg_equal_count_f32": (c_int, [P(c_void), c_int, c_u64, c_void, c_void]),
    "fedagg_equal_count_f64": (c_int, [P(c_void), c_int, c_u64, c_void, c_void]),
    "fedagg_read_probe_f32": (c_int, [c_void, c_u64, c_void, c_int, c_void]),
    "fedagg_read_probe_tile_f32": (c_int, [c_void, c_u64, c_void, c_int, c_void]),
    "fedagg_cast": (c_int, [c_void, c_int, c_void, c_int, c_u64, c_void]),
    "fedagg_flat_gather_f32": (c_int, [P(c_void), P(c_u64), c_int, c_void, c_void]),
    "fedagg_flat_scatter_f32": (c_int, [P(c_void), P(c_u64), c_int, c_void, c_void]),
    "fedagg_flat_wsum_f32": (c_int, [P(c_void), c_int, P(c_dbl), P(c_u64), c_int, c_void, c_void]),
    "fedagg_flat_increment_f32": (c_int, [P(c_void), P(c_u64), c_int, c_void, c_dbl, c_void]),
    "fedagg_flat_gather": (c_int, [P(c_void), c_int, P(c_u64), c_int, c_void, c_void]),
    "fedagg_flat_wsum": (c_int, [P(c_void), P(c_int), c_int, P(c_dbl), P(c_u64), c_int, c_void, c_int, c_void]),
    "fedagg_flat_increment": (c_int, [P(c_void), P(c_u64), c_int, c_void, c_int, c_dbl, c_void]),
    "fedagg_scale_cast": (c_int, [c_void, c_int, c_dbl, c_void, c_int, c_u64, c_void]),
    # client-sharded building blocks (chain / split pairwise trees)
    "fedagg_fedavg_chain_f32": (c_int, [P(c_void), P(ctypes.c_float), c_int, c_u64, c_int, c_void, c_void]),
    "fedagg_fedavg_chain_push_f32": (c_int, [P(c_void), P(ctypes.c_float), c_int, c_u64, c_void, c_void, c_void]),
    "fedagg_fedavg_chain_push_bf16": (c_int, [P(c_void), P(ctypes.c_float), c_int, c_u64, c_void, c_void, c_void]),
    "fedagg_fedavg_chain_bf16": (c_int, [P(c_void), P(ctypes.c_float), c_int, c_u64, c_int, c_void, c_void]),
    "fedagg_scaffold_chain_push_f32": (c_int, [P(c_void), P(c_dbl), c_int, c_u64, c_int, c_void, c_dbl, c_int, c_void,
                                               c_void, c_void]),
    "fedagg_scaffold_chain_push_f64": (c_int, [P(c_void), P(c_dbl), c_int, c_u64, c_int, c_void, c_dbl, c_int, c_void,
                                               c_void, c_void]),
    "fedagg_fedavg_chain_f64": (c_int, [P(c_void), P(c_dbl), c_int, c_u64, c_int, c_void, c_void]),
    "fedagg_fedavg_chain_f16": (c_int, [P(c_void), P(ctypes.c_uint16), c_int, c_u64, c_int, c_void, c_void]),
    "fedagg_fedavg_chain_tiled_f32": (c_int, [c_void, P(ctypes.c_float), c_int, c_u64, c_u64, c_int, c_void, c_void]),
    "fedagg_fedavg_chain_tiled_bf16": (c_int, [c_void, P(ctypes.c_float), c_int, c_u64, c_u64, c_int, c_void, c_void]),
    "fedagg_pairwise_products_f32": (c_int, [P(c_void), P(ctypes.c_float), c_int, P(c_u64), c_int, c_i64, c_int,
                                             c_void, c_void]),
    "fedagg_pairwise_products_bf16": (c_int, [P(c_void), P(ctypes.c_float), c_int, P(c_u64), c_int, c_i64, c_int,
                                              c_void, c_void]),
    "fedagg_pairwise_products_f64": (c_int, [P(c_void), P(c_dbl), c_int, P(c_u64), c_int, c_i64, c_int, c_void,
                                             c_void]),
    "fedagg_pairwise_products_f16": (c_int, [P(c_void), P(ctypes.c_uint16), c_int, P(c_u64), c_int, c_i64, c_int,
                                             c_void, c_void]),
    "fedagg_pairwise_finish_f32": (c_int, [c_void, c_i64, c_i64, P(c_u64), c_int, c_void, c_void]),
    "fedagg_pairwise_finish_f64": (c_int, [c_void, c_i64, c_i64, P(c_u64), c_int, c_void, c_void]),
    "fedagg_pairwise_finish_f16": (c_int, [c_void, c_i64, c_i64, P(c_u64), c_int, c_void, c_void]),
    "fedagg_scaffold_chain_f32": (c_int, [P(c_void), P(c_void), c_void, P(c_dbl), c_int, c_u64, c_int, c_int, c_dbl,
                                          c_void, c_void, c_void]),
    "fedagg_scaffold_chain_f64": (c_int, [P(c_void), P(c_void), c_void, P(c_dbl), c_int, c_u64, c_int, c_int, c_dbl,
                                          c_void, c_void, c_void]),
    "fedagg_scaffold_products_f32": (c_int, [P(c_void), P(c_void), P(c_dbl), c_int, c_int, c_int, P(c_u64), c_int,
                                             c_void, c_void]),
    "fedagg_scaffold_products_f64": (c_int, [P(c_void), P(c_void), P(c_dbl), c_int, c_int, c_int, P(c_u64), c_int,
                                             c_void, c_void]),
    "fedagg_scaffold_finish_f32": (c_int, [c_void, c_int, c_void, P(c_u64), c_int, c_dbl, c_void, c_void, c_void]),
    "fedagg_scaffold_finish_f64": (c_int, [c_void, c_int, c_void, P(c_u64), c_int, c_dbl, c_void, c_void, c_void]),
    # native lockstep executor over RCCL (csrc/lockstep.hip)
    "fedagg_comm_unique_id": (c_int, [ctypes.c_char_p, c_void]),
    "fedagg_comm_create": (c_int, [ctypes.c_char_p, c_int, c_int, c_void, c_int, P(c_void)]),
    "fedagg_comm_destroy": (c_int, [c_void]),
    "fedagg_comm_abort": (c_int, [c_void]),
    "fedagg_comm_async_error": (c_int, [c_void]),
    "fedagg_comm_count": (c_int, [c_void, P(c_int)]),
    "fedagg_comm_last_error": (ctypes.c_char_p, []),
    "fedagg_lockstep_execute": (c_int, [c_void, c_void, c_int, c_void, c_int, c_int, c_void, c_u64, c_int, c_int,
                                        c_void]),
    # push executor (csrc/lockstep.hip; substrafl_amd/push.py)
    "fedagg_ipc_get": (c_int, [c_void, c_void, P(c_u64)]),
    "fedagg_ipc_open": (c_int, [c_void, P(c_void)]),
    "fedagg_ipc_close": (c_int, [c_void]),
    "fedagg_host_map": (c_int, [c_void, c_u64, P(c_void)]),
    "fedagg_host_unmap": (c_int, [c_void]),
    "fedagg_wall_clock_hz": (c_int, [P(c_u64)]),
    "fedagg_device_alloc_uncached": (c_int, [c_u64, P(c_void)]),
    "fedagg_device_free": (c_int, [c_void]),
    "fedagg_push_execute": (c_int, [c_void, c_int, c_void, c_int, c_void, c_int, c_int, c_void, c_int, c_int, c_u64,
                                    c_u64, c_void, c_void, c_u64, c_int, c_void, c_void, c_int, c_void, c_int, c_void]),
    "fedagg_session_create": (c_void, [c_int]),
    "fedagg_session_destroy": (None, [c_void]),
    "fedagg_session_stream": (c_void, [c_void]),
    "fedagg_session_set": (c_int, [c_void, ctypes.c_char_p, ctypes.c_longlong]),
    "fedagg_session_affinity": (c_int, [c_void, P(c_int), c_int]),
    "fedagg_session_ring_node": (c_int, [c_void]),
    "fedagg_device_pci_bus_id": (c_int, [c_int, ctypes.c_char_p, c_int]),
    "fedagg_session_buffer": (c_int, [c_void, c_int, c_u64, P(c_void)]),
    "fedagg_session_warm": (c_int, [c_void, P(c_u64), c_int]),
    "fedagg_session_stage": (c_int, [c_void, c_void, c_u64, c_int, c_int, P(c_void), P(c_u64)]),
    "fedagg_session_stage_range": (c_int, [c_void, c_void, c_u64, c_int, c_int, P(c_void), P(c_u64), c_u64, c_u64]),
    "fedagg_session_stage_tiled": (c_int, [c_void, c_void, c_u64, c_int, c_int, P(c_void), P(c_u64)]),
    "fedagg_session_stage_tiled_row": (c_int, [c_void, c_void, c_u64, c_int, c_int, c_int, P(c_void), P(c_u64)]),
    "fedagg_session_stage_check": (c_int, [c_void, c_void, c_int, c_int, P(c_void), P(c_u64), c_u64, c_u64, c_int,
                                           P(c_u64)]),
    "fedagg_session_event_record": (c_int, [c_void, c_int]),
    "fedagg_session_event_elapsed": (c_int, [c_void, c_int, c_int, P(ctypes.c_float)]),
    "fedagg_session_activate": (c_int, [c_void]),
    "fedagg_device_count": (c_int, []),
    "fedagg_device_get": (c_int, [P(c_int)]),
    "fedagg_device_set": (c_int, [c_int]),
    "fedagg_device_memory": (c_int, [c_int, P(c_u64), P(c_u64)]),
    "fedagg_session_fetch": (c_int, [c_void, c_void, c_void, c_u64]),
    "fedagg_session_memset": (c_int, [c_void, c_void, c_int, c_u64]),
    "fedagg_session_copy_d2d": (c_int, [c_void, c_void, c_void, c_u64]),
    "fedagg_session_sync": (c_int, [c_void]),
    "fedagg_session_timing": (c_int, [c_void, P(c_dbl), P(c_dbl)]),
    "fedagg_session_phases": (c_int, [c_void, P(c_dbl), c_int]),
    # one process, several GPUs (csrc/multi.hip)
    "fedagg_multi_create": (c_void, [c_int, P(c_int), c_int]),
    "fedagg_multi_destroy": (None, [c_void]),
    "fedagg_multi_set": (c_int, [c_void, ctypes.c_char_p, ctypes.c_longlong]),
    "fedagg_multi_fedavg_f32": (c_int, [c_void, c_int, c_int, P(c_void), P(c_u64), c_void, c_void, c_int, c_void]),
    "fedagg_multi_fedavg_f64": (c_int, [c_void, c_int, c_int, P(c_void), P(c_u64), c_void, c_void, c_int, c_void]),
    "fedagg_multi_fedavg_f16": (c_int, [c_void, c_int, c_int, P(c_void), P(c_u64), c_void, c_void, c_int, c_void]),
    "fedagg_multi_shard_info": (c_int, [c_void, c_int, P(c_int), P(c_int), P(c_int), P(c_int), P(c_u64), P(c_u64),
                                        P(c_int)]),
}

# entry points only a FEDAGG_TUNING build exports (include/fedagg.h "#if FEDAGG_TUNING"): bound
# when the loaded library is one, absent from the product library
TUNING_SIGNATURES = {
    "fedagg_copy_async": (c_int, [c_void, c_void, c_u64, c_void]),
}

ABI_VERSION = 17
FEDAGG_KCHUNK = 128
FEDAGG_KCHUNK_SCAFFOLD = 64
FEDAGG_FUSED_PAIRWISE = 16
FEDAGG_TILE_VECTORS_F32 = 8192
FEDAGG_TILE_VECTORS_F32_FEW = 2048
FEDAGG_TILE_VECTORS_BF16 = 4096
FEDAGG_MAX_PAIRWISE = 64
FEDAGG_FLAT_MAX_LISTS = 4
FEDAGG_SESSION_BUFFERS = 16
FEDAGG_SESSION_EVENTS = 8
FEDAGG_SESSION_PHASES = 6
FEDAGG_F16 = 0  # kinds (include/fedagg.h enum)
FEDAGG_F32 = 1
FEDAGG_F64 = 2
FEDAGG_BF16 = 12
FEDAGG_RUN_FEDAVG, FEDAGG_RUN_FEDAVG_TILED, FEDAGG_RUN_SCAFFOLD, FEDAGG_RUN_FEDAVG_PUSH = 0, 1, 2, 3
FEDAGG_RUN_SCAFFOLD_PUSH_DELTA, FEDAGG_RUN_SCAFFOLD_PUSH_CV = 4, 5


class NativeLibraryError(RuntimeError):
    """libfedagg.so is missing, failed to load, or a call returned an error code."""


_lib: Optional[ctypes.CDLL] = None


def load() -> ctypes.CDLL:
    """Load (once) and return the native library; raise loudly if it is not there."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). The aggregation engine has no CPU fallback."
        )
    try:
        lib = ctypes.CDLL(str(LIB_PATH))
    except OSError as e:  # pragma: no cover - depends on the box
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    sigs = dict(SIGNATURES)
    if lib.fedagg_tuning_build():
        sigs.update(TUNING_SIGNATURES)
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.fedagg_abi_version() != ABI_VERSION:
        raise NativeLibraryError("libfedagg ABI version mismatch")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().fedagg_last_error().decode(errors="replace")
        raise NativeLibraryError(f"{what} failed ({rc}): {msg}")


def ptr_array(ptrs) -> ctypes.Array:
    arr = (c_void * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = int(p)
    return arr


def tuning_build() -> bool:
    """Whether the loaded library is a FEDAGG_TUNING build (every experiment variant and knob;
    ``FEDAGG_LIB=substrafl_amd/libfedagg_tuning.so``, built by ``build(tuning=True)``)."""
    return bool(load().fedagg_tuning_build())


def tune(**knobs) -> None:
    """Set launch knobs of the library (``fedagg_tune``, include/fedagg.h): the product knobs, and
    in a tuning build the experiment knobs."""
    lib = load()
    for k, v in knobs.items():
        check(lib.fedagg_tune(k.encode(), int(v)), f"fedagg_tune({k})")
