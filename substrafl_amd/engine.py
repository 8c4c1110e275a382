"""Aggregation engine: HBM buckets, HIP streams and launches of the libfedagg kernels.

Two entry levels:

* Device-resident plans (``FedAvgPlan`` / ``ScaffoldPlan``): client buckets already in HBM as
  one ``[K, ld]`` tensor or K device pointers; ``plan.launch(stream)`` enqueues the bucket kernel
  (with the numel == 1 pairwise patch fused in).  This is what ``bench.py`` times
  (BASELINE.json metric).
* Host entry (``AggregationEngine.fedavg`` / ``.scaffold``, plus ``.ingest`` and ``.prewarm``):
  the drop-in path behind ``FedAvg.avg_shared_states`` / ``Scaffold.avg_shared_states``.  Shared
  states arrive as host NumPy arrays (unpickled by ``RemoteMethod.generic_function``,
  substrafl/remote/substratools_methods.py:54-66); the native session (:mod:`runtime`) packs
  them through its pinned ring into HBM, the kernels reduce them, and one D2H copy brings the
  result home as per-layer views of one owned array.  No PyTorch on this path.  A call whose
  buckets exceed the GPU's HBM budget is streamed through it in parameter ranges
  (:mod:`multi_device`), and ``engine_for`` with several devices returns that module's engine.

Every arithmetic step of the reduction runs in libfedagg's HIP kernels; if the library or a GPU
is missing the engine raises -- there is no CPU fallback.  Results never depend on engine state:
what is kept between calls is the one-shot record of rows staged by :meth:`ingest` (used only for
the very same array objects), grow-only HBM buffers and result host buffers that are recycled
only once nothing references them.  Calls are serialised per GPU.  The GPU is initialised lazily on
first use (tests fork after import: tests/conftest.py:52-59), so strategies stay
cloudpickle-able for RemoteStruct (remote_struct.py:84-114); the engine itself is never pickled.
"""

from __future__ import annotations

import ctypes
import functools
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _native, handoff, runtime
from .layout import BucketLayout
from .wire import flat_of

KINDS = ("f32", "bf16", "f64", "f16")

# GPU selection of the strategies (resolve_devices): an index, several indices, or "all"
Devices = Optional[Union[int, Sequence[int], str]]


def _torch():
    import torch

    return torch


def torch_dtype(kind_or_np):
    torch = _torch()
    m = {
        "f32": torch.float32,
        "bf16": torch.bfloat16,
        "f64": torch.float64,
        "f16": torch.float16,
        np.dtype(np.float32): torch.float32,
        np.dtype(np.float64): torch.float64,
        np.dtype(np.float16): torch.float16,
    }
    return m[kind_or_np if isinstance(kind_or_np, str) else np.dtype(kind_or_np)]


def kind_of(np_dtype) -> str:
    d = np.dtype(np_dtype)
    if d == np.float32:
        return "f32"
    if d == np.float64:
        return "f64"
    if d == np.float16:
        return "f16"
    raise NotImplementedError(f"no aggregation kernel for dtype {d}")


def native_byte_order(rows):
    """``rows`` (lists of arrays) with every array in non-native byte order (a pickle written on
    a big-endian host) replaced by a native copy -- exact, and the byte order NumPy's ufuncs give
    the reference's results anyway; ``rows`` itself when every array is native (the usual case)."""
    if all(np.asarray(a).dtype.isnative for row in rows for a in row):
        return rows
    return [[a if np.asarray(a).dtype.isnative else np.asarray(a).astype(np.asarray(a).dtype.newbyteorder("="))
             for a in row] for row in rows]


def fedavg_weights(n_samples: Sequence[int], kind: str) -> np.ndarray:
    """``fl(n_k / n)``: Python-int total, double division, then rounded to the product type
    (fed_avg.py:217,221; a Python float is a weak scalar under NEP 50)."""
    n_all = sum(int(n) for n in n_samples)
    w64 = np.array([int(n) / n_all for n in n_samples], dtype=np.float64)
    if kind in ("f32", "bf16"):
        return w64.astype(np.float32)
    if kind == "f64":
        return w64
    if kind == "f16":
        return w64.astype(np.float16)
    raise ValueError(kind)


def scaffold_weights(n_samples: Sequence[int]) -> np.ndarray:
    """``int64 array / np.sum(int64 array)`` -> float64 (scaffold.py:319-320)."""
    arr = np.array([int(n) for n in n_samples])
    return (arr / np.sum(arr)).astype(np.float64)


def _stream_handle(stream) -> int:
    if isinstance(stream, int):
        return stream
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


# ======================================================================================
# device-resident plans
# ======================================================================================
class FedAvgPlan:
    """One FedAvg reduction over device-resident client buckets, arguments pre-bound.

    ``clients``: list of K device pointers (or a ``[K, ld]`` tensor), each a row of ``M``
    elements of ``kind``; ``out``: device tensor of >= M elements (fp32 for f32/bf16).
    """

    def __init__(self, kind: str, clients, weights: np.ndarray, M: int, out, pairwise_idx=None, ws=None):
        if kind not in KINDS:
            raise ValueError(f"unknown kind {kind}")
        self.lib = _native.load()
        self.kind = kind
        ptrs = _row_pointers(clients)
        self.K = len(ptrs)
        if self.K == 0:
            raise ValueError("FedAvgPlan needs at least one client")
        if len(weights) != self.K:
            raise ValueError("one weight per client")
        self.M = int(M)
        self._keep = (clients, out, ws)
        self._ptrs = _native.ptr_array(ptrs)
        self._out = _ptr(out)
        if kind in ("f32", "bf16"):
            self._w = (ctypes.c_float * self.K)(*[float(v) for v in np.asarray(weights, np.float32)])
        elif kind == "f64":
            self._w = (ctypes.c_double * self.K)(*[float(v) for v in np.asarray(weights, np.float64)])
        else:
            bits = np.asarray(weights, np.float16).view(np.uint16)
            self._w = (ctypes.c_uint16 * self.K)(*[int(v) for v in bits])
        idx = np.asarray(pairwise_idx if pairwise_idx is not None else [], dtype=np.uint64)
        self.P = int(idx.size)
        self._idx = (ctypes.c_uint64 * max(1, self.P))(*[int(v) for v in idx])
        self._ws = 0
        if self.P > _native.FEDAGG_FUSED_PAIRWISE or (self.P and self.K > _native.FEDAGG_KCHUNK):
            if ws is None:  # the numel==1 patch cannot be fused into the bucket launch
                torch = _torch()
                nbytes = self.lib.fedagg_pairwise_ws_bytes(self.K, self.P, 8)
                ws = torch.empty(nbytes, dtype=torch.uint8, device=out.device)
                self._keep = (clients, out, ws)
            self._ws = _ptr(ws)
        self._main = getattr(self.lib, f"fedagg_fedavg_{kind}")

    def launch(self, stream=None) -> None:
        """Enqueue the bucket reduction (numel==1 patch fused when possible) on ``stream``."""
        rc = self._main(self._ptrs, self._w, self.K, self.M, self._idx, self.P, self._ws, self._out,
                        _stream_handle(stream))
        _native.check(rc, "fedavg")

    def bytes_alg(self) -> int:
        s_in = {"f32": 4, "bf16": 2, "f64": 8, "f16": 2}[self.kind]
        s_out = {"f32": 4, "bf16": 4, "f64": 8, "f16": 2}[self.kind]
        return self.K * self.M * s_in + self.M * s_out


TILED_KINDS = ("f32", "bf16")
_ELEMS_PER_VEC = {"f32": 4, "bf16": 8}


def tiled_recommended(kind: str, K: int, M: int) -> bool:
    """Whether the library recommends the tile-interleaved layout for K clients of M elements
    (its row-layout kernel for that shape walks one of the tiled kernels' tiles;
    fedagg_fedavg_tile_vectors_*)."""
    if kind not in TILED_KINDS:
        return False
    return bool(getattr(_native.load(), f"fedagg_fedavg_tile_vectors_{kind}")(int(K), int(M)))


def tiled_tile(kind: str, K: int, M: int) -> int:
    """16-B vectors per client tile of the tile-interleaved layout for K clients of M elements:
    the recommended tile, else the tile of the kernel the row layout would use for K clients
    (FEDAGG_TILE_VECTORS_*)."""
    rec = int(getattr(_native.load(), f"fedagg_fedavg_tile_vectors_{kind}")(int(K), int(M)))
    if rec:
        return rec
    if kind == "bf16":
        return _native.FEDAGG_TILE_VECTORS_BF16
    return _native.FEDAGG_TILE_VECTORS_F32 if K >= 32 else _native.FEDAGG_TILE_VECTORS_F32_FEW


def tiled_elems(kind: str, K: int, M: int, tv: int) -> int:
    """Elements of a tile-interleaved buffer of K clients of M elements, tiles of ``tv`` 16-B
    vectors (the last tile of every client padded)."""
    L = _ELEMS_PER_VEC[kind]
    nvec = -(-int(M) // L)
    return -(-nvec // int(tv)) * int(K) * int(tv) * L


def tiled_index(kind: str, K: int, k, e, tv: int):
    """Element offset, in the tile-interleaved buffer, of element ``e`` of client ``k`` (NumPy
    broadcasting): vector v = e // L of client k sits at ((v // tv) * K + k) * tv + v % tv."""
    L, T = _ELEMS_PER_VEC[kind], int(tv)
    e = np.asarray(e, dtype=np.int64)
    v = e // L
    return (((v // T) * int(K) + np.asarray(k, dtype=np.int64)) * T + v % T) * L + e % L


def tiled_client_view(buf, kind: str, K: int, k: int, tv: int):
    """Client ``k``'s tiles of a tile-interleaved torch buffer: a strided ``[tiles, tv * L]`` view
    (its first M elements in row-major order are the client's bucket)."""
    return buf.view(-1, int(K), int(tv) * _ELEMS_PER_VEC[kind])[:, int(k), :]


class TiledFedAvgPlan(FedAvgPlan):
    """FedAvg over tile-interleaved client buckets (``fedagg_fedavg_tiled_{f32,bf16}``): ``base``
    is one device buffer (tensor or pointer) of :func:`tiled_elems` elements in which tile t of
    client k is tile ``t * K + k``; a workgroup then reads one contiguous K-tile region per step.
    ``tv``: the tile (default :func:`tiled_tile`).  Same kernel arithmetic and results as
    :class:`FedAvgPlan` over the row layout."""

    def __init__(self, kind: str, base, K: int, weights: np.ndarray, M: int, out, pairwise_idx=None, ws=None,
                 tv: Optional[int] = None):
        if kind not in TILED_KINDS:
            raise ValueError(f"tile-interleaved buckets take {TILED_KINDS}")
        T = int(tv) if tv is not None else tiled_tile(kind, K, M)
        # the per-client tile-0 pointers size the pairwise workspace and validate K like the rows plan
        super().__init__(kind, [_ptr(base) + k * T * 16 for k in range(int(K))], weights, M, out, pairwise_idx, ws)
        self._keep = (base,) + tuple(self._keep)
        self._base, self._tv = _ptr(base), T
        self._tiled = getattr(self.lib, f"fedagg_fedavg_tiled_{kind}")

    def launch(self, stream=None) -> None:
        rc = self._tiled(self._base, self._w, self.K, self.M, self._tv, self._idx, self.P, self._ws, self._out,
                         _stream_handle(stream))
        _native.check(rc, "fedavg_tiled")


class ScaffoldPlan:
    """Scaffold two-bucket reduction over device-resident buckets (fp32 or fp64 inputs, fp64 out)."""

    def __init__(self, kind: str, delta, cv, c, weights: np.ndarray, M: int, lr: float, delta_out, c_out,
                 pairwise_idx=None, ws=None):
        if kind not in ("f32", "f64"):
            raise ValueError("Scaffold kernels take f32 or f64 inputs")
        self.lib = _native.load()
        self.kind = kind
        dp, cp = _row_pointers(delta), _row_pointers(cv)
        self.K = len(dp)
        if self.K == 0 or len(cp) != self.K or len(weights) != self.K:
            raise ValueError("ScaffoldPlan: K mismatch")
        self.M = int(M)
        self.lr = float(lr)
        self._keep = [delta, cv, c, delta_out, c_out, ws]
        self._dp = _native.ptr_array(dp)
        self._cp = _native.ptr_array(cp)
        self._c = _ptr(c)
        self._w = (ctypes.c_double * self.K)(*[float(v) for v in np.asarray(weights, np.float64)])
        self._dout = _ptr(delta_out)
        self._cout = _ptr(c_out)
        idx = np.asarray(pairwise_idx if pairwise_idx is not None else [], dtype=np.uint64)
        self.P = int(idx.size)
        self._idx = (ctypes.c_uint64 * max(1, self.P))(*[int(v) for v in idx])
        self._ws = 0
        if self.P > _native.FEDAGG_FUSED_PAIRWISE or (self.P and self.K > _native.FEDAGG_KCHUNK_SCAFFOLD):
            if ws is None:
                torch = _torch()
                ws = torch.empty(self.lib.fedagg_pairwise_ws_bytes(self.K, self.P, 8), dtype=torch.uint8,
                                 device=delta_out.device)
                self._keep.append(ws)
            self._ws = _ptr(ws)
        self._main = getattr(self.lib, f"fedagg_scaffold_{kind}")

    def launch(self, stream=None) -> None:
        rc = self._main(self._dp, self._cp, self._c, self._w, self.K, self.M, self._idx, self.P, self._ws, self.lr,
                        self._dout, self._cout, _stream_handle(stream))
        _native.check(rc, "scaffold")

    def bytes_alg(self) -> int:
        s_in = 4 if self.kind == "f32" else 8
        return 2 * self.K * self.M * s_in + self.M * s_in + 2 * self.M * 8


def equal_count(kind: str, copies, M: int, counter, stream=None) -> None:
    """Enqueue the server-control-variate equality check (adds mismatches to ``counter``)."""
    lib = _native.load()
    ptrs = _row_pointers(copies)
    fn = getattr(lib, f"fedagg_equal_count_{kind}")
    _native.check(fn(_native.ptr_array(ptrs), len(ptrs), int(M), _ptr(counter), _stream_handle(stream)),
                  "equal_count")


def _ptr(x) -> int:
    return int(x) if isinstance(x, int) else int(x.data_ptr())


def _row_pointers(clients) -> List[int]:
    if isinstance(clients, (list, tuple)) and all(isinstance(c, int) for c in clients):
        return [int(c) for c in clients]
    torch = _torch()
    if isinstance(clients, torch.Tensor):
        if clients.dim() != 2:
            raise ValueError("client buckets tensor must be [K, ld]")
        if not clients.is_cuda:
            raise ValueError("client buckets must be device tensors")
        base = clients.data_ptr()
        step = clients.stride(0) * clients.element_size()
        return [base + k * step for k in range(clients.shape[0])]
    out = []
    for c in clients:
        if isinstance(c, int):
            out.append(c)
        else:
            if not c.is_cuda:
                raise ValueError("client buckets must be device tensors")
            out.append(c.data_ptr())
    return out


# ======================================================================================
# host entry (drop-in path)
# ======================================================================================
def direct_rows(rows: List[List[np.ndarray]], dt: np.dtype, M: int) -> Optional[List[List[np.ndarray]]]:
    """Rows as stageable segments when every array already has dtype ``dt`` (flat wire-format
    rows as one segment each), else None."""
    if not all(a.dtype == dt for row in rows for a in row):
        return None
    flats = [flat_of(row) for row in rows]
    if all(f is not None and f.size == M for f in flats):
        return [[f] for f in flats]
    return [[np.ascontiguousarray(a) for a in row] for row in rows]


def serialized(method):
    """Run an engine call under the locks of the engine's devices (``runtime.device_lock``), taken
    in device order, so concurrent callers never share a session's buffers mid-call; the calling
    thread's current HIP device is restored on return (the session calls bind their own device to
    the thread, and the caller's later work -- its training, in simulate_experiment -- must stay
    on the GPU it chose)."""

    @functools.wraps(method)
    def wrapper(self, *args, **kwargs):
        locks = [runtime.device_lock(d) for d in sorted(set(self.lock_devices()))]
        held = []
        lib, dev = None, ctypes.c_int(-1)
        try:
            for lk in locks:
                lk.acquire()
                held.append(lk)
            # inside the try: a missing library or an ABI mismatch raises to this caller and the
            # locks are released, never left held for the other threads of the process
            lib = _native.load()
            if lib.fedagg_device_get(ctypes.byref(dev)) != 0:
                dev.value = -1
            handoff.invalidate_slots(self.lock_devices())  # this call may rewrite its output slots
            return method(self, *args, **kwargs)
        finally:
            if lib is not None and dev.value >= 0:
                lib.fedagg_device_set(dev.value)
            for lk in reversed(held):
                lk.release()

    return wrapper


@dataclass
class StagedRows:
    """Where one FedAvg call's client rows are in HBM (:meth:`AggregationEngine._resolve_rows`):
    ``reason`` names the path; ``ptrs`` the K row addresses (row layouts) or ``base`` / ``tv`` the
    tile-interleaved bucket; ``handoff_rows`` how many rows came from the hand-off."""

    reason: str
    ptrs: Optional[List[int]]
    base: Optional[int]
    tv: Optional[int]
    handoff_rows: int


class AggregationEngine:
    """Drop-in host path bound to one GPU (``device``, else ``LOCAL_RANK``, else 0).

    Runs on the native session (:mod:`substrafl_amd.runtime`): pinned-ring pack + H2D, the HIP
    kernels on the session stream, D2H into owned NumPy arrays.  No PyTorch on this path."""

    # HBM buffer slots of the session
    _B_BUCKET, _B_OUT, _B_WS, _B_TMP, _B_CV, _B_C, _B_COUT, _B_CNT = range(8)
    _B_HANDOFF_C = 12  # the hand-off's copy of Scaffold's new c: written only by copy_d2d (handoff.py)

    def __init__(self, device: Optional[int] = None, pack_threads: Optional[int] = None,
                 max_bucket_bytes: Optional[int] = None, c_check: str = "host"):
        self._device_index = device
        self._pack_threads = pack_threads
        if c_check not in ("host", "device"):
            raise ValueError("c_check must be 'host' or 'device'")
        # where Scaffold's server-control-variate equality check runs (scaffold.py:193-196)
        self.c_check = os.environ.get("FEDAGG_C_CHECK", c_check)
        # HBM the staged buckets of one call may take before the call is streamed through the GPU
        # in parameter ranges (multi_device.MultiDeviceEngine with this one device); default:
        # 85 % of the device's free HBM at call time
        self.max_bucket_bytes = max_bucket_bytes
        # HBM layout of FedAvg buckets (staged by a call, or client by client by ingest): "auto" =
        # tile-interleaved where fedagg_fedavg_tile_vectors_* recommends it (from 32 fp32 clients
        # over large buckets), True / False to force
        env = os.environ.get("FEDAGG_TILED", "auto")
        self.tiled: Union[str, bool] = {"0": False, "1": True}.get(env, "auto")
        self._ooc = None
        self.last_timing: Dict[str, float] = {}
        # rows already on the device from ingest(): slot -> (d_bucket, ld_bytes, {k: row arrays},
        # write generation of the slot after the ingest) -- valid only while nothing else (another
        # engine on this GPU's shared session, or this engine's own other paths) wrote the slot
        self._prestaged: Dict[int, list] = {}

    def _out_of_core(self, need_bytes: int, slots: Sequence[int]):
        """The range-streaming engine when ``need_bytes`` of buckets exceed this GPU's budget
        (K x M beyond 288 GB on one MI355X), else None.  ``slots``: the session buffers the
        in-core call would (re)use; only their bytes count as available besides the free HBM."""
        from .multi_device import HBM_HEADROOM, MultiDeviceEngine

        if self.max_bucket_bytes is not None:
            budget = int(self.max_bucket_bytes)
        else:
            free = runtime.device_memory(self._index())[0] + self.session().held_bytes(slots)
            budget = int(free * HBM_HEADROOM)
        if need_bytes <= budget:
            return None
        if self._ooc is None:
            self._ooc = MultiDeviceEngine([self._index()], max_shard_bytes=self.max_bucket_bytes,
                                          pack_threads=self._pack_threads)
        self._prestaged = {}
        return self._ooc

    def lock_devices(self) -> List[int]:
        return [self._index()]

    def _index(self) -> int:
        idx = self._device_index
        return int(os.environ.get("LOCAL_RANK", "0")) if idx is None else idx

    def prewarm(self) -> None:
        """Start :func:`runtime.prewarm` for this engine's GPU (HIP start-up, pinned ring, worker
        pool, code object) on a background thread; HBM buffers are sized by the first call
        (``hipMalloc`` is ~0.1 ms, not worth guessing sizes for)."""
        runtime.prewarm(self._index())

    @serialized
    def ingest(self, paths: Sequence, strategy: str, load, max_workers: int = 0) -> List:
        """Load K shared-state files (``load(path)``, e.g. ``PickleSerializer.load``) on a thread
        pool and stage each client's bucket rows to HBM as soon as that client is loaded, so the
        H2D copies overlap the remaining unpickling.  Returns the states
        in path order, exactly as ``[load(p) for p in paths]``; the first failing path's error
        is raised.  The staged rows are used by the next :meth:`fedavg` / :meth:`scaffold` call
        only if it receives the very same array objects in the same layout; anything else is
        staged again there (the rows are only a head start, never a cache)."""
        from concurrent.futures import ThreadPoolExecutor, as_completed

        paths = list(paths)
        K = len(paths)
        self._prestaged = {}
        if K == 0:
            return []
        workers = max_workers or min(K, 16, os.cpu_count() or 1)
        t0 = time.perf_counter()
        staged = 0
        with ThreadPoolExecutor(workers) as ex:
            futures = [ex.submit(load, p) for p in paths]
            index = {f: k for k, f in enumerate(futures)}
            plan = None
            checks = []  # Scaffold: value checks of the c copies, on the loader threads
            for f in as_completed(futures):
                if f.exception() is not None:
                    plan = False  # stop staging; the error is raised below in path order
                if plan is False:
                    continue
                try:
                    if plan is None:
                        plan = self._ingest_plan(f.result(), strategy, K)
                    if plan and self._ingest_row(plan, index[f], f.result(), lambda *a: checks.append(ex.submit(*a))):
                        staged += 1
                except Exception:  # noqa: BLE001 - staging is best effort; aggregation re-validates
                    plan = False
                    self._prestaged = {}
            states = [f.result() for f in futures]
            try:
                self._c_mism = sum(c.result() for c in checks)
            except Exception:  # noqa: BLE001 - the aggregation call checks again
                self._prestaged.pop(self._B_C, None)
        s = getattr(self, "_prestaged_session", None)
        for slot, rec in self._prestaged.items():  # seal: the slots as this ingest left them
            rec.append(s.generation(slot) if s is not None else -1)
        self.last_ingest = {"load_and_stage_s": time.perf_counter() - t0, "prestaged_clients": staged}
        return states

    def _ingest_plan(self, state, strategy: str, K: int):
        """Layouts and buffers for staging rows shaped like ``state``'s (None: do not prestage)."""
        if strategy == "scaffold":
            # server control variates: ONE copy is staged (the first client loaded), every other
            # client's copy is compared with it on the host as it arrives (Session.check) -- the
            # check of scaffold.py:193-196 overlapped with the loading, K-1 PCIe copies saved
            lists = (("parameters_update", self._B_BUCKET), ("control_variate_update", self._B_CV))
        else:
            lists = (("parameters_update", self._B_BUCKET),)
        rows = []
        for field, slot in lists:
            row = list(getattr(state, field, None) or [])
            if not row or not all(isinstance(a, np.ndarray) for a in row):
                return None
            if any(a.dtype != row[0].dtype for a in row) or row[0].dtype.kind not in "biuf":
                return None  # per-layer dtype groups are staged by the aggregation call
            rows.append(row)
        if strategy == "scaffold":  # scaffold engine: fp32 buckets only when every list is fp32
            c_row = list(getattr(state, "server_control_variate", None) or [])
            all32 = all(r[0].dtype == np.float32 for r in rows) and all(
                isinstance(a, np.ndarray) and a.dtype == np.float32 for a in c_row)
            targets = [np.dtype(np.float32 if all32 else np.float64)] * len(rows)
        else:  # FedAvg: NumPy's product type of the layer (ints -> fp64)
            targets = [np.result_type(rows[0][0].dtype, 1.0)]
            if targets[0] not in (np.float16, np.float32, np.float64):
                return None
        plan = []
        s = self.session()
        self._ingest_K = K
        for (field, slot), row, dt in zip(lists, rows, targets):
            layout = BucketLayout(list(range(len(row))), [a.shape for a in row], dt)
            ld_bytes = layout.ld * dt.itemsize
            kind = kind_of(dt)
            if strategy != "scaffold" and row[0].dtype == dt and self.tiled is not False and kind in TILED_KINDS and (
                    self.tiled is True or tiled_recommended(kind, K, layout.M)):
                # tile-interleaved, as fedavg() would stage them: each client's tiles land at
                # their K-strided places (Session.stage_tiled_row); ld_bytes -tv marks the layout
                tv = tiled_tile(kind, K, layout.M)
                d = s.buffer(slot, tiled_elems(kind, K, layout.M, tv) * dt.itemsize)
                ld_bytes = -tv
            else:
                d = s.buffer(slot, K * ld_bytes)
            self._prestaged[slot] = [d, ld_bytes, {}]
            plan.append((field, slot, layout, d, ld_bytes, row[0].dtype, False))
        if strategy == "scaffold" and self.c_check == "host" and c_row and all(
                isinstance(a, np.ndarray) and a.dtype == targets[0] for a in c_row):
            dt = targets[0]
            layout = BucketLayout(list(range(len(c_row))), [a.shape for a in c_row], dt)
            ld_bytes = layout.ld * dt.itemsize
            d = s.buffer(self._B_C, ld_bytes)  # ONE copy staged, the others checked on the host
            self._prestaged[self._B_C] = [d, ld_bytes, {}]
            self._c_ref, self._c_mism = None, 0
            plan.append(("server_control_variate", self._B_C, layout, d, ld_bytes, dt, True))
        self._prestaged_session = s
        return plan

    def _ingest_row(self, plan, k: int, state, submit=None) -> bool:
        s = self.session()
        for field, slot, layout, d, ld_bytes, src, check in plan:
            row = list(getattr(state, field))
            if len(row) != len(layout.segments) or any(
                    a.dtype != src or a.shape != g.shape for a, g in zip(row, layout.segments)):
                return False
        for field, slot, layout, d, ld_bytes, src, check in plan:
            row = list(getattr(state, field))
            if not check and ld_bytes < 0:
                s.stage_tiled_row(d, -ld_bytes * 16, self._ingest_K, k, direct_rows([row], layout.dtype, layout.M)[0])
            elif not check:
                self._stage_rows(s, [row], layout, d + k * ld_bytes)
            elif self._c_ref is None:  # the first client loaded: its c is the staged copy
                self._stage_rows(s, [row], layout, d)
                self._c_ref = row
            elif submit is not None:  # value check against the staged copy, beside the staging
                submit(s.check, [self._c_ref, row], src)  # (equality is an equivalence: +0 == -0, NaN == NaN)
            else:
                self._c_mism += s.check([self._c_ref, row], src)
            self._prestaged[slot][2][k] = row  # holds the arrays: their ids stay unique
        return True

    def _take_prestaged(self, slot: int, d_bucket: int, ld_bytes: int, rows) -> bool:
        """True when every row was staged by :meth:`ingest` from these very arrays."""
        rec = self._prestaged.pop(slot, None)
        if rec is None or len(rec) != 4 or rec[0] != d_bucket or rec[1] != ld_bytes or len(rec[2]) != len(rows):
            return False
        if rec[3] != self.session().generation(slot):  # the slot was written since the ingest
            return False
        for k, row in enumerate(rows):
            got = rec[2].get(k)
            if got is None or len(got) != len(row) or any(a is not b for a, b in zip(got, row)):
                return False
        return True

    def _tiled_rows(self, rows, R: np.dtype, kind: str, K: int, M: int):
        """The rows as stageable segments when this call stages them tile-interleaved (``tiled``:
        "auto" where the library recommends the layout, True wherever a tiled kernel exists for
        the dtype, False never), else None (also when a dtype conversion is needed: those stage
        raw rows and cast on the device)."""
        mode = self.tiled
        if mode is False or kind not in TILED_KINDS or (mode == "auto" and not tiled_recommended(kind, K, M)):
            return None
        return direct_rows(rows, R, M)

    def session(self):
        s = runtime.session(self._index())
        if self._pack_threads:
            s.set("threads", self._pack_threads)
        return s

    # ----------------------------------------------------------------------------------
    def _stage_rows(self, s, rows: List[List[np.ndarray]], layout: BucketLayout, d_bucket: int,
                    prescale: Optional[Dict[int, float]] = None) -> None:
        """Stage K clients' arrays (in ``layout`` segment order) as ``[K, ld]`` rows of
        ``layout.dtype`` at ``d_bucket``.  Arrays of another dtype are staged raw and converted on
        the device (exact casts); clients listed in ``prescale`` are multiplied by their weight in
        their own float type first (mixed-dtype layers)."""
        isz = layout.dtype.itemsize
        ld_bytes = layout.ld * isz
        prescale = prescale or {}
        direct = not prescale and all(a.dtype == layout.dtype for row in rows for a in row)
        if direct:
            flats = [flat_of(row) for row in rows]
            if all(f is not None and f.size == layout.M for f in flats):
                rows = [[f] for f in flats]  # flat wire format: one segment per client
            s.stage(d_bucket, ld_bytes, rows)
            return
        src = {a.dtype for row in rows for a in row}
        if not prescale and len(src) == 1:
            # every array has one other dtype (e.g. Scaffold's fp32 deltas next to fp64 control
            # variates from round 2 on): stage the raw rows with the SAME element stride, then one
            # exact device cast over the whole [K, ld] block
            (sdt,) = src
            K = len(rows)
            tmp = s.buffer(self._B_TMP, K * layout.ld * sdt.itemsize)
            s.stage(tmp, layout.ld * sdt.itemsize, rows)
            s.cast(tmp, sdt, d_bucket, layout.dtype, K * layout.ld)
            return
        for k, row in enumerate(rows):
            for seg, a in zip(layout.segments, row):
                dst = d_bucket + k * ld_bytes + seg.offset * isz
                if k not in prescale and a.dtype == layout.dtype:
                    s.stage(dst, a.nbytes, [[a]])
                    continue
                tmp = s.buffer(self._B_TMP, a.nbytes)
                s.stage(tmp, a.nbytes, [[a]])
                if k in prescale:
                    s.scale_cast(tmp, a.dtype, prescale[k], dst, layout.dtype, a.size)
                else:
                    s.cast(tmp, a.dtype, dst, layout.dtype, a.size)
                s.sync()  # tmp is reused by the next segment's stage

    _last_handoff: List[bool] = []

    _handoff_keep = None

    def _handoff_rows(self, s, rows: List[List[np.ndarray]], layout: BucketLayout, R: np.dtype, K: int):
        """Simulation mode (``handoff``): client rows whose bytes are still on this GPU (an
        ``accelerate_algo`` export recorded with its device bucket).  All of them: the list of
        their device pointers -- the kernel reads the clients' buckets in place, nothing is copied
        (kept alive in ``_handoff_keep`` until the result is fetched).  Some: those are copied
        device to device into the ``[K, ld]`` rows, the others staged from the host as usual, and
        the bucket's address is returned.  None when no row can be handed off (the caller stages
        everything, tiled where recommended)."""
        hits = [handoff.lookup(row, s.device) for row in rows]
        self._last_handoff = [h is not None and h[1] == layout.M * R.itemsize and all(a.dtype == R for a in row)
                              for h, row in zip(hits, rows)]
        if not any(self._last_handoff):
            return None
        if all(self._last_handoff):
            self._handoff_keep = hits
            return [int(h[0]) for h in hits]
        ld_bytes = layout.ld * R.itemsize
        d_bucket = s.buffer(self._B_BUCKET, K * ld_bytes)
        for k, (row, h, ok) in enumerate(zip(rows, hits, self._last_handoff)):
            if ok:
                s.copy_d2d(d_bucket + k * ld_bytes, h[0], h[1])
            else:
                self._stage_rows(s, [row], layout, d_bucket + k * ld_bytes)
        s.sync()  # the copies' sources are kept alive by `hits` only until here
        return d_bucket

    def _handoff_into(self, s, rows: List[List[np.ndarray]], lay: BucketLayout, d: int):
        """All K rows recorded by the hand-off (one source dtype).  Of the bucket's dtype: the
        list of their device pointers -- the kernel reads the clients' buckets in place (kept
        alive in ``_handoff_keep`` until the results are fetched).  Of another float type
        (Scaffold's fp32 deltas into its fp64 buckets): copied device to device into ``[K,
        lay.ld]`` at ``d`` through one exact device cast, as ``_stage_rows`` does for host rows,
        and True.  False (nothing written) otherwise."""
        hits = [handoff.lookup(row, s.device) for row in rows]
        if not hits or any(h is None for h in hits):
            return False
        src = {row[0].dtype for row in rows}
        if len(src) != 1:
            return False
        (sdt,) = src
        if any(h[1] != lay.M * sdt.itemsize for h in hits):
            return False
        K = len(rows)
        if sdt == lay.dtype:
            self._handoff_keep = (self._handoff_keep or []) + hits
            return [int(h[0]) for h in hits]
        else:
            tmp = s.buffer(self._B_TMP, K * lay.ld * sdt.itemsize)
            for k, h in enumerate(hits):
                s.copy_d2d(tmp + k * lay.ld * sdt.itemsize, h[0], h[1])
            s.cast(tmp, sdt, d, lay.dtype, K * lay.ld)
        s.sync()  # the copies' sources are kept alive by `hits` only until here
        return True

    def _resolve_rows(self, s, rows: List[List[np.ndarray]], layout: BucketLayout, R: np.dtype, kind: str, K: int,
                      prescale: Optional[Dict[int, float]], single: bool) -> "StagedRows":
        """Where the K client rows of one FedAvg dtype group come from, and where they are in HBM
        (VERDICT r05 "Next 3": one resolver, one reason).  In order of preference:

        * ``prestaged-tiles`` / ``prestaged-rows``: :meth:`ingest` staged these very arrays while
          the task loaded them (tile-interleaved or ``[K, ld]`` rows) and nothing wrote the slot since;
        * ``handoff-in-place``: simulation mode, every row is a client export still on this GPU
          (``handoff``): the kernel reads the clients' own buckets, nothing is copied;
        * ``handoff-partial``: some rows are: copied device to device into ``[K, ld]``, the others
          staged from the host;
        * ``host-tiles`` / ``host-rows``: staged over PCIe through the pinned ring (tiled where the
          library recommends it; rows with exact device casts for other dtypes).

        The prestaged and hand-off paths take only one dtype group with no per-client prescale
        (what :meth:`ingest` and the exports produce).  The out-of-core path (``out-of-core``) is
        decided before this, for the whole call."""
        isz = R.itemsize
        ld_bytes = layout.ld * isz
        d_rows = s.buffer(self._B_BUCKET, K * ld_bytes)
        rows_at = lambda d: [d + k * ld_bytes for k in range(K)]  # noqa: E731
        if prescale is None and single:
            rec = self._prestaged.get(self._B_BUCKET)
            if rec is not None and rec[1] < 0 and kind in TILED_KINDS:  # ingest staged them tiled
                d_t = s.buffer(self._B_BUCKET, tiled_elems(kind, K, layout.M, -rec[1]) * isz)
                if self._take_prestaged(self._B_BUCKET, d_t, rec[1], rows):
                    return StagedRows("prestaged-tiles", None, d_t, -rec[1], 0)
            elif self._take_prestaged(self._B_BUCKET, d_rows, ld_bytes, rows):
                return StagedRows("prestaged-rows", rows_at(d_rows), None, None, 0)
            hand = self._handoff_rows(s, rows, layout, R, K)
            if hand is not None:
                self._prestaged.pop(self._B_BUCKET, None)
                n = sum(1 for r in self._last_handoff if r)
                if isinstance(hand, list):
                    return StagedRows("handoff-in-place", hand, None, None, n)
                return StagedRows("handoff-partial", rows_at(hand), None, None, n)
        self._prestaged.pop(self._B_BUCKET, None)
        tiled = self._tiled_rows(rows, R, kind, K, layout.M) if prescale is None else None
        if tiled is not None:  # tile-interleaved buckets, one gather per pinned chunk
            tv = tiled_tile(kind, K, layout.M)
            d_t = s.buffer(self._B_BUCKET, tiled_elems(kind, K, layout.M, tv) * isz)
            s.stage_tiled(d_t, tv * 16, tiled)
            return StagedRows("host-tiles", None, d_t, tv, 0)
        d_rows = s.buffer(self._B_BUCKET, K * ld_bytes)  # current after a regrow
        self._stage_rows(s, rows, layout, d_rows, prescale)
        return StagedRows("host-rows", rows_at(d_rows), None, None, 0)

    # ----------------------------------------------------------------------------------
    @serialized
    def fedavg(self, parameters_updates: List[List[np.ndarray]], n_samples: Sequence[int],
               wire: bool = False) -> List[np.ndarray]:
        """GPU equivalent of fed_avg.py:217-222 for validated inputs (same layer count and shapes
        across clients, ``sum(n_samples) != 0``).  Returns one array per layer (0-d layers as
        NumPy scalars, like ``np.sum``): plain views of one owned array, or with ``wire``
        :class:`wire.BucketArray` layers that pickle as one buffer."""
        t_start = time.perf_counter()
        parameters_updates = native_byte_order(parameters_updates)
        s = self.session()
        self.last_timing = tm = {}
        K = len(parameters_updates)
        L = len(parameters_updates[0])
        if L == 0:
            return []
        # group layers by (result dtype, per-client product dtypes): NumPy promotion per layer
        groups: Dict[Tuple, List[int]] = {}
        for li in range(L):
            pds = tuple(np.result_type(pu[li].dtype, 1.0) for pu in parameters_updates)
            for d in pds:
                if d not in (np.float16, np.float32, np.float64):
                    raise NotImplementedError(f"FedAvg engine: unsupported layer dtype {d}")
            R = np.result_type(*pds)
            key = (R.str, None if all(d == R for d in pds) else tuple(d.str for d in pds))
            groups.setdefault(key, []).append(li)

        if len(groups) == 1:
            (rstr, mixed), = groups.keys()
            R = np.dtype(rstr)
            direct = mixed is None and all(a.dtype == R for pu in parameters_updates for a in pu)
            need = (K + 1) * BucketLayout(range(L), [a.shape for a in parameters_updates[0]], R).ld * R.itemsize
            ooc = self._out_of_core(need, (self._B_BUCKET, self._B_OUT, self._B_WS)) if direct else None
            if ooc is not None:
                out = ooc.fedavg(parameters_updates, n_samples, wire)
                self.last_timing = {"out_of_core": ooc.last_timing, "staging": "out-of-core"}
                return out
        results: List[Optional[np.ndarray]] = [None] * L
        if len(groups) != 1:
            self._prestaged = {}
        for (rstr, mixed), layer_ids in groups.items():
            R = np.dtype(rstr)
            kind = kind_of(R)
            layout = BucketLayout(layer_ids, [parameters_updates[0][li].shape for li in layer_ids], R)
            rows = [[pu[li] for li in layer_ids] for pu in parameters_updates]
            w = fedavg_weights(n_samples, kind)
            prescale = None
            if mixed is not None:
                w64 = [int(n) / sum(int(m) for m in n_samples) for n in n_samples]
                prescale = {k: w64[k] for k, d in enumerate(mixed) if np.dtype(d) != R}
                for k in prescale:
                    w[k] = 1  # x * 1 is exact: the client's product was formed in its own dtype
            t0 = time.perf_counter()
            st = self._resolve_rows(s, rows, layout, R, kind, K, prescale, len(groups) == 1)
            tm["staging"] = st.reason if len(groups) == 1 else "per-dtype-groups"
            if st.handoff_rows:
                tm["handoff_rows"] = st.handoff_rows
            tm["prestaged"] = st.reason.startswith("prestaged")
            tv = st.tv
            tm["stage_s"] = tm.get("stage_s", 0.0) + time.perf_counter() - t0
            tm["layout"] = "tiles" if tv is not None else "rows"
            d_out = s.buffer(self._B_OUT, layout.ld * R.itemsize)
            ws = s.buffer(self._B_WS, _native.load().fedagg_pairwise_ws_bytes(K, layout.pairwise_idx.size, 8))
            t1 = time.perf_counter()
            if tv is not None:
                TiledFedAvgPlan(kind, st.base, K, w, layout.M, d_out, layout.pairwise_idx, ws, tv).launch(s.stream)
            else:
                FedAvgPlan(kind, st.ptrs, w, layout.M, d_out, layout.pairwise_idx, ws).launch(s.stream)
            out = runtime.reusable_host_array(layout.M, R, f"fedavg{'-mixed' if mixed else ''}")
            s.fetch(d_out, out)  # stream-ordered after the kernel; returns when the data is home
            self._handoff_keep = None  # the kernel is done with the clients' buckets
            if len(groups) == 1:
                handoff.record_slot(out, s, self._B_OUT, d_out)  # simulation mode: clients copy it on the device
            tm["kernel_fetch_s"] = tm.get("kernel_fetch_s", 0.0) + time.perf_counter() - t1
            for li, arr in layout.unpack(out, wire):
                results[li] = arr
        tm.update({f"native_{k}": v for k, v in s.timing().items()})
        tm["total_s"] = time.perf_counter() - t_start
        return results  # type: ignore[return-value]

    # ----------------------------------------------------------------------------------
    @serialized
    def sequential_sum(self, rows: List[List[np.ndarray]], n_samples: Sequence[int],
                       wire: bool = False) -> List[np.ndarray]:
        """NewtonRaphson's averaging (substrafl/strategies/newton_raphson.py:195-211) per element:
        ``total = x_0 * c_0``, then ``total += x_k * c_k`` in client order, ``c_k = n_k / n``
        (a Python float: rounded to the array's float type, NEP 50).  Two differences from
        FedAvg's ``np.sum`` (:meth:`fedavg`): no ``+0.0`` seed -- a column of ``-0.0`` products
        stays ``-0.0`` -- and no pairwise order for ``numel == 1`` layers (the loop is an explicit
        ``+=``).  On the device: client 0's product written by ``fedagg_scale_cast`` (its own
        float type, exactly ``x_0 * c_0``), then ``fedagg_fedavg_chain_*`` continuing that
        accumulator over clients 1..K-1 (seed 0), one fetch.

        dtypes: each client's product type is ``result_type(x_k, float)`` (fp16 / fp32 / fp64;
        integers multiply as fp64, cast on the device); the accumulator keeps CLIENT 0's type, as
        the in-place ``+=`` does.  A client of another type is added the way NumPy's
        ``+=`` adds it: its product in its own type, the sum in the promoted type P of the two
        (accumulator widened exactly, ``fedagg_fedavg_chain`` with weight 1.0: ``acc + p``), then
        rounded back into client 0's type (``fedagg_cast``).  Every client's layers must share one
        product type (a concatenated gradient is one array)."""
        rows = native_byte_order(rows)
        K, L = len(rows), len(rows[0])
        if L == 0:
            return []
        pdt = []
        for row in rows:
            ds = {np.result_type(a.dtype, 1.0) for a in row}
            if len(ds) != 1 or next(iter(ds)) not in (np.float16, np.float32, np.float64):
                raise NotImplementedError(f"sequential_sum: one float16 / float32 / float64 product dtype per client "
                                          f"(got {sorted(str(d) for d in ds)})")
            pdt.append(np.dtype(next(iter(ds))))
        T0 = pdt[0]  # total = x_0 * c_0 keeps this type through every +=
        n_all = sum(int(n) for n in n_samples)
        if n_all == 0:
            raise ZeroDivisionError("division by zero")  # n_samples / n_all_samples (newton_raphson.py:201)
        coeff = [int(n) / n_all for n in n_samples]
        shapes = [a.shape for a in rows[0]]
        layout = BucketLayout(list(range(L)), shapes, T0)
        M = layout.M
        s = self.session()
        self._prestaged = {}
        self.last_timing = tm = {}
        t0 = time.perf_counter()
        uniform = all(d == T0 for d in pdt)
        # row stride: room for a row of any float type (the fp16 layout's ld is a multiple of the others')
        stride = layout.ld * T0.itemsize if uniform else BucketLayout(list(range(L)), shapes, np.float16).ld * 8
        d_bucket = s.buffer(self._B_BUCKET, K * stride)
        if uniform:
            self._stage_rows(s, rows, layout, d_bucket)
        else:
            for k in range(K):
                self._stage_rows(s, [rows[k]], BucketLayout(list(range(L)), shapes, pdt[k]), d_bucket + k * stride)
        tm["stage_s"] = time.perf_counter() - t0
        d_out = s.buffer(self._B_OUT, stride)
        s.scale_cast(d_bucket, T0, coeff[0], d_out, T0, M)
        k = 1
        while k < K:
            if pdt[k] == T0:  # a run of clients of client 0's type: one chain launch continues the total
                j = k
                while j < K and pdt[j] == T0:
                    j += 1
                self._chain(s, kind_of(T0), [d_bucket + i * stride for i in range(k, j)],
                            [coeff[i] for i in range(k, j)], M, d_out)
                k = j
                continue
            P = np.dtype(np.result_type(T0, pdt[k]))  # the type NumPy's += adds in
            d_p = s.buffer(self._B_CV, stride)
            s.scale_cast(d_bucket + k * stride, pdt[k], coeff[k], d_p, P, M)  # x_k * c_k in its own type
            if P == T0:
                self._chain(s, kind_of(P), [d_p], [1.0], M, d_out)
            else:
                d_acc = s.buffer(self._B_C, stride)
                s.cast(d_out, T0, d_acc, P, M)  # exact widening
                self._chain(s, kind_of(P), [d_p], [1.0], M, d_acc)
                s.cast(d_acc, P, d_out, T0, M)  # rounded back into client 0's type
            k += 1
        out = runtime.reusable_host_array(M, T0, "seqsum")
        s.fetch(d_out, out)
        tm["total_s"] = time.perf_counter() - t0
        tm["mixed_dtypes"] = not uniform
        return [arr for _, arr in layout.unpack(out, wire)]

    @staticmethod
    def _chain(s, kind: str, ptrs: List[int], coeffs: List[float], M: int, d_acc: int) -> None:
        """acc = fl(acc + fl(x_i * fl_kind(c_i))) over the rows ``ptrs`` in order, on the session
        stream (``fedagg_fedavg_chain_{kind}``, seed 0: the accumulator continues)."""
        lib = _native.load()
        w = np.asarray(coeffs, dtype=np.float64)
        if kind == "f32":
            warr = (ctypes.c_float * len(w))(*[float(v) for v in w.astype(np.float32)])
        elif kind == "f64":
            warr = (ctypes.c_double * len(w))(*[float(v) for v in w])
        else:
            warr = (ctypes.c_uint16 * len(w))(*[int(v) for v in w.astype(np.float16).view(np.uint16)])
        _native.check(getattr(lib, f"fedagg_fedavg_chain_{kind}")(_native.ptr_array(ptrs), warr, len(ptrs), M, 0,
                                                                    d_acc, s.stream), "fedavg_chain")

    # ----------------------------------------------------------------------------------
    @serialized
    def scaffold(
        self,
        parameters_updates: List[List[np.ndarray]],
        control_variate_updates: List[List[np.ndarray]],
        server_control_variates: List[List[np.ndarray]],
        n_samples: Sequence[int],
        aggregation_lr,
        wire: bool = False,
    ):
        """GPU equivalent of scaffold.py:193-196 (c equality check, returned as the mismatch
        count) and scaffold.py:297-337 (fp64 reductions).  Returns
        ``(mismatches, new_server_control_variate, avg_parameters_update)``."""
        t_start = time.perf_counter()
        parameters_updates, control_variate_updates, server_control_variates = (
            native_byte_order(x) for x in (parameters_updates, control_variate_updates, server_control_variates))
        s = self.session()
        self.last_timing = tm = {}
        K = len(parameters_updates)
        L = len(parameters_updates[0])
        if L == 0:
            return 0, [], []
        lists = (parameters_updates, control_variate_updates, server_control_variates)
        for lst in lists:
            for client in lst:
                for a in client:
                    if a.dtype.kind not in "biuf" or a.dtype == np.longdouble:
                        raise NotImplementedError(f"Scaffold engine: unsupported dtype {a.dtype}")
        all_f32 = all(a.dtype == np.float32 for lst in lists for client in lst for a in client)
        kind = "f32" if all_f32 else "f64"
        sdt = np.dtype(np.float32 if all_f32 else np.float64)
        lid = list(range(L))
        lay_d = BucketLayout(lid, [a.shape for a in parameters_updates[0]], sdt)
        lay_c = BucketLayout(lid, [a.shape for a in control_variate_updates[0]], sdt)
        lay_s = BucketLayout(lid, [a.shape for a in server_control_variates[0]], sdt)
        same = [g.shape for g in lay_d.segments] == [g.shape for g in lay_c.segments] == \
            [g.shape for g in lay_s.segments]
        # every client holding the very same c arrays (simulation mode: the server's broadcast):
        # assert_array_equal holds by identity, so one copy is staged and the check is skipped
        same_c = all(len(row) == len(server_control_variates[0]) and all(a is b for a, b in zip(row, server_control_variates[0]))
                     for row in server_control_variates[1:])
        # otherwise (task process: K separately unpickled copies) the check runs on the host while
        # the bytes are staged: ONE copy crosses PCIe, the others are compared with it on the pack
        # workers (Session.stage_check); the device check over K staged copies stays as a knob
        # (c_check="device") and for c lists of another dtype than the buckets
        host_c = (not same_c and self.c_check == "host"
                  and all(a.dtype == sdt for row in server_control_variates for a in row))
        Kc = 1 if (same_c or host_c) else K  # rows of c in HBM: one copy unless the device checks all K
        if same and all(a.dtype == sdt for lst in lists for client in lst for a in client):
            ooc = self._out_of_core((2 * K + Kc) * lay_d.ld * sdt.itemsize + 2 * lay_d.ld * 8,
                                    (self._B_BUCKET, self._B_CV, self._B_C, self._B_OUT, self._B_COUT, self._B_WS,
                                     self._B_CNT))
            if ooc is not None:
                out = ooc.scaffold(*lists, n_samples, aggregation_lr, wire)
                self.last_timing = {"out_of_core": ooc.last_timing}
                return out
        w = scaffold_weights(n_samples)
        lr = float(aggregation_lr)
        isz = sdt.itemsize
        t0 = time.perf_counter()
        d_d = s.buffer(self._B_BUCKET, K * lay_d.ld * isz)
        d_cv = s.buffer(self._B_CV, K * lay_c.ld * isz)
        d_cc = s.buffer(self._B_C, Kc * lay_s.ld * isz)
        pre = 0
        host_mism = 0
        in_place: Dict[int, List[int]] = {}  # bucket slot -> the clients' own device rows (hand-off)
        self._handoff_keep = None
        for rows, lay, d, slot in ((parameters_updates, lay_d, d_d, self._B_BUCKET),
                                   (control_variate_updates, lay_c, d_cv, self._B_CV)):
            rows = [list(r) for r in rows]
            if self._take_prestaged(slot, d, lay.ld * isz, rows):
                pre += 1
                continue
            hand = self._handoff_into(s, rows, lay, d)  # simulation mode: the clients' exports, on the device
            if hand is False:
                self._stage_rows(s, rows, lay, d)
                continue
            tm["handoff_rows"] = tm.get("handoff_rows", 0) + len(rows)
            if isinstance(hand, list):
                in_place[slot] = hand
        c_rows = [list(r) for r in server_control_variates]
        c_ingested = host_c and self._take_prestaged(self._B_C, d_cc, lay_s.ld * isz, c_rows)
        # simulation mode: every client's c is its export, still on this GPU (handoff.py) -- one
        # copy device to device for the kernel, and the equality check on the device over the
        # recorded copies (what the host arrays hold, byte for byte) instead of host compares
        c_hits = None
        if host_c and not c_ingested and not same_c:
            c_hits = [handoff.lookup(r, s.device) for r in c_rows]
            if any(h is None or h[1] != lay_s.M * isz for h in c_hits):
                c_hits = None
        if same_c:
            # simulation mode with the hand-off: the clients return the c they received, which is
            # the previous call's output, still on this GPU (record_slot(stable=True) below)
            hit = handoff.lookup(c_rows[0], s.device)
            if hit is not None and hit[1] == lay_s.M * isz:
                s.copy_d2d(d_cc, hit[0], hit[1])
                s.sync()
                tm["c_handoff"] = True
            else:
                self._stage_rows(s, c_rows[:1], lay_s, d_cc)
        elif c_ingested:  # one copy staged and the others checked while ingest() was loading them
            host_mism = self._c_mism
        elif c_hits is not None:
            s.copy_d2d(d_cc, c_hits[0][0], c_hits[0][1])
        elif host_c:
            flats = [flat_of(r) for r in c_rows]
            if all(f is not None and f.size == lay_s.M for f in flats):
                c_rows = [[f] for f in flats]  # flat wire format: one segment per client
            host_mism = s.stage_check(d_cc, c_rows, sdt)
        else:
            self._stage_rows(s, c_rows, lay_s, d_cc)
        self._prestaged = {}
        tm["prestaged"] = pre == 2
        tm["c_check"] = "identity" if same_c else ("host-ingest" if c_ingested else "device-handoff" if c_hits
                                                   else "host" if host_c else "device")
        tm["stage_s"] = time.perf_counter() - t0
        t1 = time.perf_counter()
        cnt = s.buffer(self._B_CNT, 8)
        s.memset(cnt, 0, 8)
        if not same_c and not host_c:
            equal_count(kind, [d_cc + k * lay_s.ld * isz for k in range(K)], lay_s.M, cnt, s.stream)
        elif c_hits is not None:  # the recorded copies stay alive through `c_hits` until the fetch below
            equal_count(kind, [h[0] for h in c_hits], lay_s.M, cnt, s.stream)
        dout = s.buffer(self._B_OUT, lay_d.ld * 8)
        cout = s.buffer(self._B_COUT, lay_c.ld * 8)
        ws = s.buffer(self._B_WS, _native.load().fedagg_pairwise_ws_bytes(
            K, max(1, lay_d.pairwise_idx.size, lay_c.pairwise_idx.size), 8))
        rows_d = in_place.get(self._B_BUCKET) or [d_d + k * lay_d.ld * isz for k in range(K)]
        rows_c = in_place.get(self._B_CV) or [d_cv + k * lay_c.ld * isz for k in range(K)]
        if [g.shape for g in lay_d.segments] == [g.shape for g in lay_c.segments]:
            ScaffoldPlan(kind, rows_d, rows_c, d_cc, w, lay_d.M, lr, dout, cout, lay_d.pairwise_idx, ws).launch(s.stream)
        else:
            # delta and control-variate layers have different shapes: two passes of the fused
            # kernel, each one's other half written to scratch
            scratch = s.buffer(self._B_TMP, max(lay_d.ld, lay_c.ld) * 8 + 16)
            zeros = s.buffer(self._B_CNT + 1, lay_d.ld * isz)
            s.memset(zeros, 0, lay_d.ld * isz)
            ScaffoldPlan(kind, rows_d, rows_d, zeros, w, lay_d.M, lr, dout, scratch, lay_d.pairwise_idx,
                         ws).launch(s.stream)
            ScaffoldPlan(kind, rows_c, rows_c, d_cc, w, lay_c.M, lr, scratch, cout, lay_c.pairwise_idx,
                         ws).launch(s.stream)
        out_d = runtime.reusable_host_array(lay_d.M, np.float64, "scaffold-delta")
        out_c = runtime.reusable_host_array(lay_c.M, np.float64, "scaffold-c")
        mism = np.zeros(1, np.int64)
        s.fetch(cnt, mism)
        s.fetch(dout, out_d)
        s.fetch(cout, out_c)
        self._handoff_keep = None  # the kernels are done with the clients' buckets
        handoff.record_slot(out_d, s, self._B_OUT, dout)  # simulation mode: the clients copy them on the device
        if handoff.enabled():
            # c outlives this call on the device: the clients send it back as their c next round
            hc = s.buffer(self._B_HANDOFF_C, lay_c.ld * 8)
            s.copy_d2d(hc, cout, lay_c.M * 8)
            s.sync()
            handoff.record_slot(out_c, s, self._B_HANDOFF_C, hc, stable=True)
        tm["kernel_fetch_s"] = time.perf_counter() - t1
        avg = [a for _, a in lay_d.unpack(out_d, wire)]
        new_c = [a for _, a in lay_c.unpack(out_c, wire)]
        tm["total_s"] = time.perf_counter() - t_start
        return int(mism[0]) + host_mism, new_c, avg


_default_engine: Optional[AggregationEngine] = None


def default_engine() -> AggregationEngine:
    global _default_engine
    if _default_engine is None:
        _default_engine = AggregationEngine()
    return _default_engine


_engines: Dict[object, object] = {}


def _device_count() -> int:
    n = _native.load().fedagg_device_count()
    if n <= 0:
        raise _native.NativeLibraryError("no HIP device visible (the aggregation engine runs on MI355X only)")
    return n


def resolve_devices(device) -> Optional[object]:
    """``device`` as the strategies take it: ``None`` (``FEDAGG_DEVICES`` if set, else the
    single default GPU), an int, a sequence of ints, or ``"all"`` (every visible GPU)."""
    if device is None:
        env = os.environ.get("FEDAGG_DEVICES", "").strip()
        if not env:
            return None
        device = env
    if isinstance(device, str):
        if device == "all":
            return tuple(range(_device_count()))
        parts = [p for p in device.replace(" ", "").split(",") if p]
        return int(parts[0]) if len(parts) == 1 else tuple(int(p) for p in parts)
    if isinstance(device, (list, tuple)):
        return int(device[0]) if len(device) == 1 else tuple(int(d) for d in device)
    return int(device)


def engine_for(device=None):
    """The process-wide engine of ``device`` (see :func:`resolve_devices`), so rows staged by
    :meth:`AggregationEngine.ingest` are found by the aggregation call that follows.  Several
    devices give a :class:`multi_device.MultiDeviceEngine` (parameter-range shards, bit-exact)."""
    dev = resolve_devices(device)
    if dev is None:
        return default_engine()
    e = _engines.get(dev)
    if e is None:
        if isinstance(dev, tuple):
            from .multi_device import MultiDeviceEngine

            e = MultiDeviceEngine(dev)
        else:
            e = AggregationEngine(dev)
        _engines[dev] = e
    return e
