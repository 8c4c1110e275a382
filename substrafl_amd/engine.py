"""Aggregation engine: HBM buckets, HIP streams and launches of the libfedagg kernels.

Two entry levels:

* Device-resident plans (``FedAvgPlan`` / ``ScaffoldPlan``): client buckets already in HBM as
  one ``[K, ld]`` tensor; ``plan.launch(stream)`` enqueues the bucket kernel and the
  numel == 1 pairwise patch.  This is what ``bench.py`` times (BASELINE.json metric).
* Host entry (``AggregationEngine.fedavg`` / ``.scaffold``): the drop-in path behind
  ``FedAvg.avg_shared_states`` / ``Scaffold.avg_shared_states``.  Shared states arrive as host
  NumPy arrays (unpickled by ``RemoteMethod.generic_function``,
  substrafl/remote/substratools_methods.py:54-66), are packed into pinned staging buckets,
  copied H2D, reduced on the GPU, copied D2H into one owned array and returned as per-layer
  views.

PyTorch is used only for device memory, pinned host memory, streams and events.  Every
arithmetic step of the reduction runs in libfedagg's HIP kernels; if the library or a GPU is
missing the engine raises -- there is no CPU fallback.  The engine holds no cross-call state
(the reference aggregator is stateless per round: strategies/schemas.py:66-68) and initialises
the GPU lazily on first use (tests fork after import: tests/conftest.py:52-59), so strategies
that own an engine stay cloudpickle-able for RemoteStruct (remote_struct.py:84-114).
"""

from __future__ import annotations

import ctypes
import os
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _native
from .layout import BucketLayout

KINDS = ("f32", "bf16", "f64", "f16")


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
        self._out = int(out.data_ptr())
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
            self._ws = int(ws.data_ptr())
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
        self._c = int(c.data_ptr())
        self._w = (ctypes.c_double * self.K)(*[float(v) for v in np.asarray(weights, np.float64)])
        self._dout = int(delta_out.data_ptr())
        self._cout = int(c_out.data_ptr())
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
            self._ws = int(ws.data_ptr())
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
    _native.check(fn(_native.ptr_array(ptrs), len(ptrs), int(M), int(counter.data_ptr()), _stream_handle(stream)),
                  "equal_count")


def _row_pointers(clients) -> List[int]:
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
class AggregationEngine:
    """Per-process engine bound to one GPU (``device`` or ``LOCAL_RANK`` or 0), created lazily."""

    def __init__(self, device: Optional[int] = None, pack_threads: Optional[int] = None):
        self._device_index = device
        self._pack_threads = pack_threads
        self.last_timing: Dict[str, float] = {}

    # ----------------------------------------------------------------------------------
    def _setup(self):
        torch = _torch()
        _native.load()
        if not torch.cuda.is_available():
            raise _native.NativeLibraryError(
                "no ROCm GPU visible to this process: the aggregation engine runs on MI355X only (no CPU fallback)"
            )
        idx = self._device_index
        if idx is None:
            idx = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        self.device = torch.device("cuda", idx)
        return torch

    def _pool(self, n):
        t = self._pack_threads or min(8, os.cpu_count() or 1)
        return ThreadPoolExecutor(max_workers=max(1, min(t, n)))

    # ----------------------------------------------------------------------------------
    def _stage(self, rows: List[List[np.ndarray]], layout: BucketLayout, K: int):
        """Pack K clients' layers into a pinned [K, ld] staging buffer and copy it to HBM.

        Rows are packed by a thread pool; each row's H2D copy is enqueued as soon as that row is
        packed, so the PCIe transfer of client k overlaps the packing of the clients after it."""
        torch = self._setup() if not hasattr(self, "device") else _torch()
        tdt = torch_dtype(layout.dtype)
        t0 = time.perf_counter()
        host = torch.empty((K, layout.ld), dtype=tdt, pin_memory=True)
        t1 = time.perf_counter()
        dev = torch.empty((K, layout.ld), dtype=tdt, device=self.device)
        hv = host.numpy()
        if K > 1:
            with self._pool(K) as ex:
                futs = [ex.submit(layout.pack_row, rows[k], hv[k]) for k in range(K)]
                for k, f in enumerate(futs):
                    f.result()
                    dev[k].copy_(host[k], non_blocking=True)
        else:
            layout.pack_row(rows[0], hv[0])
            dev.copy_(host, non_blocking=True)
        t2 = time.perf_counter()
        tm = self.last_timing
        tm["pin_alloc_s"] = tm.get("pin_alloc_s", 0.0) + t1 - t0
        tm["pack_enqueue_s"] = tm.get("pack_enqueue_s", 0.0) + t2 - t1
        tm["h2d_bytes"] = tm.get("h2d_bytes", 0) + K * layout.ld * host.element_size()
        return dev, host

    def _fetch(self, dev_out, layout: BucketLayout) -> np.ndarray:
        torch = _torch()
        host = torch.empty(dev_out.shape, dtype=dev_out.dtype, pin_memory=True)
        host.copy_(dev_out, non_blocking=True)
        return host

    # ----------------------------------------------------------------------------------
    def fedavg(self, parameters_updates: List[List[np.ndarray]], n_samples: Sequence[int]) -> List[np.ndarray]:
        """GPU equivalent of fed_avg.py:217-222 for validated inputs (same layer count and shapes
        across clients, ``sum(n_samples) != 0``).  Returns one array per layer (0-d layers as
        NumPy scalars, like ``np.sum``)."""
        torch = self._setup()
        self.last_timing = {}
        t_start = time.perf_counter()
        K = len(parameters_updates)
        L = len(parameters_updates[0])
        if L == 0:
            return []
        # group layers by (result dtype, per-client product dtypes); NumPy promotion per layer
        groups: Dict[Tuple, List[int]] = {}
        for li in range(L):
            pds = tuple(np.result_type(pu[li].dtype, 1.0) for pu in parameters_updates)
            for d in pds:
                if d.kind != "f" or d not in (np.float16, np.float32, np.float64):
                    raise NotImplementedError(f"FedAvg engine: unsupported layer dtype {d}")
            R = np.result_type(*pds)
            key = (R.str, None if all(d == R for d in pds) else tuple(d.str for d in pds))
            groups.setdefault(key, []).append(li)

        stream = torch.cuda.current_stream(self.device)
        results: List[Optional[np.ndarray]] = [None] * L
        pending = []
        with torch.cuda.device(self.device):
            for (rstr, mixed), layer_ids in groups.items():
                R = np.dtype(rstr)
                kind = kind_of(R)
                shapes = [parameters_updates[0][li].shape for li in layer_ids]
                layout = BucketLayout(layer_ids, shapes, R)
                w = fedavg_weights(n_samples, kind)
                if mixed is None:
                    dev, host_in = self._stage(parameters_updates, layout, K)
                else:
                    dev, host_in = self._stage_mixed(parameters_updates, layout, K, mixed, n_samples)
                    w = np.ones(K, dtype=w.dtype)
                    for k, d in enumerate(mixed):
                        if np.dtype(d) == R:
                            w[k] = fedavg_weights(n_samples, kind)[k]
                out = torch.empty(layout.ld, dtype=torch_dtype(kind), device=self.device)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record(stream)  # after the H2D copies
                plan = FedAvgPlan(kind, dev, w, layout.M, out, layout.pairwise_idx)
                plan.launch(stream)
                ev[1].record(stream)
                host_out = self._fetch(out, layout)
                ev[2].record(stream)
                pending.append((layout, host_out, ev, host_in, dev, plan))
            t_wait = time.perf_counter()
            stream.synchronize()
            t_sync = time.perf_counter()
            kernel_ms = d2h_ms = 0.0
            for layout, host_out, ev, _hin, _dev, _plan in pending:
                kernel_ms += ev[0].elapsed_time(ev[1])
                d2h_ms += ev[1].elapsed_time(ev[2])
                # zero-copy: the per-layer views keep the pinned output block alive (its ndarray
                # base is the tensor), so it is recycled only once the caller drops the result
                flat = host_out.numpy()[: layout.M]
                for li, arr in layout.unpack(flat):
                    results[li] = arr
        tm = self.last_timing
        tm["kernel_s"] = kernel_ms / 1e3
        tm["d2h_s"] = d2h_ms / 1e3
        tm["sync_wait_s"] = t_sync - t_wait
        tm["unpack_s"] = time.perf_counter() - t_sync
        tm["total_s"] = time.perf_counter() - t_start
        return results  # type: ignore[return-value]

    def _stage_mixed(self, parameters_updates, layout: BucketLayout, K: int, pds, n_samples):
        """Mixed-dtype layer group (e.g. fp32 and fp64 clients): NumPy computes each client's
        product in its own dtype and then upcasts it when stacking (fed_avg.py:221-222).  Clients
        whose product dtype differs from the result dtype are pre-multiplied on the device in their
        own dtype (one IEEE multiply), cast exactly to the result dtype, and enter the bucket
        kernel with weight 1 (x * 1 is exact)."""
        torch = _torch()
        dev, host = self._stage(parameters_updates, layout, K)  # rows for same-dtype clients
        R = layout.dtype
        for k, d in enumerate(pds):
            d = np.dtype(d)
            if d == R:
                continue
            sub = BucketLayout([s.layer for s in layout.segments], [s.shape for s in layout.segments], d)
            h = np.empty(sub.ld, dtype=d)
            sub.pack_row(parameters_updates[k], h)
            t = torch.from_numpy(h[: sub.M]).to(self.device)
            wk = torch.tensor(fedavg_weights(n_samples, kind_of(d))[k], dtype=t.dtype, device=self.device)
            dev[k, : layout.M].copy_(torch.mul(t, wk).to(torch_dtype(R)))
        return dev, host

    # ----------------------------------------------------------------------------------
    def scaffold(
        self,
        parameters_updates: List[List[np.ndarray]],
        control_variate_updates: List[List[np.ndarray]],
        server_control_variates: List[List[np.ndarray]],
        n_samples: Sequence[int],
        aggregation_lr,
    ):
        """GPU equivalent of scaffold.py:193-196 (c equality check, returned as the mismatch
        count) and scaffold.py:297-337 (fp64 reductions).  Returns
        ``(mismatches, new_server_control_variate, avg_parameters_update)``."""
        torch = self._setup()
        self.last_timing = {}
        t_start = time.perf_counter()
        K = len(parameters_updates)
        L = len(parameters_updates[0])
        if L == 0:
            return 0, [], []
        all_f32 = all(
            a.dtype == np.float32
            for lst in (parameters_updates, control_variate_updates, server_control_variates)
            for client in lst
            for a in client
        )
        for lst in (parameters_updates, control_variate_updates, server_control_variates):
            for client in lst:
                for a in client:
                    if a.dtype.kind not in "biuf":
                        raise NotImplementedError(f"Scaffold engine: unsupported dtype {a.dtype}")
        kind = "f32" if all_f32 else "f64"
        sdt = np.float32 if all_f32 else np.float64
        lid = list(range(L))
        lay_d = BucketLayout(lid, [a.shape for a in parameters_updates[0]], sdt)
        lay_c = BucketLayout(lid, [a.shape for a in control_variate_updates[0]], sdt)
        lay_s = BucketLayout(lid, [a.shape for a in server_control_variates[0]], sdt)
        w = scaffold_weights(n_samples)
        lr = float(aggregation_lr)
        stream = torch.cuda.current_stream(self.device)
        with torch.cuda.device(self.device):
            d_dev, h1 = self._stage(parameters_updates, lay_d, K)
            c_dev, h2 = self._stage(control_variate_updates, lay_c, K)
            s_dev, h3 = self._stage(server_control_variates, lay_s, K)
            counter = torch.zeros(1, dtype=torch.int64, device=self.device)
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record(stream)
            equal_count(kind, s_dev, lay_s.M, counter, stream)
            same = [s.shape for s in lay_d.segments] == [s.shape for s in lay_c.segments]
            dout = torch.empty(lay_d.ld, dtype=torch.float64, device=self.device)
            cout = torch.empty(lay_c.ld, dtype=torch.float64, device=self.device)
            c_row = s_dev[0]
            if same:
                ScaffoldPlan(kind, d_dev, c_dev, c_row, w, lay_d.M, lr, dout, cout, lay_d.pairwise_idx).launch(stream)
            else:
                # delta and control-variate layers have different shapes: run the two
                # reductions as two passes of the fused kernel (the unused half is scratch)
                scratch_c = torch.empty(lay_d.ld, dtype=torch.float64, device=self.device)
                zeros = torch.zeros(lay_d.ld, dtype=d_dev.dtype, device=self.device)
                ScaffoldPlan(kind, d_dev, d_dev, zeros, w, lay_d.M, lr, dout, scratch_c,
                             lay_d.pairwise_idx).launch(stream)
                scratch_d = torch.empty(lay_c.ld, dtype=torch.float64, device=self.device)
                ScaffoldPlan(kind, c_dev, c_dev, c_row, w, lay_c.M, lr, scratch_d, cout,
                             lay_c.pairwise_idx).launch(stream)
            ev1.record(stream)
            hd = self._fetch(dout, lay_d)
            hc = self._fetch(cout, lay_c)
            hcnt = torch.empty(1, dtype=torch.int64, pin_memory=True)
            hcnt.copy_(counter, non_blocking=True)
            stream.synchronize()
            mismatches = int(hcnt.item())
            flat_d = np.array(hd.numpy()[: lay_d.M], copy=True)
            flat_c = np.array(hc.numpy()[: lay_c.M], copy=True)
        avg = [a for _, a in lay_d.unpack(flat_d)]
        new_c = [a for _, a in lay_c.unpack(flat_c)]
        self.last_timing["kernel_s"] = ev0.elapsed_time(ev1) / 1e3
        self.last_timing["total_s"] = time.perf_counter() - t_start
        return mismatches, new_c, avg


_default_engine: Optional[AggregationEngine] = None


def default_engine() -> AggregationEngine:
    global _default_engine
    if _default_engine is None:
        _default_engine = AggregationEngine()
    return _default_engine
