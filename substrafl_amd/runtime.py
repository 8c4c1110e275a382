"""Python handle on the native host runtime (``fedagg_session_*`` in include/fedagg.h).

A :class:`Session` owns one GPU, one HIP stream, grow-only HBM buffers and the pinned staging
ring of ``libfedagg.so``; the drop-in aggregation path (:mod:`substrafl_amd.engine`) runs
entirely through it, so an aggregate task process never creates a PyTorch CUDA context.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _native

KIND_CODE = {
    np.dtype(np.float16): 0,
    np.dtype(np.float32): 1,
    np.dtype(np.float64): 2,
    np.dtype(np.int8): 3,
    np.dtype(np.int16): 4,
    np.dtype(np.int32): 5,
    np.dtype(np.int64): 6,
    np.dtype(np.uint8): 7,
    np.dtype(np.uint16): 8,
    np.dtype(np.uint32): 9,
    np.dtype(np.uint64): 10,
    np.dtype(np.bool_): 11,
}


def kind_code(dtype) -> int:
    d = np.dtype(dtype)
    if d not in KIND_CODE:
        raise NotImplementedError(f"no device conversion for dtype {d}")
    return KIND_CODE[d]


class Session:
    """One GPU's native runtime context (create lazily; never pickled)."""

    def __init__(self, device: int = 0, threads: Optional[int] = None):
        self.lib = _native.load()
        h = self.lib.fedagg_session_create(int(device))
        if not h:
            raise _native.NativeLibraryError(
                "cannot open a HIP session on device %d: %s (the aggregation engine runs on MI355X only, "
                "no CPU fallback)" % (device, self.lib.fedagg_last_error().decode(errors="replace"))
            )
        self._h = ctypes.c_void_p(h)
        self.device = int(device)
        self._held: Dict[int, int] = {}
        self._ptr: Dict[int, int] = {}
        # write generation per buffer slot: bumped by every call that writes into the slot
        # (stage, cast, memset, regrowth), so a record of rows staged earlier (engine.ingest) can
        # tell whether any engine sharing this session has written the slot since
        self._gen: Dict[int, int] = {}
        self.stream = int(self.lib.fedagg_session_stream(self._h) or 0)
        nthreads = threads or int(os.environ.get("FEDAGG_PACK_THREADS", "0")) or min(16, os.cpu_count() or 1)
        self.set("threads", nthreads)
        if os.environ.get("FEDAGG_COPY_STREAMS"):  # measurement switch: 1 or 2 H2D queues (default 2)
            self.set("copy_streams", int(os.environ["FEDAGG_COPY_STREAMS"]))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.fedagg_session_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __reduce__(self):
        raise TypeError("a Session holds a GPU context and cannot be pickled")

    # ----------------------------------------------------------------------------------
    def set(self, key: str, value: int) -> None:
        _native.check(self.lib.fedagg_session_set(self._h, key.encode(), int(value)), f"session_set({key})")

    def affinity(self, cpus: Optional[Sequence[int]]) -> None:
        """Bind this session's pack workers, and allocate its pinned ring, on ``cpus`` (None or
        empty: no binding) -- ``fedagg_session_affinity``; the ring is re-allocated at the next
        stage / fetch."""
        cpus = [int(c) for c in (cpus or [])]
        arr = (ctypes.c_int * max(1, len(cpus)))(*cpus)
        _native.check(self.lib.fedagg_session_affinity(self._h, arr, len(cpus)), "session_affinity")

    def ring_node(self) -> int:
        """NUMA node of the pinned staging ring's pages (-1: unknown, or not allocated yet)."""
        return int(self.lib.fedagg_session_ring_node(self._h))

    def warm(self, slot_bytes: Dict[int, int]) -> None:
        """Pinned ring, worker pool, HBM buffers ``{slot: bytes}`` and the kernels' code object,
        ahead of the first aggregation (``fedagg_session_warm``)."""
        n = _native.FEDAGG_SESSION_BUFFERS
        arr = (ctypes.c_uint64 * n)(*[int(slot_bytes.get(i, 0)) for i in range(n)])
        _native.check(self.lib.fedagg_session_warm(self._h, arr, n), "session_warm")

    def held_bytes(self, slots: Optional[Sequence[int]] = None) -> int:
        """HBM held by this session's grow-only buffers (all, or only ``slots``: the buffers a
        call will reuse -- the others stay allocated and are not free for it)."""
        if slots is None:
            return sum(self._held.values())
        return sum(self._held.get(int(k), 0) for k in set(slots))

    def buffer(self, slot: int, nbytes: int) -> int:
        slot = int(slot)
        need = max(16, int(nbytes))
        grew = need > self._held.get(slot, 0)  # the native slot reallocates: contents undefined
        self._held[slot] = max(self._held.get(slot, 0), need)
        p = ctypes.c_void_p()
        _native.check(self.lib.fedagg_session_buffer(self._h, slot, need, ctypes.byref(p)), "session_buffer")
        if grew or self._ptr.get(slot) != int(p.value):
            # bumped on every regrowth, even when hipMalloc hands back the same address
            self._ptr[slot] = int(p.value)
            self._gen[slot] = self._gen.get(slot, 0) + 1
        return int(p.value)

    # ----------------------------------------------------------------------------------
    def _slot_of(self, d: int) -> Optional[int]:
        for slot, base in self._ptr.items():
            if base <= d < base + self._held.get(slot, 0):
                return slot
        return None

    def _bump(self, d: int) -> None:
        slot = self._slot_of(int(d))
        if slot is not None:
            self._gen[slot] = self._gen.get(slot, 0) + 1

    def generation(self, slot: int) -> int:
        """Write generation of buffer ``slot`` (see ``_gen``)."""
        return self._gen.get(int(slot), 0)

    def stage(self, d_dst: int, ld_bytes: int, rows: Sequence[Sequence[np.ndarray]],
              byte_range: Optional[tuple] = None) -> None:
        """rows[k] = client k's host arrays, in bucket order, each C-contiguous; row k lands at
        ``d_dst + k * ld_bytes``.  ``byte_range=(lo, hi)`` stages only bytes ``[lo, hi)`` of every
        row (a parameter-range shard), to ``d_dst + k * ld_bytes`` likewise."""
        K = len(rows)
        nseg, ptrs, sizes, keep = _segments(rows)
        self._bump(d_dst)
        if byte_range is None:
            _native.check(self.lib.fedagg_session_stage(self._h, ctypes.c_void_p(d_dst), int(ld_bytes), K, nseg,
                                                        ptrs, sizes), "session_stage")
        else:
            lo, hi = (int(v) for v in byte_range)
            _native.check(self.lib.fedagg_session_stage_range(self._h, ctypes.c_void_p(d_dst), int(ld_bytes), K,
                                                              nseg, ptrs, sizes, lo, hi), "session_stage_range")

    def stage_tiled(self, d_dst: int, tile_bytes: int, rows: Sequence[Sequence[np.ndarray]]) -> None:
        """rows[k] = client k's host arrays (bucket order) into the tile-interleaved layout of
        ``engine.TiledFedAvgPlan``: tile t of row k at ``d_dst + (t * K + k) * tile_bytes``
        (``fedagg_session_stage_tiled``)."""
        nseg, ptrs, sizes, keep = _segments(rows)
        self._bump(d_dst)
        _native.check(self.lib.fedagg_session_stage_tiled(self._h, ctypes.c_void_p(d_dst), int(tile_bytes), len(rows),
                                                          nseg, ptrs, sizes), "session_stage_tiled")

    def stage_tiled_row(self, d_dst: int, tile_bytes: int, K: int, k: int, row: Sequence[np.ndarray]) -> None:
        """Client ``k``'s host arrays (bucket order) alone into the tile-interleaved layout of K
        clients: its tile t at ``d_dst + (t * K + k) * tile_bytes``
        (``fedagg_session_stage_tiled_row``; the other clients' tiles are left as they are)."""
        nseg, ptrs, sizes, keep = _segments([row])
        self._bump(d_dst)
        _native.check(self.lib.fedagg_session_stage_tiled_row(self._h, ctypes.c_void_p(d_dst), int(tile_bytes), int(K),
                                                              int(k), nseg, ptrs, sizes), "session_stage_tiled_row")

    def stage_check(self, d_dst: int, rows: Sequence[Sequence[np.ndarray]], dtype,
                    byte_range: Optional[tuple] = None) -> int:
        """Stage ``rows[0]`` (bytes ``byte_range`` of it, default all) to ``d_dst`` and compare the
        same bytes of every other row with it by value on the host
        (``fedagg_session_stage_check``: Scaffold's server-control-variate check,
        scaffold.py:193-196).  Returns the number of mismatching elements."""
        kind = {np.dtype(np.float32): _native.FEDAGG_F32, np.dtype(np.float64): _native.FEDAGG_F64}[np.dtype(dtype)]
        nseg, ptrs, sizes, keep = _segments(rows)
        for row in rows:
            for a in row:
                if a.dtype != dtype:
                    raise ValueError("stage_check: every array must have the checked dtype")
        lo, hi = (0, sum(int(sizes[i]) for i in range(nseg))) if byte_range is None else byte_range
        if d_dst:
            self._bump(d_dst)
        mism = ctypes.c_uint64(0)
        _native.check(self.lib.fedagg_session_stage_check(self._h, ctypes.c_void_p(d_dst), len(rows), nseg, ptrs,
                                                          sizes, int(lo), int(hi), kind, ctypes.byref(mism)),
                      "session_stage_check")
        return int(mism.value)

    def check(self, rows: Sequence[Sequence[np.ndarray]], dtype) -> int:
        """Value mismatches of rows[1:] against rows[0] on the pack workers (nothing staged)."""
        return self.stage_check(0, rows, dtype)

    def event_record(self, ev: int) -> None:
        _native.check(self.lib.fedagg_session_event_record(self._h, int(ev)), "session_event_record")

    def event_elapsed_ms(self, ev0: int, ev1: int) -> float:
        ms = ctypes.c_float()
        _native.check(self.lib.fedagg_session_event_elapsed(self._h, int(ev0), int(ev1), ctypes.byref(ms)),
                      "session_event_elapsed")
        return float(ms.value)

    def activate(self) -> None:
        """Make this session's GPU the calling thread's current device (before kernel launches)."""
        _native.check(self.lib.fedagg_session_activate(self._h), "session_activate")

    def fetch(self, d_src: int, out: np.ndarray) -> np.ndarray:
        """Copy ``out.nbytes`` from HBM into ``out`` (synchronous; ``out`` may be a contiguous
        slice of a larger array)."""
        if not out.flags.c_contiguous:
            raise ValueError("fetch destination must be C-contiguous")
        _native.check(self.lib.fedagg_session_fetch(self._h, ctypes.c_void_p(d_src),
                                                    ctypes.c_void_p(out.ctypes.data), out.nbytes), "session_fetch")
        return out

    def memset(self, d: int, value: int, nbytes: int) -> None:
        self._bump(d)
        _native.check(self.lib.fedagg_session_memset(self._h, ctypes.c_void_p(d), int(value), int(nbytes)),
                      "session_memset")

    def copy_d2d(self, d_dst: int, d_src: int, nbytes: int) -> None:
        """Device-to-device copy on the session stream (``fedagg_session_copy_d2d``)."""
        self._bump(d_dst)
        _native.check(self.lib.fedagg_session_copy_d2d(self._h, ctypes.c_void_p(d_dst), ctypes.c_void_p(d_src),
                                                       int(nbytes)), "session_copy_d2d")

    def sync(self) -> None:
        _native.check(self.lib.fedagg_session_sync(self._h), "session_sync")

    def timing(self) -> Dict[str, float]:
        a, b = ctypes.c_double(), ctypes.c_double()
        self.lib.fedagg_session_timing(self._h, ctypes.byref(a), ctypes.byref(b))
        return {"stage_s": a.value, "fetch_s": b.value}

    PHASES = ("hip_init_s", "streams_s", "ring_s", "pool_s", "buffers_s", "code_object_s")

    def phases(self) -> Dict[str, float]:
        """Start-up phases of this session (``fedagg_session_phases``): the HIP runtime's start and
        the device, the streams, then the warm's pinned ring, worker pool, HBM buffers and
        code-object load; seconds, 0.0 for a phase that has not run."""
        n = _native.FEDAGG_SESSION_PHASES
        out = (ctypes.c_double * n)()
        _native.check(self.lib.fedagg_session_phases(self._h, out, n), "session_phases")
        return {k: round(float(v), 6) for k, v in zip(self.PHASES, out)}

    # ----------------------------------------------------------------------------------
    def cast(self, d_in: int, in_dtype, d_out: int, out_dtype, n: int) -> None:
        self._bump(d_out)
        _native.check(self.lib.fedagg_cast(ctypes.c_void_p(d_in), kind_code(in_dtype), ctypes.c_void_p(d_out),
                                           kind_code(out_dtype), int(n), ctypes.c_void_p(self.stream)), "cast")

    def scale_cast(self, d_in: int, in_dtype, w: float, d_out: int, out_dtype, n: int) -> None:
        self._bump(d_out)
        _native.check(self.lib.fedagg_scale_cast(ctypes.c_void_p(d_in), kind_code(in_dtype), float(w),
                                                 ctypes.c_void_p(d_out), kind_code(out_dtype), int(n),
                                                 ctypes.c_void_p(self.stream)), "scale_cast")


def _segments(rows: Sequence[Sequence[np.ndarray]]):
    """ctypes tables of K rows of nseg C-contiguous host arrays: (nseg, pointers, sizes, keep)."""
    K = len(rows)
    nseg = len(rows[0]) if K else 0
    keep: List[np.ndarray] = []
    ptrs = (ctypes.c_void_p * max(1, K * nseg))()
    sizes = (ctypes.c_uint64 * max(1, nseg))()
    for k, row in enumerate(rows):
        if len(row) != nseg:
            raise ValueError("every client row needs the same segments")
        for i, a in enumerate(row):
            a = np.ascontiguousarray(a)
            keep.append(a)
            ptrs[k * nseg + i] = a.ctypes.data if a.nbytes else None
            if k == 0:
                sizes[i] = a.nbytes
            elif a.nbytes != sizes[i]:
                raise ValueError("segment sizes differ between clients")
    return nseg, ptrs, sizes, keep


_device_locks: Dict[int, threading.RLock] = {}


def device_lock(device: int) -> threading.RLock:
    """The lock that serialises aggregation calls on ``device``: its session's buffers and stream
    are shared by every engine of the process (the reference runs one aggregation at a time;
    this keeps concurrent callers correct rather than racing on the HBM buffers)."""
    with _lock:
        lk = _device_locks.get(int(device))
        if lk is None:
            lk = _device_locks[int(device)] = threading.RLock()
        return lk


_host_cache: Dict[tuple, dict] = {}
_host_lock = threading.Lock()
HOST_POOL_DEPTH = 64  # buffers kept per call site and dtype ...
HOST_POOL_BYTES = 16 << 30  # ... within this many bytes
HOST_POOL_IDLE = 2  # a free buffer not handed out again within this many turns of its pool is released


def reusable_host_array(n: int, dtype, tag: str) -> np.ndarray:
    """A host array of ``n`` elements for a D2H result (``tag`` names the call site).  A fresh
    100 MB allocation costs ~8 ms of first-touch page faults (glibc maps every block above 32 MiB
    anew), three times the D2H itself, so earlier calls' buffers are recycled -- but only one that
    nothing references any more (every array handed out from it was a view holding it), so no
    caller ever sees its data change.  The pool follows the site's working set: in simulation mode
    the previous round's results are still held while the next round's are made (the strategy
    keeps its last train states, and its last average, until the new ones are returned), K
    clients' exports of two rounds at once, so it grows to that and then recycles it; a free buffer
    not handed out again within ``HOST_POOL_IDLE`` turns of the pool (one turn = as many requests
    as the pool holds buffers) is released, so a working set that shrinks gives its buffers back
    (ADVICE r05); ``HOST_POOL_DEPTH`` / ``HOST_POOL_BYTES`` bound it, the least recently used going
    first (its holders keep it; it is freed with them)."""
    import sys

    key = (tag, np.dtype(dtype))
    with _host_lock:
        site = _host_cache.setdefault(key, {"tick": 0, "pool": []})
        site["tick"] += 1
        tick, pool = site["tick"], site["pool"]  # entries [buffer, tick of its last hand-out]
        out = None
        # the most recently used free buffer first (warm pages; the others can age out)
        for i in range(len(pool) - 1, -1, -1):  # (not enumerate: its cached tuple would hold one more reference)
            buf = pool[i][0]
            # references: the entry, the local name and getrefcount's argument; a live view adds one
            if buf.size >= n and sys.getrefcount(buf) <= 3:
                ent = pool.pop(i)
                ent[1] = tick
                pool.append(ent)  # most recently used last
                buf.flags.writeable = True  # a device hand-off (handoff.py) may have frozen it
                out = buf[:n]
                break
        buf = None
        if out is None:
            out = np.empty(n, dtype=key[1])
            pool.append([out, tick])
        idle = HOST_POOL_IDLE * max(2, len(pool))
        keep = []
        for ent in pool:  # free buffers idle past the working set go (a held one stays listed)
            b = ent[0]
            if tick - ent[1] > idle and b is not out and b is not getattr(out, "base", None) \
                    and sys.getrefcount(b) <= 3:
                continue
            keep.append(ent)
        b = None
        pool[:] = keep
        while len(pool) > 1 and (len(pool) > HOST_POOL_DEPTH or sum(e[0].nbytes for e in pool) > HOST_POOL_BYTES):
            pool.pop(0)  # the least recently used; still alive through its holders' views, if any
        return out


def drop_host_pools() -> None:
    """Forget the recycled result buffers: each is freed once nothing else holds it."""
    with _host_lock:
        _host_cache.clear()


def device_pci_bus_id(device: int) -> str:
    """``dddd:bb:dd.f`` of ``device`` (hipDeviceGetPCIBusId), lower case as sysfs names it."""
    lib = _native.load()
    buf = ctypes.create_string_buffer(64)
    _native.check(lib.fedagg_device_pci_bus_id(int(device), buf, len(buf)), "device_pci_bus_id")
    return buf.value.decode().lower()


def device_memory(device: int) -> tuple:
    """``(free, total)`` HBM bytes of ``device`` (``hipMemGetInfo``)."""
    lib = _native.load()
    f, t = ctypes.c_uint64(), ctypes.c_uint64()
    _native.check(lib.fedagg_device_memory(int(device), ctypes.byref(f), ctypes.byref(t)), "device_memory")
    return int(f.value), int(t.value)


_sessions: Dict[int, Session] = {}
_lock = threading.Lock()
_warming: Dict[int, threading.Thread] = {}
_warm_errors: Dict[int, BaseException] = {}
warm_times: Dict[int, tuple] = {}  # device -> (perf_counter at start, at end) of the last prewarm
# device -> the prewarm's phases, seconds (VERDICT r05 "Next 4"): library_load_s (dlopen of
# libfedagg.so and its code object's registration), session_s (the session object: the native
# create below plus the Python side), then Session.phases() -- hip_init_s, streams_s, ring_s,
# pool_s, buffers_s, code_object_s -- and total_s; "created_by_prewarm" False when another caller
# had opened the session first (its create phases were then paid there)
warm_phases: Dict[int, dict] = {}


def session(device: int = 0) -> Session:
    """The process-wide session of ``device`` (created on first use; waits for a
    :func:`prewarm` of that device still in flight)."""
    t = _warming.get(device)
    if t is not None and t is not threading.current_thread():
        t.join()
    with _lock:
        s = _sessions.get(device)
        if s is None:
            s = _sessions[device] = Session(device)
        return s


def prewarm(device: int = 0, slot_bytes: Optional[Dict[int, int]] = None) -> threading.Thread:
    """Open ``device``'s session and warm it (:meth:`Session.warm`) on a background thread, so a
    one-shot aggregate task pays HIP start-up, pinned-ring and HBM allocation while it is still
    unpickling its inputs.  Idempotent per device; a failure here is not raised -- the real call
    opens the session itself and reports the error then."""
    with _lock:
        t = _warming.get(device)
        if t is not None:
            return t

        def run():
            import time

            t0 = time.perf_counter()
            ph: Dict[str, object] = {}
            try:
                _native.load()
                t1 = time.perf_counter()
                ph["library_load_s"] = round(t1 - t0, 6)
                with _lock:
                    created = device not in _sessions
                s = session(device)
                ph["session_s"] = round(time.perf_counter() - t1, 6)
                ph["created_by_prewarm"] = created
                s.warm(slot_bytes or {})
                ph.update(s.phases())
            except BaseException as e:  # noqa: BLE001 - surfaced by the aggregation call
                _warm_errors[device] = e
            t_end = time.perf_counter()
            ph["total_s"] = round(t_end - t0, 6)
            warm_phases[device] = ph
            warm_times[device] = (t0, t_end)

        t = threading.Thread(target=run, name=f"fedagg-prewarm-{device}", daemon=True)
        _warming[device] = t
    t.start()
    return t
