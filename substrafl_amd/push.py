"""Push executor of the client-sharded lockstep schedules (``fedagg_push_execute``,
csrc/lockstep.hip; DESIGN.md §6 "Push").

The RCCL executor (:mod:`rccl`) moves each step's accumulators with RCCL's P2P kernels, which on
MI355X hide only part of their time under an HBM-saturating chain kernel (DESIGN.md §6
"Overlap").  Here there are no exchange kernels: a run's chain kernel writes its accumulator
straight into the consumer's slot -- or, for a finished piece, into the root's output -- through
an IPC mapping of the peer's buffer (xGMI stores, 1/65 of the kernel's traffic at C3), continuing
its input accumulator read from this rank's own slot (``fedagg_fedavg_chain_push_{f32,bf16}``:
the same per-element order as the chain kernels, fed_avg.py:221-222).  Order across the processes: one monotonic
progress counter per rank in a node-shared host page, polled before a step by a one-lane wait kernel and published by a
one-lane signal kernel on entry to a call (``base + 1``: the rank's earlier stream work -- a
refill of its output, the previous call -- is done) and after each step t (``base + t + 2``).
Before step t a rank waits for

* each producer of its step-t inputs to have finished step t - 2 (the inputs landed), and
* each consumer of its step-t outputs to have finished step t - 2 (the consumer read the slot
  it is about to overwrite at that step: slot t % SLOTS, SLOTS = 4), or at least to have
  entered the call (steps 0 and 1, the root's output for finished pieces, its staging row);

after the last step the root waits for every rank's last step.

A counter reaches host memory over PCIe while the data of the same step travels over xGMI into
the consumer's HBM, so the counter alone does not prove the data landed.  Landing tags close that
gap: a run storing into a peer (``FEDAGG_RUN_FEDAVG_PUSH``, the Scaffold push runs) writes with
system-scope write-through stores (``sc0 sc1``) and every wave waits for their acknowledgement
(``s_waitcnt vmcnt(0)``) before it retires -- no L2 writeback, no release fence: the stores are
acknowledged by the memory they target (only ``push_copy_kernel``, the root's landing copies and
staging row, ends with a release fence) -- and the step's signal kernel, behind those runs on the
stream, then writes the call's generation into one tag word per consumer it pushed to -- in the
consumer's own HBM, over the same link as the data -- before it publishes the counter.  A consumer waits for the producer's counter AND the tag
before it reads the pushes (at step t + 2, or after its last step for finished pieces and the
staging row); a tag found missing once the counter was there is counted (``late_tags``: the gap,
measured on the node) and waited out, and one that never comes is a timeout error, not a wrong
number: the wait records what it waited for in its rank's error word, every other wait of the
group gives up as soon as it sees a set error word (one timeout per failure, not one per wait), and
``client_sharded_fedavg`` / ``client_sharded_scaffold`` raise on every rank that waited, after
synchronising (never returning the root's output).  A failed transport stays failed.  Every wait points to a strictly earlier step of another rank, so the schedule cannot
deadlock whatever hardware queues the kernels share.  The numel == 1 products go to a staging row of the
root per rank (one copy after step 0's waits) and are summed on the root (one owner per column: exact).

Scope: row-layout client blocks of FedAvg over fp32 (the bench's C3 schedule) or bf16 buckets
(C5; fp32 accumulators), and of Scaffold over fp32 or fp64 buckets (fp64 accumulators: each run is
two launches, the delta bucket and the control-variate bucket, ``fedagg_scaffold_chain_push_*``,
scaffold.py:262-263, 293); FedAvg's fp64 / fp16 kinds keep the RCCL executor.  Every rank must be
on this node (the counters live in ``/dev/shm``).
"""

from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _native, lockstep
from .rccl import _Run

PAGE = 4096


class _Wait(ctypes.Structure):
    _fields_ = [("step", ctypes.c_int32), ("rank", ctypes.c_int32), ("value", ctypes.c_int64),
                ("tag", ctypes.c_void_p)]


class _Tag(ctypes.Structure):
    _fields_ = [("step", ctypes.c_int32), ("reserved", ctypes.c_int32), ("tag", ctypes.c_void_p)]


class _Copy(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("src", ctypes.c_void_p), ("bytes", ctypes.c_uint64)]


# include/fedagg.h fedagg_push_wait / _tag / _copy
assert ctypes.sizeof(_Wait) == 24 and ctypes.sizeof(_Tag) == 16 and ctypes.sizeof(_Copy) == 24

GPU_MAX_HW_QUEUES = 4  # HIP's hardware queues per process on the boxes (GPU_MAX_HW_QUEUES, HIP's default)
RCCL_STREAMS = 3  # a live fedagg_comm: its own stream + RCCL's internal device and host streams


def aux_stream_budget(hw_queues: int = GPU_MAX_HW_QUEUES, rccl_live: bool = False) -> int:
    """Aux streams the push executor may spread a step's per-consumer launches over: what the
    hardware queues leave after the caller's stream (and, with a native RCCL communicator live in
    the same process, after its stream and RCCL's own two), at most 3.  More streams than queues
    share queues and serialise anyway (DESIGN.md §6 "Streams")."""
    return max(0, min(3, hw_queues - 1 - (RCCL_STREAMS if rccl_live else 0)))


def _check(rc: int, what: str) -> None:
    if rc != 0:
        lib = _native.load()
        msg = lib.fedagg_comm_last_error().decode(errors="replace") or lib.fedagg_last_error().decode(errors="replace")
        raise _native.NativeLibraryError(f"{what} failed ({rc}): {msg}")


class PushTransport:
    """The push executor over the ranks of ``group`` (a torch.distributed group -- gloo is
    enough: it carries only the set-up handshakes)."""

    native = True
    push = True
    fault: Optional[Tuple[str, int, int]] = None  # TEST ONLY: see __init__
    _settle_failed = False  # settle() ran out of time: some rank neither finished nor failed
    _timeout_s = 60.0

    def __init__(self, group=None, device: Optional[int] = None, timeout_s: float = 60.0,
                 aux_streams: Optional[int] = None, fault: Optional[Tuple[str, int, int]] = None):
        """``timeout_s``: how long a wait kernel polls before it gives up (the call then raises on
        every rank that waited, naming what it waited for; the transport stays failed).
        ``fault``: TEST ONLY (tests/test_push_gpu.py), a failure injected on one rank:
        ``("signal", rank, t)`` -- that rank stops before its step t, so it never signals step t
        (a peer stuck mid-call); ``("exit", rank, t)`` -- the same, then that rank's process exits
        without releasing anything (a peer that died mid-call: it never meets another collective);
        ``("tag", rank, i)`` -- that rank never writes the i-th landing tag of its program (its data
        lands, the proof of it never does)."""
        import torch
        import torch.distributed as dist
        from multiprocessing import shared_memory

        self.lib = _native.load()
        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.device = torch.cuda.current_device() if device is None else int(device)
        # counters [0, G), wait errors [G, 2G), late landing tags [2G, 3G)
        nbytes = PAGE * max(1, -(-(3 * self.world * 8) // PAGE))
        name = [None]
        if self.rank == 0:
            self._shm = shared_memory.SharedMemory(create=True, size=nbytes)
            self._shm.buf[:nbytes] = bytes(nbytes)
            name = [self._shm.name]
        self._src0 = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(name, src=self._src0, group=group)
        if self.rank != 0:
            self._shm = shared_memory.SharedMemory(name=name[0])
        self._page = np.frombuffer(self._shm.buf, dtype=np.uint64, count=nbytes // 8)
        dev = ctypes.c_void_p()
        _check(self.lib.fedagg_host_map(self._page.ctypes.data, nbytes, ctypes.byref(dev)), "fedagg_host_map")
        self._dev = dev.value
        hz = ctypes.c_uint64()
        _check(self.lib.fedagg_wall_clock_hz(ctypes.byref(hz)), "fedagg_wall_clock_hz")
        self._timeout = int(timeout_s * hz.value)
        self._timeout_s = float(timeout_s)
        self._settle_failed = False  # settle() ran out of time: some rank neither finished nor failed
        self.base = 0
        if fault is not None and (fault[0] not in ("signal", "exit", "tag") or len(fault) != 3):
            raise ValueError(f"push fault injection: ('signal' | 'exit' | 'tag', rank, step | index), not {fault!r}")
        self.fault = fault
        self._maps: Dict[bytes, int] = {}
        self._programs: List["PushProgram"] = []
        self._py = None
        n_aux = aux_stream_budget(_hw_queues()) if aux_streams is None else int(aux_streams)
        self._aux = [torch.cuda.Stream(device=self.device) for _ in range(n_aux)]
        self._aux_ptrs = _native.ptr_array([st.cuda_stream for st in self._aux])
        dist.barrier(group=group)

    # -- set-up helpers --------------------------------------------------------------------
    def ipc_info(self, ptr: int) -> Tuple[bytes, int]:
        """(handle, byte offset) of a device address."""
        h = (ctypes.c_char * _native_ipc_bytes())()
        off = ctypes.c_uint64()
        _check(self.lib.fedagg_ipc_get(int(ptr), h, ctypes.byref(off)), "fedagg_ipc_get")
        return bytes(h.raw), int(off.value)

    def remote(self, info: Tuple[bytes, int], owner: Optional["PushProgram"] = None) -> int:
        """Address, in this process, of another rank's (handle, offset); ``owner``: the program the
        mapping belongs to (closed with it, :meth:`release_programs`)."""
        h, off = info
        if h not in self._maps:
            base = ctypes.c_void_p()
            buf = (ctypes.c_char * len(h)).from_buffer_copy(h)
            _check(self.lib.fedagg_ipc_open(buf, ctypes.byref(base)), "fedagg_ipc_open")
            self._maps[h] = int(base.value)
        if owner is not None:
            owner._handles.add(h)
        return self._maps[h] + off

    def release_programs(self) -> None:
        """Free every compiled program: its uncached slots / landing / tag / staging buffers and the
        IPC mappings of the peers' ones.  Collective (every rank at once): this rank's stream is
        synchronised and the group meets first, so no rank's kernels still read or write what goes
        away.  Without it each call with new client blocks (the host entry points) would keep a
        program -- and every peer's mappings of its buffers -- alive."""
        if not self._programs:
            return
        import torch

        torch.cuda.synchronize(self.device)
        self.settle()
        if self.failed():
            # a rank whose peer died would wait in this barrier for the backend's timeout, and a
            # gloo barrier that raises would replace the error that names the failed wait: after a
            # failure nothing collective runs, the buffers stay allocated
            self._abandon_programs()
            return
        if self.world > 1:
            self.dist.barrier(group=self.group)
        for p in self._programs:
            for h in p._handles:
                base = self._maps.pop(h, None)
                if base is not None:
                    self.lib.fedagg_ipc_close(base)
        self._programs = []

    def all_gather(self, obj) -> list:
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def all_sum_int(self, v: int) -> int:
        import torch

        t = torch.tensor([int(v)], dtype=torch.int64)
        self.dist.all_reduce(t, group=self.group)
        return int(t.item())

    def python_transport(self):
        """The torch.distributed transport of the same group (sharding.DistTransport) for what this
        executor does not run; its backend must carry device tensors (RCCL)."""
        if self._py is None:
            from .sharding import DistTransport

            self._py = DistTransport(self.group)
        return self._py

    def errors(self) -> Dict[int, str]:
        """Ranks whose wait kernel gave up: rank -> what it waited for (a rank's progress counter,
        or the landing tag of a rank's push), or which rank's failure it stopped waiting after."""
        e = self._page[self.world: 2 * self.world]
        return {r: _describe_wait_error(int(v)) for r, v in enumerate(e) if v}

    def late_tags(self) -> List[int]:
        """Per rank: landing-tag waits that found the producer's counter published but its data's
        tag not yet landed (the PCIe-counter / xGMI-data ordering gap, waited out), cumulative."""
        return [int(v) for v in self._page[2 * self.world: 3 * self.world]]

    # -- the schedule ----------------------------------------------------------------------
    def program(self, **kw) -> "PushProgram":
        """The compiled program of this schedule and these buffers: the cached one when the call
        repeats (same plan, client blocks and outputs: the device-resident loop), else a new one --
        the cached program is released first (collective, like the compile), so one program's
        buffers and mappings are alive at a time."""
        self.raise_errors()  # a failed group cannot compile a program (its set-up is collective)
        for p in self._programs:
            if p.matches(**kw):
                p.rebase_outs(kw["outs"])
                return p
        self.release_programs()
        p = PushProgram(self, **kw)
        self._programs = [p]
        return p

    def raise_errors(self) -> None:
        """Raise if any rank's wait kernel gave up: that rank went on with inputs that had not
        landed, so the call's result is wrong.  Read it once the executing stream is synchronised
        (the root's last wait follows every rank's last step, so its synchronisation covers all
        ranks' waits); :meth:`execute` also checks it before issuing the next call."""
        bad = self.errors()
        if bad:
            raise _native.NativeLibraryError(f"push executor: a wait timed out (rank -> what it waited for: {bad})")
        if self._settle_failed:
            raise _native.NativeLibraryError("push executor: a rank neither finished the call nor reported a failed "
                                             f"wait within {self._timeout_s + 5.0:.0f} s")

    def execute(self, prog: "PushProgram", stream: int, ws=None, ws_kind: str = "f32") -> None:
        self.raise_errors()
        ws_src = ws_dst = None
        ws_bytes = 0
        if ws is not None and self.world > 1:
            ws_bytes = ws.numel() * ws.element_size()
            ws_src, ws_dst = ws.data_ptr(), prog.ws_dst(ws_bytes)
        root = self.rank == prog.plan.root and self.world > 1
        stage = prog.stage_u.ptr if root and ws_bytes else None
        ncopies = prog.ncopies if root else 0
        # a native RCCL communicator live in this process holds three streams of the hardware queues
        from .rccl import RcclTransport

        naux = min(len(self._aux), aux_stream_budget(_hw_queues(), RcclTransport.live() > 0))
        runs, nruns, waits, nwaits, tags, ntags, nsteps = (prog.runs, prog.nruns, prog.waits, prog.nwaits, prog.tags,
                                                           prog.ntags, prog.nsteps)
        if self.fault is not None and self.fault[1] == self.rank:  # TEST ONLY: the injected failure
            what, _r, at = self.fault
            if what in ("signal", "exit"):  # stop before step `at`: its signal (and every later one) never comes
                keep = lambda arr, n: [x for x in arr[:n] if x.step < at]  # noqa: E731
                r_, w_, t_ = keep(runs, nruns), keep(waits, nwaits), keep(tags, ntags)
                nsteps, ws_src, ws_dst, ws_bytes, stage, ncopies = min(at, nsteps), None, None, 0, None, 0
            else:  # the at-th landing tag is never written
                r_, w_, t_ = list(runs[:nruns]), list(waits[:nwaits]), [x for i, x in enumerate(tags[:ntags]) if i != at]
            runs, waits, tags = ((type(a[0]) * max(1, len(lst)))(*lst) for a, lst in ((runs, r_), (waits, w_),
                                                                                         (tags, t_)))
            nruns, nwaits, ntags = len(r_), len(w_), len(t_)
        _check(self.lib.fedagg_push_execute(ctypes.byref(runs) if nruns else None, nruns,
                                            ctypes.byref(waits) if nwaits else None, nwaits,
                                            ctypes.byref(tags) if ntags else None, ntags,
                                            nsteps, self._dev, self.rank, self.world, self.base, self._timeout,
                                            ws_src, ws_dst, ws_bytes,
                                            _native.FEDAGG_F64 if ws_kind == "f64" else _native.FEDAGG_F32, stage,
                                            ctypes.byref(prog.copies) if ncopies else None, ncopies,
                                            self._aux_ptrs if naux else None, naux, int(stream)), "fedagg_push_execute")
        self.base += prog.nsteps + 1
        if self.fault is not None and self.fault[1] == self.rank and self.fault[0] == "exit":  # TEST ONLY
            import torch

            torch.cuda.synchronize(self.device)  # its steps before `at` are done; then it dies
            os._exit(FAULT_EXIT_CODE)

    def settle(self) -> None:
        """Host-side end of a call (this rank's stream already synchronised): wait until every
        rank's progress counter shows the call finished (the counters' final value is the next
        call's base) or some rank's wait gave up -- so a rank whose own part succeeded learns
        whether the GROUP's call did before it meets its peers again (a peer that died never
        would).  Bounded by the wait kernels' timeout: past it plus a margin the transport is
        marked failed."""
        import time

        if self._page is None or self.world == 1:
            return
        deadline = time.monotonic() + self._timeout_s + 5.0
        while not self.errors():
            if all(int(v) >= self.base for v in self._page[: self.world]):
                return
            if time.monotonic() > deadline:
                self._settle_failed = True
                return
            time.sleep(0.0005)

    def failed(self) -> bool:
        """Whether a wait of some rank gave up (:meth:`errors`): the group cannot meet again -- a
        peer may have died, and a surviving one may still be finishing its steps into this rank's
        buffers.  A failed transport runs no collective and frees no program buffer any more."""
        return self._page is not None and (bool(self.errors()) or self._settle_failed)

    def _abandon_programs(self) -> None:
        """Keep the programs' buffers alive for the life of the process (a surviving peer may still
        push into them after its waits gave up) and drop this transport's references to them."""
        _ABANDONED.extend(self._programs)
        self._programs = []

    def close(self) -> None:
        if getattr(self, "_dev", None) is None:
            return
        import torch

        torch.cuda.synchronize(self.device)
        if self.failed():  # no barrier a dead peer would never meet
            self._abandon_programs()
        else:
            self.dist.barrier(group=self.group)  # nobody writes into a mapping that is going away
        self._programs.clear()
        for base in self._maps.values():
            self.lib.fedagg_ipc_close(base)
        self._maps.clear()
        self.lib.fedagg_host_unmap(self._page.ctypes.data)
        self._dev = None
        self._page = None
        self._shm.close()
        if self.rank == 0:
            self._shm.unlink()


FAULT_EXIT_CODE = 17  # TEST ONLY: the exit status of a rank the ("exit", rank, t) fault kills
_ABANDONED: List["PushProgram"] = []  # programs of failed transports: never freed while the process lives

PUSH_TAG_ERR, PUSH_PEER_ERR = 1 << 32, 1 << 33  # csrc/lockstep.hip: the err word's cause bits


def _describe_wait_error(v: int) -> str:
    """A rank's err word (csrc/lockstep.hip ``push_wait_kernel``) in words."""
    who = (v & 0xFFFFFFFF) - 1
    if v & PUSH_PEER_ERR:
        return f"stopped after rank {who}'s wait failed"
    if v & PUSH_TAG_ERR:
        return f"landing tag of rank {who}"
    return f"counter of rank {who}"


def _native_ipc_bytes() -> int:
    return 64  # FEDAGG_IPC_HANDLE_BYTES


def _hw_queues() -> int:
    try:
        return max(1, int(os.environ.get("GPU_MAX_HW_QUEUES", GPU_MAX_HW_QUEUES)))
    except ValueError:
        return GPU_MAX_HW_QUEUES


class _Uncached:
    """Device memory no L2 caches (fedagg_device_alloc_uncached), freed with its owner."""

    def __init__(self, lib, nbytes: int):
        self.lib, self.bytes = lib, int(nbytes)
        p = ctypes.c_void_p()
        _check(lib.fedagg_device_alloc_uncached(self.bytes, ctypes.byref(p)), "fedagg_device_alloc_uncached")
        self.ptr = int(p.value)

    def __del__(self):
        try:
            self.lib.fedagg_device_free(self.ptr)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


class PushProgram:
    """One rank's schedule compiled for the push executor: its runs split by consumer with
    every output address resolved (a mapped peer slot, the root's output, or its own output),
    and the waits of every step.  Built collectively (every rank at once).  FedAvg: one fp32
    accumulator per element; Scaffold: two fp64 accumulators (``which`` 0: the delta sum into
    ``outs[0]``, 1: the control-variate sum into ``outs[1]``), each run two launches."""

    def __init__(self, tr: PushTransport, plan: lockstep.RankPlan, blocks, accs, outs, kind: str, scaffold: bool,
                 c=None, lr: float = 1.0):
        import torch

        if (kind not in ("f32", "f64")) if scaffold else (kind not in ("f32", "bf16")):
            raise ValueError("push executor: FedAvg over fp32 / bf16 buckets (fp32 accumulators) or Scaffold over "
                             "fp32 / fp64 buckets; the other kinds take the RCCL executor")
        for sh in blocks.values():
            rows = (sh.delta, sh.cv) if scaffold else (getattr(sh, "rows", None),)
            if not all(isinstance(r, torch.Tensor) for r in rows):
                raise ValueError("push executor: row-layout client blocks only")
        self.plan, self.blocks, self.accs, self.outs, self.kind = plan, blocks, accs, outs, kind
        self.scaffold, self.c, self.lr = scaffold, c, float(lr)
        self._keep: list = []
        self._handles: set = set()  # the peers' IPC handles this program mapped (closed with it)
        G, me, root = plan.world, plan.rank, plan.root
        nacc = 2 if scaffold else 1
        outs = list(outs[:nacc])
        out_n = int(outs[0].numel())
        esz = outs[0].element_size()
        if any(o.numel() != out_n or o.element_size() != esz for o in outs):
            raise ValueError("push executor: the Scaffold outputs must have the same size and dtype")
        # What peers write lands in memory no L2 caches (a consumer's L2 could still hold the lines
        # a slot had four steps earlier): the slots, and a landing copy of the output's index space
        # (the last block's input on every rank, the finished pieces on the root), one per
        # accumulator.  The caller's slots are not used; the root copies the landed finished pieces
        # into its outputs.
        se = max(1, plan.slot_elems)
        self.slots_u = _Uncached(tr.lib, nacc * lockstep.SLOTS * se * esz)
        self.land_u = _Uncached(tr.lib, nacc * out_n * esz)
        # landing tags: word q * n_steps + t = the generation of the call whose step-t pushes of
        # rank q into this rank landed (written by q after its data, over the same link)
        self.tags_u = _Uncached(tr.lib, max(1, G * plan.n_steps) * 8)
        self.stage_u = None  # the root's numel == 1 product staging, at first use
        mine = {"slots": tr.ipc_info(self.slots_u.ptr) if G > 1 else None,
                "land": tr.ipc_info(self.land_u.ptr) if G > 1 else None,
                "tags": tr.ipc_info(self.tags_u.ptr) if G > 1 else None,
                "out_n": out_n, "se": se,
                "recv": [(g, o.peer, o.key, o.buf, o.n) for g, ops in enumerate(plan.groups) for o in ops
                         if o.kind == "recv"]}
        infos = tr.all_gather(mine) if G > 1 else [mine]

        def offset(rank: int, loc, which: int) -> int:
            """Byte offset of ``loc`` in ``rank``'s landing buffer ("out") or slots."""
            where, slot, off = loc
            if where == "out":
                return (which * infos[rank]["out_n"] + off) * esz
            return ((which * lockstep.SLOTS + slot) * infos[rank]["se"] + off) * esz

        def local(loc, which: int) -> int:
            return (self.land_u.ptr if loc[0] == "out" else self.slots_u.ptr) + offset(me, loc, which)

        def at(rank: int, loc, which: int) -> int:
            if rank == me:
                # the root's own finished pieces: straight into the caller's outputs
                return outs[which].data_ptr() + loc[2] * esz if loc[0] == "out" and rank == root else local(loc, which)
            return tr.remote(infos[rank]["land" if loc[0] == "out" else "slots"], self) + offset(rank, loc, which)

        specs, wait_list = push_schedule(plan, [info["recv"] for info in infos])
        # the output ranges other ranks finish (landed on the root, copied into its outputs)
        own = sorted((p.dst[2], p.dst[2] + p.n) for p in specs if p.dst_rank == me and p.dst[0] == "out")
        ranges, a = [], 0
        for lo, hi in own + [(out_n, out_n)]:
            if lo > a:
                ranges.append((a, lo))
            a = max(a, hi)
        copies = [_Copy(outs[w].data_ptr() + lo * esz, self.land_u.ptr + (w * out_n + lo) * esz, (hi - lo) * esz)
                  for lo, hi in ranges for w in range(nacc)]
        self.land_ranges = ranges
        self.ncopies = len(copies)
        self.copies = (_Copy * max(1, len(copies)))(*copies)
        runs = [rec for p in specs for rec in self._runs(p, [at(p.dst_rank, p.dst, w) for w in range(nacc)],
                                                          [local(p.src, w) if p.src is not None else 0
                                                           for w in range(nacc)])]
        n_steps = plan.n_steps
        outgoing = push_outgoing(plan, specs)
        everyone = tr.all_gather(outgoing) if G > 1 else [outgoing]
        tag_waits = push_tag_waits(me, n_steps, everyone)
        # counter waits first within a step, then the tag waits (each after its own producer's counter)
        waits = sorted([(t, 0, q, v, None) for t, q, v in wait_list] +
                       [(t, 1, q, v, self.tags_u.ptr + idx * 8) for t, q, v, idx in tag_waits],
                       key=lambda x: (x[0], x[1]))
        waits = [_Wait(t, q, v, tag) for t, _k, q, v, tag in waits]
        tags = [_Tag(t, 0, tr.remote(infos[c]["tags"], self) + (me * n_steps + t) * 8) for t, c, _e in outgoing]
        self.outgoing, self.tag_waits = outgoing, tag_waits
        self.nruns, self.nwaits, self.ntags, self.nsteps = len(runs), len(waits), len(tags), n_steps
        self.runs = (_Run * max(1, len(runs)))(*runs)
        self.waits = (_Wait * max(1, len(waits)))(*waits)
        self.tags = (_Tag * max(1, len(tags)))(*tags)
        self._tr = tr
        self._stage_info = None
        self._out_ptrs, self._out_bytes = [o.data_ptr() for o in outs], out_n * esz

    def ws_dst(self, ws_bytes: int) -> int:
        """This rank's staging row on the root for the numel == 1 products (collective at first use)."""
        tr, G = self._tr, self.plan.world
        if self._stage_info is None or self._stage_info[1] != ws_bytes:
            if self.plan.rank == self.plan.root:
                self.stage_u = _Uncached(tr.lib, G * ws_bytes)
                info = tr.ipc_info(self.stage_u.ptr)
            else:
                info = None
            infos = tr.all_gather(info)
            self._stage_info = (infos[self.plan.root], ws_bytes)
        if self.plan.rank == self.plan.root:
            return self.stage_u.ptr + self.plan.rank * ws_bytes
        return tr.remote(self._stage_info[0], self) + self.plan.rank * ws_bytes

    def _runs(self, p: "PushRun", dst: List[int], src: List[int]) -> List[_Run]:
        """The launches of one push run: the block's clients (rows at column ``p.col``, ``p.n``
        elements) continuing the accumulator at ``src`` (0: from +0.0) into ``dst`` -- FedAvg one
        launch (``FEDAGG_RUN_FEDAVG_PUSH``), Scaffold two (``FEDAGG_RUN_SCAFFOLD_PUSH_DELTA`` then
        ``_CV``; a finished piece applies lr / adds c).  Every launch is a push run (input
        accumulator separate from the output, system-scope write-through stores) -- also the
        root's own final runs into its outputs, which keeps one arithmetic path for every piece."""
        sh = self.blocks[p.block]
        if not self.scaffold:
            kind = _native.FEDAGG_BF16 if self.kind == "bf16" else _native.FEDAGG_F32
            return [self._run(p, _native.FEDAGG_RUN_FEDAVG_PUSH, kind, sh.rows, np.asarray(sh.w, np.float32),
                              ctypes.c_float, dst[0], src[0])]
        kind = _native.FEDAGG_F32 if self.kind == "f32" else _native.FEDAGG_F64
        w = np.asarray(sh.w, np.float64)
        recs = [self._run(p, _native.FEDAGG_RUN_SCAFFOLD_PUSH_DELTA, kind, sh.delta, w, ctypes.c_double, dst[0], src[0]),
                self._run(p, _native.FEDAGG_RUN_SCAFFOLD_PUSH_CV, kind, sh.cv, w, ctypes.c_double, dst[1], src[1])]
        for rec in recs:
            rec.finish, rec.lr = int(p.final), self.lr
            if p.final:  # c of the piece's global elements (scaffold.py:262-263)
                rec.c = self.c.data_ptr() + p.dst[2] * self.c.element_size()
        return recs

    def _run(self, p: "PushRun", op: int, kind: int, rows, w: np.ndarray, wtype, dst: int, src: int) -> _Run:
        rec = _Run()
        rec.step, rec.op, rec.kind, rec.seed, rec.finish, rec.n = p.step, op, kind, 0 if src else 1, 0, p.n
        base, step, esz = rows.data_ptr(), rows.stride(0) * rows.element_size(), rows.element_size()
        arr = _native.ptr_array([base + k * step + p.col * esz for k in range(rows.shape[0])])
        warr = (wtype * len(w))(*[float(v) for v in w])
        self._keep += [arr, warr]
        rec.K = rows.shape[0]
        rec.x, rec.w, rec.acc, rec.acc2 = ctypes.addressof(arr), ctypes.addressof(warr), dst, src or None
        return rec

    def matches(self, plan, blocks, accs, outs, kind, scaffold, c=None, lr=1.0) -> bool:
        """Whether a call can run this program.  Only what is the same on every rank by construction
        (the caller's plan / blocks / c objects, kind, lr, the outputs' size) decides: the compile
        of a miss is collective, so a decision that could differ between ranks -- the outputs'
        addresses, fresh tensors that one rank's allocator happens to place where the last ones
        were -- would leave one rank compiling while the others execute.  New output addresses are
        patched in instead (:meth:`rebase_outs`)."""
        nacc = 2 if self.scaffold else 1
        return (plan is self.plan and blocks is self.blocks and kind == self.kind and scaffold == self.scaffold
                and c is self.c and float(lr) == self.lr and len(outs) >= nacc
                and all(int(o.numel()) * o.element_size() == self._out_bytes
                        and o.element_size() == self.outs[0].element_size() for o in outs[:nacc]))

    def rebase_outs(self, outs) -> None:
        """Point the launches and landing copies that write the caller's outputs (the root's
        finished pieces) at ``outs``; a no-op when the addresses did not move."""
        nacc = 2 if self.scaffold else 1
        new = [o.data_ptr() for o in outs[:nacc]]
        if new == self._out_ptrs:
            return
        span = self._out_bytes

        def moved(addr):
            if addr:
                for old, nw in zip(self._out_ptrs, new):
                    if old <= addr < old + span:
                        return addr - old + nw
            return None

        for r in self.runs[: self.nruns]:
            a = moved(r.acc)
            if a is not None:
                r.acc = a
        for cp in self.copies[: self.ncopies]:
            a = moved(cp.dst)
            if a is not None:
                cp.dst = a
        self._out_ptrs, self.outs = new, list(outs)


@dataclass(frozen=True)
class PushRun:
    """One launch of the push executor: ``n`` elements at column ``col`` of ``block``'s buffer;
    input accumulator at ``src`` on this rank (None: seeded with +0.0), output at ``dst`` on
    ``dst_rank`` (locations as :class:`lockstep.Run.acc`)."""

    step: int
    block: int
    col: int
    n: int
    src: Optional[Tuple[str, int, int]]
    dst_rank: int
    dst: Tuple[str, int, int]
    final: bool = False  # a finished piece (read by the root after the last step, not at step + 2)


def push_schedule(plan: lockstep.RankPlan, recvs: Sequence[Sequence[tuple]]):
    """This rank's push runs and waits (pure: a function of the plan and every rank's receive
    ops ``(group, sender, key, buf, n)``).  A run's output goes where the lockstep schedule would
    have received it (the matching receive of group t + 1 on the consumer; a finished piece: the
    root's output at its global offset), split per consumer.  Waits ``(step, rank, value)``:
    before step t, counter(rank) >= base + value, ``value = max(t, 1)`` for the producers of the
    step's inputs and the consumers of its outputs (finished step t - 2, or entered the call),
    the root at step 0 and wherever a finished piece goes to it; at ``n_steps`` the root waits
    for every rank's last step (``n_steps + 1``)."""
    G, me, root = plan.world, plan.rank, plan.root
    recv_of = {}  # (group, sender, receiver, key) -> the receiver's buffer location
    for r, ops in enumerate(recvs):
        for g, q, key, buf, n in ops:
            recv_of[(g, q, r, key)] = (buf, n)
    specs: List[PushRun] = []
    waits: List[Tuple[int, int, int]] = []
    for t, step_runs in enumerate(plan.runs):
        producers, consumers = set(), set()
        inputs = [r for r in step_runs if not r.seed]  # they arrived in group t - 1
        for o in (plan.groups[t - 1] if t >= 1 else []):
            if o.kind == "recv" and any(_overlap(o.buf, o.n, r.acc, r.n) for r in inputs):
                producers.add(o.peer)
        sends = [o for o in plan.groups[t + 1] if o.kind == "send"] if t + 1 < len(plan.groups) else []
        for r in step_runs:
            src = None if r.seed else r.acc
            if r.final:  # a finished piece: straight into the root's output
                specs.append(PushRun(t, r.block, r.col, r.n, src, root, ("out", 0, r.lo), final=True))
                if me != root:
                    consumers.add(root)
                continue
            covered = 0
            for o in sends:
                a0, n0 = _intersect(o.buf, o.n, r.acc, r.n)
                if not n0:
                    continue
                dloc, _dn = recv_of[(t + 1, me, o.peer, o.key)]
                j = a0 - r.acc[2]
                specs.append(PushRun(t, r.block, r.col + j, n0, None if src is None else (src[0], src[1], src[2] + j),
                                     o.peer, (dloc[0], dloc[1], dloc[2] + (a0 - o.buf[2]))))
                consumers.add(o.peer)
                covered += n0
            if covered != r.n:
                raise AssertionError(f"push: step {t} run of {r.n} elements has {covered} consumed")
        if t == 0 and me != root:
            consumers.add(root)  # the root entered the call: its output and staging row are free
        for q in sorted(producers | consumers):
            if q != me:
                waits.append((t, q, max(t, 1)))
    if me == root:
        waits += [(plan.n_steps, q, plan.n_steps + 1) for q in range(G) if q != me]
    return specs, waits


def push_outgoing(plan: lockstep.RankPlan, specs: Sequence[PushRun]) -> List[Tuple[int, int, bool]]:
    """``(step, consumer, at_end)`` of every landing tag this rank writes: one per consumer its
    step pushed to, and at step 0 always one to the root (its numel == 1 staging row is copied
    there after step 0's waits).  ``at_end``: the consumer reads those pushes only after its last
    step (finished pieces and the staging row on the root), not at step + 2.  Sorted by step."""
    ends: Dict[Tuple[int, int], bool] = {}
    for s in specs:
        if s.dst_rank != plan.rank:
            key = (s.step, s.dst_rank)
            ends[key] = ends.get(key, True) and s.final
    if plan.rank != plan.root and plan.n_steps > 0:
        ends.setdefault((0, plan.root), True)
    return sorted((t, c, e) for (t, c), e in ends.items())


def push_tag_waits(me: int, n_steps: int, outgoing: Sequence[Sequence[Tuple[int, int, bool]]]
                   ) -> List[Tuple[int, int, int, int]]:
    """This rank's landing-tag waits from every rank's :func:`push_outgoing`: ``(wait step,
    producer q, counter value, tag index)``.  A push of q at step t is an input of this rank's step
    t + 2 (computed at t, consumed at t + 2), or is read after the last step (``at_end``); its tag is
    waited for before that step, after q's counter says step t is done (value t + 2) -- a wait on a
    strictly earlier step of another rank, like every other wait of the schedule."""
    res = []
    for q, lst in enumerate(outgoing):
        if q == me:
            continue
        for t, c, at_end in lst:
            if c == me:
                res.append((n_steps if at_end else min(t + 2, n_steps), q, t + 2, q * n_steps + t))
    return sorted(res)


def _intersect(loc_a, n_a: int, loc_b, n_b: int) -> Tuple[int, int]:
    """(start, length) of the intersection of two buffer ranges (same buffer and slot), else (0, 0)."""
    if loc_a[0] != loc_b[0] or loc_a[1] != loc_b[1]:
        return 0, 0
    lo = max(loc_a[2], loc_b[2])
    hi = min(loc_a[2] + n_a, loc_b[2] + n_b)
    return (lo, hi - lo) if hi > lo else (0, 0)


def _overlap(loc_a, n_a: int, loc_b, n_b: int) -> bool:
    return _intersect(loc_a, n_a, loc_b, n_b)[1] > 0
