"""Native RCCL communicator and lockstep executor (``fedagg_comm_*``, ``fedagg_lockstep_execute``;
csrc/lockstep.hip): the client-sharded relay / striped schedules of :mod:`lockstep` issued from C++
instead of Python, one RCCL group and a handful of kernel launches per step.

:class:`RcclTransport` is a drop-in ``transport`` for :func:`sharding.lockstep_fedavg` /
:func:`sharding.lockstep_scaffold`: the schedule is compiled once into a :class:`NativeProgram`
(flat run / message tables with every device pointer resolved) and each call is ONE ctypes call.
The communicator is set up through a ``torch.distributed`` group (rank 0's RCCL unique id is
broadcast over it); RCCL itself is the instance already in the process when torch has loaded
one, else ROCm's ``librccl.so.1``.
"""

from __future__ import annotations

import ctypes
import os
import sys
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np

from . import _native, lockstep


class _Run(ctypes.Structure):
    _fields_ = [("step", ctypes.c_int32), ("op", ctypes.c_int32), ("kind", ctypes.c_int32), ("K", ctypes.c_int32),
                ("seed", ctypes.c_int32), ("finish", ctypes.c_int32), ("n", ctypes.c_uint64),
                ("tile_vectors", ctypes.c_uint64), ("x", ctypes.c_void_p), ("x2", ctypes.c_void_p),
                ("w", ctypes.c_void_p), ("c", ctypes.c_void_p), ("lr", ctypes.c_double), ("acc", ctypes.c_void_p),
                ("acc2", ctypes.c_void_p)]


class _Msg(ctypes.Structure):
    _fields_ = [("group", ctypes.c_int32), ("send", ctypes.c_int32), ("peer", ctypes.c_int32),
                ("kind", ctypes.c_int32), ("buf", ctypes.c_void_p), ("count", ctypes.c_uint64)]


assert ctypes.sizeof(_Run) == 96 and ctypes.sizeof(_Msg) == 32  # include/fedagg.h layouts

_KIND = {"f32": _native.FEDAGG_F32, "bf16": _native.FEDAGG_BF16, "f64": _native.FEDAGG_F64, "f16": _native.FEDAGG_F16}
_ACC_KIND = {"f32": _native.FEDAGG_F32, "bf16": _native.FEDAGG_F32, "f64": _native.FEDAGG_F64,
             "f16": _native.FEDAGG_F16}


def rccl_path() -> str:
    """The RCCL to dlopen: torch's bundled one when torch is in the process (one RCCL instance per
    process), else ROCm's."""
    if "torch" in sys.modules:
        p = Path(sys.modules["torch"].__file__).parent / "lib" / "librccl.so"
        if p.exists():
            return str(p)
    for p in ("/opt/rocm/lib/librccl.so.1", "librccl.so.1"):
        if p.startswith("/") and not os.path.exists(p):
            continue
        return p
    return "librccl.so.1"


def _check(rc: int, what: str) -> None:
    if rc != 0:
        lib = _native.load()
        msg = lib.fedagg_comm_last_error().decode(errors="replace") or lib.fedagg_last_error().decode(errors="replace")
        raise _native.NativeLibraryError(f"{what} failed ({rc}): {msg}")


class RcclTransport:
    """A native RCCL communicator over the ranks of ``group`` (a torch.distributed group, used only
    for the unique-id broadcast and host-side bookkeeping).  ``rank`` / ``world`` as the group's."""

    native = True

    def __init__(self, group=None, device: Optional[int] = None):
        import torch
        import torch.distributed as dist

        self.lib = _native.load()
        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.device = torch.cuda.current_device() if device is None else int(device)
        path = rccl_path().encode()
        uid = (ctypes.c_char * 128)()
        if self.rank == 0:
            _check(self.lib.fedagg_comm_unique_id(path, uid), "fedagg_comm_unique_id")
        obj = [bytes(uid.raw)]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(obj, src=src, group=group)
        uid = (ctypes.c_char * 128).from_buffer_copy(obj[0])
        h = ctypes.c_void_p()
        _check(self.lib.fedagg_comm_create(path, self.world, self.rank, uid, self.device, ctypes.byref(h)),
               "fedagg_comm_create")
        self._h = h
        self._programs: List["NativeProgram"] = []
        self._py = None
        RcclTransport._live += 1  # push.aux_stream_budget counts the live communicators

    _live = 0  # communicators of this process not yet closed

    @classmethod
    def live(cls) -> int:
        return cls._live

    def comm_count(self) -> int:
        """ncclCommCount: the ranks RCCL counts in this communicator."""
        n = ctypes.c_int()
        _check(self.lib.fedagg_comm_count(self._h, ctypes.byref(n)), "fedagg_comm_count")
        return int(n.value)

    def python_transport(self):
        """The torch.distributed transport of the same group (sharding.DistTransport), for the paths
        the native executor does not run: schedules with an empty client block (fewer clients than
        ranks, or a ragged split) and the re-associating combines.  It moves device tensors, so
        the group's backend must carry them (RCCL)."""
        if self._py is None:
            from .sharding import DistTransport

            self._py = DistTransport(self.group)
        return self._py

    def close(self) -> None:
        if self._h:
            h, self._h = self._h, None
            RcclTransport._live -= 1
            _check(self.lib.fedagg_comm_destroy(h), "fedagg_comm_destroy")

    def abort(self) -> None:
        if self._h:
            self.lib.fedagg_comm_abort(self._h)

    def async_error(self) -> None:
        _check(self.lib.fedagg_comm_async_error(self._h), "RCCL")

    def program(self, **kw) -> "NativeProgram":
        """The compiled program of a schedule over these very tensors (cached: the same plan,
        blocks and buffers give the same program)."""
        for p in self._programs:
            if p.matches(**kw):
                return p
        p = NativeProgram(**kw)
        self._programs = ([p] + self._programs)[:4]
        return p

    def execute(self, prog: "NativeProgram", stream: int, ws=None, ws_kind: str = "f32") -> None:
        wsp = ws.data_ptr() if ws is not None else None
        wsn = int(ws.numel()) if wsp else 0
        _check(self.lib.fedagg_lockstep_execute(self._h, ctypes.byref(prog.runs) if prog.nruns else None, prog.nruns,
                                                ctypes.byref(prog.msgs) if prog.nmsgs else None, prog.nmsgs,
                                                prog.ngroups, wsp, wsn, _ACC_KIND[ws_kind], prog.plan.root,
                                                int(stream)), "fedagg_lockstep_execute")

    # the host-side pieces the lockstep combines need besides the schedule (over the torch group)
    def all_sum_int(self, v: int) -> int:
        import torch

        t = torch.tensor([int(v)], dtype=torch.int64)
        self.dist.all_reduce(t, group=self.group)
        return int(t.item())

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


class NativeProgram:
    """One rank's schedule compiled into the tables of ``fedagg_lockstep_execute``: every run's
    client pointers, weights and accumulator, every message's buffer, resolved once.  Holds
    references to everything it points into."""

    def __init__(self, plan: lockstep.RankPlan, blocks: Dict[int, object], accs: List, outs: List, kind: str,
                 scaffold: bool, c=None, lr: float = 1.0):
        self.plan, self.blocks, self.accs, self.outs, self.kind, self.scaffold, self.c, self.lr = (
            plan, blocks, accs, outs, kind, scaffold, c, float(lr))
        self._keep = []
        runs, msgs = [], []
        esz = outs[0].element_size()

        def loc(where, slot, off, n, which):
            base = outs[which] if where == "out" else accs[which][slot]
            return base.data_ptr() + off * esz if where == "out" else base.data_ptr() + off * base.element_size()

        for t, step_runs in enumerate(plan.runs):
            for r in step_runs:
                sh = blocks[r.block]
                rec = _Run()
                rec.step, rec.K, rec.seed, rec.finish, rec.n = t, int(sh.Kr), int(r.seed), int(r.final), int(r.n)
                if rec.K <= 0:
                    raise ValueError("native lockstep: empty client blocks take the Python executor")
                rec.kind = _KIND[kind] if not scaffold else (_native.FEDAGG_F32 if kind == "f32" else _native.FEDAGG_F64)
                if scaffold:
                    rec.op = _native.FEDAGG_RUN_SCAFFOLD
                    rec.x = self._ptrs(sh.delta, r.col)
                    rec.x2 = self._ptrs(sh.cv, r.col)
                    rec.w = self._weights("f64", sh.w)
                    if r.final:
                        rec.c = c.data_ptr() + r.lo * c.element_size()
                    rec.lr = float(lr)
                    rec.acc = loc(*r.acc, r.n, 0)
                    rec.acc2 = loc(*r.acc, r.n, 1)
                else:
                    view = sh.rows[:, r.col: r.col + r.n]
                    from .sharding import TiledView

                    if isinstance(view, TiledView):
                        rec.op = _native.FEDAGG_RUN_FEDAVG_TILED
                        rec.x = self._keep_arr(_native.ptr_array([view.base.data_ptr()]))
                        rec.tile_vectors = int(view.tv)
                    else:
                        rec.op = _native.FEDAGG_RUN_FEDAVG
                        rec.x = self._ptrs(sh.rows, r.col)
                    rec.w = self._weights(kind, sh.w)
                    rec.acc = loc(*r.acc, r.n, 0)
                runs.append(rec)
        acc_kind = _ACC_KIND[kind] if not scaffold else _native.FEDAGG_F64
        for g, ops in enumerate(plan.groups):
            for o in ops:
                for which in range(2 if scaffold else 1):
                    m = _Msg()
                    m.group, m.send, m.peer, m.kind = g, int(o.kind == "send"), int(o.peer), acc_kind
                    m.buf, m.count = loc(*o.buf, o.n, which), int(o.n)
                    msgs.append(m)
        self.nruns, self.nmsgs, self.ngroups = len(runs), len(msgs), plan.n_steps + 1
        self.runs = (_Run * max(1, len(runs)))(*runs)
        self.msgs = (_Msg * max(1, len(msgs)))(*msgs)

    def _keep_arr(self, arr) -> int:
        self._keep.append(arr)
        return ctypes.addressof(arr)

    def _ptrs(self, rows, col: int) -> int:
        base, step, esz = rows.data_ptr(), rows.stride(0) * rows.element_size(), rows.element_size()
        return self._keep_arr(_native.ptr_array([base + k * step + col * esz for k in range(rows.shape[0])]))

    def _weights(self, kind: str, w) -> int:
        if kind in ("f32", "bf16"):
            arr = (ctypes.c_float * len(w))(*[float(v) for v in np.asarray(w, np.float32)])
        elif kind == "f64":
            arr = (ctypes.c_double * len(w))(*[float(v) for v in np.asarray(w, np.float64)])
        else:
            bits = np.asarray(w, np.float16).view(np.uint16)
            arr = (ctypes.c_uint16 * len(w))(*[int(v) for v in bits])
        return self._keep_arr(arr)

    def matches(self, plan, blocks, accs, outs, kind, scaffold, c=None, lr=1.0) -> bool:
        """The same schedule over the same buffers (the program holds the tensors it points into,
        so equal addresses are the same live buffers)."""
        return (plan is self.plan and blocks is self.blocks and kind == self.kind and scaffold == self.scaffold
                and c is self.c and float(lr) == self.lr
                and [a.data_ptr() for a in accs] == [a.data_ptr() for a in self.accs]
                and [o.data_ptr() for o in outs] == [o.data_ptr() for o in self.outs])
