"""Multi-GPU aggregation, one process per GPU over ``torch.distributed`` (RCCL on ROCm).

Two layouts:

* **Parameter-range sharding (primary, bit-exact).**  The reduction is independent per element,
  so rank ``r`` owns elements ``[lo_r, hi_r)`` of every client's flat bucket, stages only that
  slice over its own PCIe link, and reduces it with the same kernel and the same client order as
  one GPU.  No arithmetic crosses GPUs; results are bit-identical to the single-GPU path and to
  the reference.  The optional final gather to every rank is a plain all-gather of the result
  slices (RCCL over xGMI), not a reduction.
* **Client sharding (the north-star mode).**  The K clients are cut into G contiguous blocks,
  block ``b``'s buckets live in the HBM of rank ``chain_rank(b)`` (the last block on the root,
  rank 0), and the reference's sequential client sum (fed_avg.py:221-222; scaffold.py:262-263,
  293) is completed across the ranks in one of three ways, all device-resident (partial sums
  stay in HBM, the exchange is RCCL over xGMI, the final step runs on the root's GPU):

  ``combine="relay"`` (default, **bit-exact**): block b CONTINUES the accumulator of blocks
  0..b-1, received chunk by chunk from the previous rank (P2P send/recv), so every element sees
  exactly the reference's rounding sequence; the chunks are pipelined, so all G ranks stream
  at once.  The root holds the last block and applies the final step (Scaffold: + c, then
  ``aggregation_lr``) inside its last kernel.
  ``combine="rccl"``: every block sums from +0.0, the partials are summed by ``dist.reduce``
  (RCCL's order) and the root applies the final scale.  Re-associates the client sum: a few ulp
  off the reference (DESIGN.md §6 drift table).
  ``combine="ordered"``: the partials are gathered on the root and added in block order by the
  bucket kernel (weight 1.0 per partial; Scaffold: lr and + c in the same launch).
  Deterministic, same drift class as ``rccl``.
  ``striped`` (:func:`client_shard_fedavg_striped`, **bit-exact**): the relay, but the bucket is
  cut into S parameter stripes and stripe s places block b on rank ``a_s * (b + 1) mod G`` for a
  different unit ``a_s`` of Z_G per stripe.  Every element still passes through blocks 0..G-1
  in order (the same rounding sequence), every stripe still ends on the root, but stripe s's
  hops all go ``a_s`` ranks ahead: on a fully connected xGMI node the S stripes' accumulators
  travel over S disjoint sets of G links at once instead of all over the same G - 1.

  The numel == 1 tensors follow NumPy's pairwise order over ALL K products,
  which no block can compute alone: every rank writes its products into its columns of a
  ``[P, K]`` workspace (zeros elsewhere), the workspaces are summed onto the root (exact: x + 0)
  and the root runs the pairwise tree -- so these elements are bit-exact in every mode.

The per-rank arithmetic and the transport are injectable: :class:`GpuShardOps` (libfedagg on this
rank's GPU) and :class:`DistTransport` (``torch.distributed``) are the product; the CPU ``gloo``
tests inject NumPy ops (test infrastructure), and :class:`LoopbackGroup` runs G ranks as threads
of one process on one GPU (the drift tool and the GPU tests of the multi-rank protocol).
"""

from __future__ import annotations

import ctypes
import threading
from collections import deque
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .layout import BucketLayout

SHARD_ALIGN = 512  # elements (2 KiB of fp32): every shard starts on a 256-B boundary
RELAY_CHUNK_ELEMS = 2 << 20  # pipelined relay: >= 2M elements (8 MB fp32) per P2P message
COMBINES = ("relay", "rccl", "ordered")  # client_shard_fedavg / _scaffold; "striped": *_striped below


def shard_bounds(M: int, world: int, align: int = SHARD_ALIGN) -> List[Tuple[int, int]]:
    """Equal, ``align``-multiple chunk per rank; the last rank may get less (or nothing)."""
    chunk = -(-M // world)
    chunk = -(-chunk // align) * align
    return [(min(M, r * chunk), min(M, (r + 1) * chunk)) for r in range(world)]


def pack_range(layout: BucketLayout, layers: Sequence[np.ndarray], dst: np.ndarray, lo: int, hi: int) -> None:
    """Copy elements ``[lo, hi)`` of one client's flat row into ``dst[0 : hi - lo]``."""
    for s in layout.segments:
        a, b = max(lo, s.offset), min(hi, s.offset + s.numel)
        if a >= b:
            continue
        src = np.asarray(layers[s.layer]).reshape(-1)
        np.copyto(dst[a - lo : b - lo], src[a - s.offset : b - s.offset], casting="unsafe")


# ======================================================================================
# client blocks
# ======================================================================================
def client_blocks(K: int, world: int) -> List[Tuple[int, int]]:
    """Block b = clients ``[k0, k1)`` (contiguous, list order); trailing blocks may be empty."""
    per = -(-K // world)
    return [(min(K, b * per), min(K, (b + 1) * per)) for b in range(world)]


def chain_rank(block: int, world: int) -> int:
    """Rank holding client block ``block``: block b on rank (b + 1) % G, so the LAST block (whose
    kernel finishes the chain) sits on the root, rank 0."""
    return (block + 1) % world


def block_of(rank: int, world: int) -> int:
    return (rank - 1) % world


def relay_chunks(M: int, chunk_elems: int = RELAY_CHUNK_ELEMS) -> List[Tuple[int, int]]:
    """Pipelining chunks of ``[0, M)`` (SHARD_ALIGN multiples; at least one)."""
    step = max(SHARD_ALIGN, -(-chunk_elems // SHARD_ALIGN) * SHARD_ALIGN)
    if M <= 0:
        return [(0, 0)]
    return [(a, min(M, a + step)) for a in range(0, M, step)]


# ======================================================================================
# per-rank problems
# ======================================================================================
@dataclass
class FedAvgShard:
    """This rank's part of a client-sharded FedAvg.

    ``rows``: ``[Kr, ld]`` tensor of this rank's client buckets (block order), ``w``: their
    GLOBAL weights ``fl(n_k / n)`` in the product type, ``kbase``: global index of the first
    client, ``K``: all clients, ``M``: bucket length, ``pairwise_idx``: numel == 1 indices."""

    kind: str
    rows: object
    w: np.ndarray
    kbase: int
    K: int
    M: int
    pairwise_idx: np.ndarray

    @property
    def Kr(self) -> int:
        return int(self.rows.shape[0]) if self.rows is not None else 0


@dataclass
class ScaffoldShard:
    """This rank's part of a client-sharded Scaffold (fp32 or fp64 buckets, fp64 sums).  ``c``
    (the server control variate, ``[ld]``) is read on the root only."""

    kind: str
    delta: object
    cv: object
    c: object
    w: np.ndarray
    kbase: int
    K: int
    M: int
    lr: float
    pairwise_idx: np.ndarray

    @property
    def Kr(self) -> int:
        return int(self.delta.shape[0]) if self.delta is not None else 0


def out_dtype(torch, kind: str):
    return {"f32": torch.float32, "bf16": torch.float32, "f64": torch.float64, "f16": torch.float16}[kind]


def ws_dtype(torch, kind: str):
    """Pairwise-sum type of the numel == 1 products (NumPy's HALF_pairwise_sum adds fp16 in fp32)."""
    return torch.float64 if kind == "f64" else torch.float32


# ======================================================================================
# per-rank arithmetic on the GPU (the product): libfedagg's kernels on torch's current stream
# ======================================================================================
def _stream():
    import torch

    return int(torch.cuda.current_stream().cuda_stream)


class GpuShardOps:
    """libfedagg entry points (``include/fedagg.h``, client-sharded building blocks) on this
    rank's GPU, enqueued on torch's current stream (so torch.distributed's RCCL calls order
    against them)."""

    def __init__(self):
        from . import _native

        self._n = _native
        self.lib = _native.load()

    # -- FedAvg --------------------------------------------------------------------------
    def _weights(self, kind: str, w):
        if kind in ("f32", "bf16"):
            return (ctypes.c_float * max(1, len(w)))(*[float(v) for v in np.asarray(w, np.float32)])
        if kind == "f64":
            return (ctypes.c_double * max(1, len(w)))(*[float(v) for v in np.asarray(w, np.float64)])
        bits = np.asarray(w, np.float16).view(np.uint16)
        return (ctypes.c_uint16 * max(1, len(w)))(*[int(v) for v in bits])

    @staticmethod
    def _rows(t, a: int = 0) -> list:
        base, step, esz = t.data_ptr(), t.stride(0) * t.element_size(), t.element_size()
        return [base + k * step + a * esz for k in range(t.shape[0])]

    def fedavg_chain(self, kind, rows, w, a: int, b: int, seed: bool, out) -> None:
        """out[a:b] = (seed ? +0 : out[a:b]) + the clients of ``rows`` in order."""
        if b <= a:
            return
        if rows.shape[0] == 0:  # an empty block passes the accumulator on (or starts it at +0)
            if seed:
                out[a:b].zero_()
            return
        fn = getattr(self.lib, f"fedagg_fedavg_chain_{kind}")
        rc = fn(self._n.ptr_array(self._rows(rows, a)), self._weights(kind, w), int(rows.shape[0]), b - a,
                int(bool(seed)), out.data_ptr() + a * out.element_size(), _stream())
        self._n.check(rc, "fedavg_chain")

    def fedavg_products(self, sh: FedAvgShard, ws) -> None:
        P = int(sh.pairwise_idx.size)
        if not P or not sh.Kr:
            return
        kind = sh.kind
        fn = getattr(self.lib, f"fedagg_pairwise_products_{kind}")
        idx = (ctypes.c_uint64 * P)(*[int(v) for v in sh.pairwise_idx])
        rc = fn(self._n.ptr_array(self._rows(sh.rows)), self._weights(kind, sh.w), sh.Kr, idx, P, sh.K, sh.kbase,
                ws.data_ptr(), _stream())
        self._n.check(rc, "pairwise_products")

    def fedavg_finish(self, kind, ws, K: int, pairwise_idx, out) -> None:
        P = int(pairwise_idx.size)
        if not P:
            return
        fn = getattr(self.lib, "fedagg_pairwise_finish_" + {"f32": "f32", "bf16": "f32", "f64": "f64",
                                                             "f16": "f16"}[kind])
        idx = (ctypes.c_uint64 * P)(*[int(v) for v in pairwise_idx])
        self._n.check(fn(ws.data_ptr(), K, K, idx, P, out.data_ptr(), _stream()), "pairwise_finish")

    def fedavg_combine(self, kind, parts, M: int, out) -> None:
        """out = +0 + parts[0] + parts[1] + ... (block order; x * 1.0 is exact), one launch."""
        pk = {"f32": "f32", "bf16": "f32", "f64": "f64", "f16": "f16"}[kind]
        self.fedavg_chain(pk, parts, np.ones(parts.shape[0]), 0, M, True, out)

    # -- Scaffold ------------------------------------------------------------------------
    def scaffold_chain(self, sh: ScaffoldShard, a: int, b: int, seed: bool, finish: bool, dout, cout) -> None:
        """dout/cout[a:b] = (seed ? +0 : themselves) + this block's clients, in order; ``finish``
        (last block): then ``+ c`` and ``* lr``."""
        if b <= a:
            return
        if sh.Kr == 0:  # an empty block: pass the accumulators on (start them at +0), finish them
            if seed:
                dout[a:b].zero_()
                cout[a:b].zero_()
            if finish:
                self._scaffold_final(sh, a, b, dout, cout)
            return
        fn = getattr(self.lib, f"fedagg_scaffold_chain_{sh.kind}")
        esz = sh.delta.element_size()
        c = sh.c.data_ptr() + a * esz if finish else None
        w = (ctypes.c_double * sh.Kr)(*[float(v) for v in sh.w])
        rc = fn(self._n.ptr_array(self._rows(sh.delta, a)), self._n.ptr_array(self._rows(sh.cv, a)), c, w, sh.Kr,
                b - a, int(bool(seed)), int(bool(finish)), float(sh.lr), dout.data_ptr() + a * 8,
                cout.data_ptr() + a * 8, _stream())
        self._n.check(rc, "scaffold_chain")

    def scaffold_products(self, sh: ScaffoldShard, ws) -> None:
        P = int(sh.pairwise_idx.size)
        if not P or not sh.Kr:
            return
        fn = getattr(self.lib, f"fedagg_scaffold_products_{sh.kind}")
        idx = (ctypes.c_uint64 * P)(*[int(v) for v in sh.pairwise_idx])
        w = (ctypes.c_double * sh.Kr)(*[float(v) for v in sh.w])
        rc = fn(self._n.ptr_array(self._rows(sh.delta)), self._n.ptr_array(self._rows(sh.cv)), w, sh.Kr, sh.kbase,
                sh.K, idx, P, ws.data_ptr(), _stream())
        self._n.check(rc, "scaffold_products")

    def scaffold_finish(self, sh: ScaffoldShard, ws, dout, cout) -> None:
        P = int(sh.pairwise_idx.size)
        if not P:
            return
        fn = getattr(self.lib, f"fedagg_scaffold_finish_{sh.kind}")
        idx = (ctypes.c_uint64 * P)(*[int(v) for v in sh.pairwise_idx])
        rc = fn(ws.data_ptr(), sh.K, sh.c.data_ptr(), idx, P, float(sh.lr), dout.data_ptr(), cout.data_ptr(),
                _stream())
        self._n.check(rc, "scaffold_finish")

    def _scaffold_final(self, sh: ScaffoldShard, a: int, b: int, dout, cout) -> None:
        """dout[a:b] = lr * (+0 + 1.0 * dout[a:b]), cout[a:b] = +0 + 1.0 * cout[a:b] + c[a:b]: the
        final step of scaffold.py:262-263,293 on accumulators that never hold -0.0, so exact."""
        import torch

        c64 = sh.c[a:b].to(torch.float64)
        w = (ctypes.c_double * 1)(1.0)
        d_in, c_in = dout[a:b].clone().unsqueeze(0), cout[a:b].clone().unsqueeze(0)
        rc = self.lib.fedagg_scaffold_chain_f64(self._n.ptr_array(self._rows(d_in)), self._n.ptr_array(self._rows(c_in)),
                                                c64.data_ptr(), w, 1, b - a, 1, 1, float(sh.lr),
                                                dout.data_ptr() + a * 8, cout.data_ptr() + a * 8, _stream())
        self._n.check(rc, "scaffold_final")

    def scaffold_combine(self, sh: ScaffoldShard, dparts, cparts, dout, cout) -> None:
        """dout = lr * (+0 + sum_b dparts[b]), cout = +0 + sum_b cparts[b] + c (block order): the
        fp64 bucket kernel with weight 1.0 per partial (exact products) -- one launch."""
        import torch

        c64 = sh.c[: sh.M].to(torch.float64) if sh.c.dtype != torch.float64 else sh.c
        G = int(dparts.shape[0])
        w = (ctypes.c_double * G)(*([1.0] * G))
        rc = self.lib.fedagg_scaffold_chain_f64(self._n.ptr_array(self._rows(dparts)),
                                                self._n.ptr_array(self._rows(cparts)), c64.data_ptr(), w, G, sh.M, 1,
                                                1, float(sh.lr), dout.data_ptr(), cout.data_ptr(), _stream())
        self._n.check(rc, "scaffold_combine")


# ======================================================================================
# transports
# ======================================================================================
class DistTransport:
    """The exchange steps over a ``torch.distributed`` group: RCCL (backend "nccl") on device
    tensors in the product; gloo on CPU tensors in the CPU tests.  Ranks are group ranks."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        # one group-wide collective before the first point-to-point call: NCCL's batched P2P must
        # not be the first operation a communicator sees on only some of its ranks (a few tens of
        # microseconds per transport; transports are built once per aggregation, not per step)
        if self.world > 1:
            self.all_sum_int(0)

    def _g(self, r: int) -> int:
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def exchange(self, ops: Sequence[Tuple[str, object, int]]) -> list:
        """Batched point-to-point (``("send"|"recv", tensor, peer)``), one NCCL group; returns the
        works (``wait()`` orders the current stream after them)."""
        if not ops:
            return []
        d = self.dist
        p2p = [d.P2POp(d.isend if kind == "send" else d.irecv, t, self._g(peer), self.group) for kind, t, peer in ops]
        return d.batch_isend_irecv(p2p)

    def reduce_sum(self, t, root: int) -> None:
        self.dist.reduce(t, dst=self._g(root), op=self.dist.ReduceOp.SUM, group=self.group)

    def reduce_sum_async(self, t, root: int):
        """As reduce_sum, returning the work: ``wait()`` orders the current stream after it, so
        the next chunk's kernel overlaps this chunk's reduction."""
        return self.dist.reduce(t, dst=self._g(root), op=self.dist.ReduceOp.SUM, group=self.group, async_op=True)

    def gather(self, t, root: int) -> Optional[list]:
        import torch

        out = [torch.empty_like(t) for _ in range(self.world)] if self.rank == root else None
        self.dist.gather(t, gather_list=out, dst=self._g(root), group=self.group)
        return out

    def all_sum_int(self, v: int) -> int:
        import torch

        dev = torch.device("cuda", torch.cuda.current_device()) if self.dist.get_backend(self.group) == "nccl" \
            else torch.device("cpu")
        t = torch.tensor([int(v)], dtype=torch.int64, device=dev)
        self.dist.all_reduce(t, group=self.group)
        return int(t.item())


class _Done:
    def wait(self):
        return None


class _LoopbackRecv:
    """A posted receive of the loopback transport: ``wait()`` takes the matching message (sent by
    ``src`` to ``owner``) and copies it into ``dst`` on the waiting thread's current stream."""

    def __init__(self, owner: "_LoopbackTransport", dst, src: int):
        self.owner, self.dst, self.src, self.done = owner, dst, src, False

    def wait(self):
        if not self.done:
            src_t, ev = self.owner._get((self.src, self.owner.rank))
            self.dst.copy_(_take(src_t, ev))
            self.done = True


class LoopbackGroup:
    """G ranks as threads of ONE process (rehearsal of the multi-rank protocol on one GPU, and
    the drift tool): point-to-point messages and collectives through in-process mailboxes.
    Device tensors are handed over with an event recorded on the sender's current stream and
    ``record_stream`` on the receiver's, so the ranks' streams stay ordered like RCCL's."""

    def __init__(self, world: int):
        self.world = int(world)
        self._cv = threading.Condition()
        self._p2p: Dict[Tuple[int, int], deque] = {}
        self._coll: Dict[Tuple[int, int], object] = {}

    def transport(self, rank: int) -> "_LoopbackTransport":
        return _LoopbackTransport(self, rank)


def _event(t):
    import torch

    if not t.is_cuda:
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    return ev


def _take(t, ev):
    import torch

    if ev is not None:
        s = torch.cuda.current_stream(t.device)
        s.wait_event(ev)
        t.record_stream(s)
    return t


class _LoopbackTransport:
    def __init__(self, group: LoopbackGroup, rank: int):
        self.g = group
        self.rank = rank
        self.world = group.world
        self._seq = 0

    def _put(self, key, value):
        with self.g._cv:
            self.g._p2p.setdefault(key, deque()).append(value)
            self.g._cv.notify_all()

    def _get(self, key):
        with self.g._cv:
            self.g._cv.wait_for(lambda: bool(self.g._p2p.get(key)))
            return self.g._p2p[key].popleft()

    def exchange(self, ops):
        works = []
        for kind, t, peer in ops:
            if kind == "send":
                self._put((self.rank, peer), (t, _event(t)))
                works.append(_Done())
            else:
                works.append(_LoopbackRecv(self, t, peer))
        return works

    def _collect(self, t, root):
        """Every rank posts (t, event) under the next collective number; the root gets all."""
        key = self._seq
        self._seq += 1
        with self.g._cv:
            self.g._coll[(key, self.rank)] = (t, _event(t))
            self.g._cv.notify_all()
            if self.rank != root:
                return None
            self.g._cv.wait_for(lambda: all((key, r) in self.g._coll for r in range(self.world)))
            got = [self.g._coll.pop((key, r)) for r in range(self.world)]
        return [_take(x, ev) for x, ev in got]

    def reduce_sum(self, t, root: int) -> None:
        got = self._collect(t, root)
        if got is not None:
            acc = got[0].clone()
            for x in got[1:]:
                acc.add_(x)
            t.copy_(acc)

    def reduce_sum_async(self, t, root: int):
        self.reduce_sum(t, root)
        return _Done()

    def gather(self, t, root: int):
        got = self._collect(t, root)
        return None if got is None else [x.clone() for x in got]

    def all_sum_int(self, v: int) -> int:
        import torch

        got = self._collect(torch.tensor([int(v)], dtype=torch.int64), 0)
        key = self._seq
        self._seq += 1
        with self.g._cv:
            if got is not None:  # [total, ranks still to read it]
                self.g._coll[(key, -1)] = [int(sum(int(x.item()) for x in got)), self.world]
                self.g._cv.notify_all()
            self.g._cv.wait_for(lambda: (key, -1) in self.g._coll)
            rec = self.g._coll[(key, -1)]
            rec[1] -= 1
            if rec[1] == 0:
                del self.g._coll[(key, -1)]
        return int(rec[0])


# ======================================================================================
# the client-sharded reductions (device level)
# ======================================================================================
def _neighbours(rank: int, world: int) -> Tuple[int, Optional[int], Optional[int]]:
    b = block_of(rank, world)
    prev = chain_rank(b - 1, world) if b > 0 else None
    nxt = chain_rank(b + 1, world) if b < world - 1 else None
    return b, prev, nxt


def _relay(transport, chunks, tensors: Callable[[int, int], list], run: Callable[[int, int, bool, bool], None],
           prev: Optional[int], nxt: Optional[int]) -> None:
    """Pipelined chain over ``chunks``: receive chunk j's accumulators from ``prev``, run this
    block on them, send them to ``nxt``; the receives run two chunks ahead and every send is
    batched with a receive, so the links of all ranks are busy at once."""
    C = len(chunks)
    recvs: Dict[int, list] = {}

    def post(js):
        ops = []
        for j in js:
            if prev is not None and j < C:
                ops += [("recv", t, prev) for t in tensors(*chunks[j])]
        return ops

    pending = []
    first = post([0, 1])
    if first:
        works = transport.exchange(first)
        n0 = len(tensors(*chunks[0]))
        recvs[0], recvs[1] = works[:n0], works[n0:]
    for j, (a, b) in enumerate(chunks):
        for w in recvs.pop(j, []):
            w.wait()
        run(a, b, prev is None, nxt is None)
        ops = [("send", t, nxt) for t in tensors(a, b)] if nxt is not None else []
        rops = post([j + 2])
        works = transport.exchange(ops + rops)
        pending += works[: len(ops)]
        if rops:
            recvs[j + 2] = works[len(ops):]
    for w in pending:
        w.wait()


def _reduce_async(transport, t, root):
    """transport.reduce_sum_async when the transport has it (else the blocking form)."""
    fn = getattr(transport, "reduce_sum_async", None)
    if fn is not None:
        return fn(t, root)
    transport.reduce_sum(t, root)
    return _Done()


def client_shard_fedavg(sh: FedAvgShard, out, transport, ops, combine: str = "relay", ws=None,
                        chunk_elems: int = RELAY_CHUNK_ELEMS) -> bool:
    """Client-sharded FedAvg (fed_avg.py:217-222) over ``transport``'s ranks: every rank passes
    its :class:`FedAvgShard`; the result lands in ``out`` (``[>= M]``, fp32 for f32/bf16) on the
    root (rank 0), which this returns True on.  ``ws``: optional ``[P, K]`` workspace."""
    import torch

    if combine not in COMBINES:
        raise ValueError(f"combine must be one of {COMBINES}")
    rank, G = transport.rank, transport.world
    root = 0
    b, prev, nxt = _neighbours(rank, G)
    P = int(sh.pairwise_idx.size)
    if P:
        if ws is None:
            ws = torch.zeros((P, sh.K), dtype=ws_dtype(torch, sh.kind), device=out.device)
        else:
            ws.zero_()
        ops.fedavg_products(sh, ws)
    if G == 1:
        ops.fedavg_chain(sh.kind, sh.rows, sh.w, 0, sh.M, True, out)
    elif combine == "relay":
        _relay(transport, relay_chunks(sh.M, chunk_elems), lambda a, b_: [out[a:b_]],
               lambda a, b_, seed, last: ops.fedavg_chain(sh.kind, sh.rows, sh.w, a, b_, seed, out), prev, nxt)
    else:
        if combine == "rccl":  # chunk j's reduction overlaps chunk j + 1's partial
            works = []
            for a, b_ in relay_chunks(sh.M, chunk_elems):
                ops.fedavg_chain(sh.kind, sh.rows, sh.w, a, b_, True, out)  # this block's partial from +0.0
                works.append(_reduce_async(transport, out[a:b_], root))
            for w in works:
                w.wait()
        else:
            ops.fedavg_chain(sh.kind, sh.rows, sh.w, 0, sh.M, True, out)  # this block's partial from +0.0
            parts = transport.gather(out[: sh.M].contiguous(), root)
            if rank == root:
                stack = torch.stack([parts[chain_rank(i, G)] for i in range(G)])  # block order
                ops.fedavg_combine(sh.kind, stack, sh.M, out)
    if P and G > 1:
        transport.reduce_sum(ws, root)  # columns of other blocks are zeros: the sum is exact
    if rank == root and P:
        ops.fedavg_finish(sh.kind, ws, sh.K, sh.pairwise_idx, out)
    return rank == root


def client_shard_scaffold(sh: ScaffoldShard, dout, cout, transport, ops, combine: str = "relay", ws=None,
                          chunk_elems: int = RELAY_CHUNK_ELEMS) -> bool:
    """Client-sharded Scaffold (scaffold.py:262-263, 293; fp64): the averaged update
    ``lr * sum_k w_k delta_k`` into ``dout`` and the new server control variate
    ``sum_k w_k cv_k + c`` into ``cout`` on the root (returns True there).  ``c`` is added last
    and ``lr`` applied after the sum, on the root, in every mode."""
    import torch

    if combine not in COMBINES:
        raise ValueError(f"combine must be one of {COMBINES}")
    rank, G = transport.rank, transport.world
    root = 0
    b, prev, nxt = _neighbours(rank, G)
    P = int(sh.pairwise_idx.size)
    if P:
        n = P * (2 * sh.K + 1)
        if ws is None:
            ws = torch.zeros(n, dtype=torch.float64, device=dout.device)
        else:
            ws.zero_()
        ops.scaffold_products(sh, ws)
    if G == 1:
        ops.scaffold_chain(sh, 0, sh.M, True, True, dout, cout)
    elif combine == "relay":
        _relay(transport, relay_chunks(sh.M, chunk_elems), lambda a, b_: [dout[a:b_], cout[a:b_]],
               lambda a, b_, seed, last: ops.scaffold_chain(sh, a, b_, seed, last, dout, cout), prev, nxt)
    else:
        if combine == "rccl":  # chunk j's reductions overlap chunk j + 1's partial sums
            works = []
            for a, b_ in relay_chunks(sh.M, chunk_elems):
                ops.scaffold_chain(sh, a, b_, True, False, dout, cout)  # plain fp64 partial sums
                works += [_reduce_async(transport, dout[a:b_], root), _reduce_async(transport, cout[a:b_], root)]
            for w in works:
                w.wait()
            if rank == root:  # final step: lr * (0 + 1.0 * sum), 0 + 1.0 * sum + c
                ops.scaffold_combine(sh, dout[: sh.M].unsqueeze(0).clone(), cout[: sh.M].unsqueeze(0).clone(),
                                     dout, cout)
        else:
            ops.scaffold_chain(sh, 0, sh.M, True, False, dout, cout)  # plain fp64 partial sums
            dp = transport.gather(dout[: sh.M].contiguous(), root)
            cp = transport.gather(cout[: sh.M].contiguous(), root)
            if rank == root:
                order = [chain_rank(i, G) for i in range(G)]
                ops.scaffold_combine(sh, torch.stack([dp[r] for r in order]), torch.stack([cp[r] for r in order]),
                                     dout, cout)
    if P and G > 1:
        transport.reduce_sum(ws, root)
    if rank == root and P:
        ops.scaffold_finish(sh, ws, dout, cout)
    return rank == root


# ======================================================================================
# striped relay: S parameter stripes, each a relay over its own chain order
# ======================================================================================
def _units(G: int) -> List[int]:
    """The units of Z_G (chain multipliers), alternating 1, G-1, 3, G-3, ... (for G = 8: 1 7 3 5)."""
    import math

    lo = [a for a in range(1, G) if math.gcd(a, G) == 1] or [1]
    out, i, j = [], 0, len(lo) - 1
    while i <= j:
        out.append(lo[i])
        if j != i:
            out.append(lo[j])
        i, j = i + 1, j - 1
    return out


def stripe_multipliers(G: int, stripes: Optional[int] = None) -> List[int]:
    """One chain multiplier per stripe (default: as many as Z_G has units, at most 4)."""
    u = _units(G)
    n = min(len(u), 4) if stripes is None else max(1, min(int(stripes), len(u)))
    return u[:n]


def stripe_rank(block: int, world: int, a: int) -> int:
    """Rank holding client block ``block`` in a stripe with multiplier ``a``: ``a * (block + 1) mod
    G`` (a = 1 is :func:`chain_rank`); the last block is on the root for every unit ``a``."""
    return (a * (block + 1)) % world


def stripe_block(rank: int, world: int, a: int) -> int:
    """Inverse of :func:`stripe_rank`: the block ``rank`` holds in that stripe."""
    inv = pow(a, -1, world) if world > 1 else 0
    return (inv * rank - 1) % world


def stripe_layout(M: int, K: int, world: int, rank: int, stripes: Optional[int] = None):
    """This rank's part of a striped client-sharded reduction: per stripe ``(lo, hi, a, block,
    k0, k1)`` -- element range, chain multiplier, the client block it holds there and that block's
    clients."""
    mult = stripe_multipliers(world, stripes)
    blocks = client_blocks(K, world)
    out = []
    for (lo, hi), a in zip(shard_bounds(M, len(mult)), mult):
        b = stripe_block(rank, world, a)
        out.append((lo, hi, a, b) + tuple(blocks[b]))
    return out


def _stripe_neighbours(rank: int, world: int, a: int) -> Tuple[Optional[int], Optional[int]]:
    b = stripe_block(rank, world, a)
    prev = stripe_rank(b - 1, world, a) if b > 0 else None
    nxt = stripe_rank(b + 1, world, a) if b < world - 1 else None
    return prev, nxt


def _run_stripes(jobs: Sequence[Callable[[], None]], device) -> None:
    """Run the stripes' relays concurrently: one host thread each, each on its own HIP stream
    (ordered after the caller's stream, and the caller's stream after all of them), so the
    stripes' P2P traffic (one communicator per stripe) and kernels overlap."""
    import torch

    if len(jobs) == 1:
        jobs[0]()
        return
    cuda = device is not None and device.type == "cuda"
    main = torch.cuda.current_stream(device) if cuda else None
    streams = [torch.cuda.Stream(device) for _ in jobs] if cuda else [None] * len(jobs)
    err: List[Optional[BaseException]] = [None] * len(jobs)

    def body(i):
        try:
            if cuda:
                torch.cuda.set_device(device)
                with torch.cuda.stream(streams[i]):
                    jobs[i]()
            else:
                jobs[i]()
        except BaseException as e:  # noqa: BLE001 -- re-raised on the caller's thread
            err[i] = e

    if cuda:
        for st in streams:
            st.wait_stream(main)
    th = [threading.Thread(target=body, args=(i,), name=f"stripe-{i}") for i in range(len(jobs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if cuda:
        for st in streams:
            main.wait_stream(st)
    for e in err:
        if e is not None:
            raise e


def client_shard_fedavg_striped(parts: Sequence[FedAvgShard], bounds: Sequence[Tuple[int, int, int]], out,
                                transports: Sequence, ops, pairwise_idx, ws=None,
                                chunk_elems: int = RELAY_CHUNK_ELEMS) -> bool:
    """Striped relay FedAvg (bit-exact, see the module docstring).  Per stripe s: ``bounds[s] =
    (lo, hi, a)``, ``parts[s]`` this rank's block for that stripe (``rows`` ``[Kb, hi - lo]``, the
    block's global weights, ``kbase``, ``K``, ``M = hi - lo``, ``pairwise_idx`` relative to
    ``lo``), ``transports[s]`` a transport of its own (one communicator per stripe).  The result
    lands in ``out[:M]`` on the root (rank 0), which this returns True on; ``pairwise_idx``: the
    global numel == 1 indices (sorted)."""
    import torch

    tr0 = transports[0]
    rank, G = tr0.rank, tr0.world
    kind, K = parts[0].kind, parts[0].K
    jobs = []
    for sh, (lo, hi, a), tr in zip(parts, bounds, transports):
        o = out[lo:hi]
        if G == 1:
            jobs.append(lambda sh=sh, o=o: ops.fedavg_chain(sh.kind, sh.rows, sh.w, 0, sh.M, True, o))
            continue
        prev, nxt = _stripe_neighbours(rank, G, a)
        jobs.append(lambda sh=sh, o=o, tr=tr, prev=prev, nxt=nxt: _relay(
            tr, relay_chunks(sh.M, chunk_elems), lambda x, y: [o[x:y]],
            lambda x, y, seed, last: ops.fedavg_chain(sh.kind, sh.rows, sh.w, x, y, seed, o), prev, nxt))
    _run_stripes(jobs, out.device)
    P = int(np.asarray(pairwise_idx).size)
    if P:
        pw = np.asarray(pairwise_idx, np.int64)
        if ws is None:
            ws = torch.zeros((P, K), dtype=ws_dtype(torch, kind), device=out.device)
        else:
            ws.zero_()
        for sh, (lo, hi, a) in zip(parts, bounds):
            p0, p1 = int(np.searchsorted(pw, lo)), int(np.searchsorted(pw, hi))
            if p1 > p0:
                ops.fedavg_products(sh, ws[p0:p1])
        if G > 1:
            tr0.reduce_sum(ws, 0)
        if rank == 0:
            ops.fedavg_finish(kind, ws, K, pw.astype(np.uint64), out)
    return rank == 0


def client_shard_scaffold_striped(parts: Sequence[ScaffoldShard], bounds: Sequence[Tuple[int, int, int]], dout,
                                  cout, transports: Sequence, ops, pairwise_idx, c=None, ws=None,
                                  chunk_elems: int = RELAY_CHUNK_ELEMS) -> bool:
    """Striped relay Scaffold (scaffold.py:262-263, 293; bit-exact): per stripe as
    :func:`client_shard_fedavg_striped`, ``parts[s].c`` the stripe's slice of the server control
    variate (read by the root, which holds every stripe's last block and applies ``+ c`` and
    ``lr`` inside its last kernel); ``c``: the whole ``c`` (root, numel == 1 elements only)."""
    import torch

    tr0 = transports[0]
    rank, G = tr0.rank, tr0.world
    K, lr = parts[0].K, parts[0].lr
    jobs = []
    for sh, (lo, hi, a), tr in zip(parts, bounds, transports):
        d, co = dout[lo:hi], cout[lo:hi]
        if G == 1:
            jobs.append(lambda sh=sh, d=d, co=co: ops.scaffold_chain(sh, 0, sh.M, True, True, d, co))
            continue
        prev, nxt = _stripe_neighbours(rank, G, a)
        jobs.append(lambda sh=sh, d=d, co=co, tr=tr, prev=prev, nxt=nxt: _relay(
            tr, relay_chunks(sh.M, chunk_elems), lambda x, y: [d[x:y], co[x:y]],
            lambda x, y, seed, last: ops.scaffold_chain(sh, x, y, seed, last, d, co), prev, nxt))
    _run_stripes(jobs, dout.device)
    P = int(np.asarray(pairwise_idx).size)
    if P:
        pw = np.asarray(pairwise_idx, np.int64)
        n = P * (2 * K + 1)
        if ws is None:
            ws = torch.zeros(n, dtype=torch.float64, device=dout.device)
        else:
            ws.zero_()
        wd, wc = ws[: P * K].view(P, K), ws[P * K:].view(P, K + 1)
        for sh, (lo, hi, a) in zip(parts, bounds):
            p0, p1 = int(np.searchsorted(pw, lo)), int(np.searchsorted(pw, hi))
            if p1 > p0 and sh.Kr:
                tmp = torch.zeros((p1 - p0) * (2 * K + 1), dtype=torch.float64, device=dout.device)
                ops.scaffold_products(sh, tmp)
                wd[p0:p1] += tmp[: (p1 - p0) * K].view(p1 - p0, K)
                wc[p0:p1] += tmp[(p1 - p0) * K:].view(p1 - p0, K + 1)
        if G > 1:
            tr0.reduce_sum(ws, 0)
        if rank == 0:
            glob = ScaffoldShard(parts[0].kind, None, None, c, np.zeros(0), 0, K, int(dout.shape[0]), lr,
                                 pw.astype(np.uint64))
            ops.scaffold_finish(glob, ws, dout, cout)
    return rank == 0


# ======================================================================================
# host entry points (every rank reads the same K host shared states, stages its block)
# ======================================================================================
def _rank_device(torch):
    return torch.device("cuda", torch.cuda.current_device())


def _one_dtype(lists, what: str) -> np.dtype:
    """The single float dtype every array of ``lists`` carries (the sharded host entry points
    stage raw bytes; mixed or integer layers go through the single-process engines, which apply
    NumPy's promotion on the device)."""
    dts = {a.dtype for row in lists for a in row}
    if len(dts) != 1 or next(iter(dts)) not in (np.float16, np.float32, np.float64):
        raise NotImplementedError(f"sharded {what}: every layer of every client must have one float dtype "
                                  f"(got {sorted(str(d) for d in dts)}); use engine_for(...) for mixed dtypes")
    return np.dtype(next(iter(dts)))


def _stage_block(torch, device, rows: List[List[np.ndarray]], layout: BucketLayout, dtype,
                 lo: int = 0, hi: Optional[int] = None):
    """The rows of this rank's clients, staged through the native session's pinned ring into a
    ``[Kr, ld]`` device tensor of ``dtype`` (no host-side packing; stream-ordered before torch's
    work).  Rows of another float dtype are staged raw and widened exactly on the device
    (``fedagg_cast``: Scaffold's fp32 deltas beside fp64 control variates from round 2 on).
    ``lo``/``hi``: only elements ``[lo, hi)`` of every row (a parameter stripe), into a
    ``[Kr, hi - lo]`` view of 64-element-padded rows."""
    from . import runtime
    from .engine import torch_dtype

    full = hi is None
    hi = layout.M if full else hi
    n = hi - lo
    ld = layout.ld if full else max(64, -(-n // 64) * 64)
    t = torch.empty((max(1, len(rows)), ld), dtype=dtype, device=device)
    if rows and n > 0:
        s = runtime.session(device.index)
        src = {a.dtype for r in rows for a in r}
        arrays = [[np.ascontiguousarray(a) for a in r] for r in rows]
        sdt = next(iter(src))
        rng = None if full else (lo * np.dtype(sdt).itemsize, hi * np.dtype(sdt).itemsize)
        if len(src) == 1 and torch_dtype(sdt) != dtype:
            raw = torch.empty((len(rows), ld), dtype=torch_dtype(sdt), device=device)
            s.stage(raw.data_ptr(), ld * raw.element_size(), arrays, byte_range=rng)
            s.cast(raw.data_ptr(), sdt, t.data_ptr(), np.dtype(str(dtype).replace("torch.", "")), len(rows) * ld)
            s.sync()
            del raw
        else:
            s.stage(t.data_ptr(), ld * t.element_size(), arrays, byte_range=rng)
            s.sync()
    return t[: len(rows)] if full else t[: len(rows), :n]


_STRIPE_GROUPS: Dict[tuple, list] = {}


def _stripe_transports(transport, group, stripes: Optional[int], transports):
    """One transport per stripe of the striped relay: given, or one new process group each (every
    rank creates them in the same order)."""
    import torch.distributed as dist

    if transports is not None:
        return list(transports)
    tr = transport or DistTransport(group)
    S = len(stripe_multipliers(tr.world, stripes))
    if tr.world == 1:
        return [tr] * S
    # keyed by the default group too: a re-initialised process group gets fresh communicators
    key = (id(dist.group.WORLD), None if group is None else tuple(dist.get_process_group_ranks(group)), S)
    if key not in _STRIPE_GROUPS:  # communicators are set up once per process, not per aggregation
        ranks = None if group is None else list(key[1])
        _STRIPE_GROUPS[key] = [dist.new_group(ranks=ranks) for _ in range(S - 1)]
    return [tr] + [DistTransport(g) for g in _STRIPE_GROUPS[key]]


def client_sharded_fedavg(parameters_updates: List[List[np.ndarray]], n_samples: Sequence[int], group=None,
                          combine: str = "relay", transport=None, stripes: Optional[int] = None, transports=None):
    """FedAvg (fed_avg.py:217-222) with the clients sharded over the process group: rank r stages
    only its block's buckets (to its own GPU), the chain / reduce runs over RCCL and the root
    (rank 0) returns the averaged layers; other ranks return None.  Layers must share one float
    dtype.  ``combine="relay"`` and ``"striped"`` are bit-identical to the reference
    (``striped``: ``stripes`` parameter stripes, one process group each, see the module
    docstring)."""
    import torch

    from .engine import fedavg_weights, kind_of, torch_dtype

    if combine == "striped":
        trs = _stripe_transports(transport, group, stripes, transports)
        tr = trs[0]
    else:
        tr = transport or DistTransport(group)
    G, rank = tr.world, tr.rank
    K, L = len(parameters_updates), len(parameters_updates[0])
    dtype = _one_dtype(parameters_updates, "FedAvg")
    kind = kind_of(dtype)
    layout = BucketLayout(range(L), [a.shape for a in parameters_updates[0]], dtype)
    dev = _rank_device(torch)
    if combine == "striped":
        w_all = fedavg_weights(n_samples, kind)
        pw = layout.pairwise_idx.astype(np.int64)
        lay = stripe_layout(layout.M, K, G, rank, len(trs))
        parts = []
        for lo, hi, a, b, k0, k1 in lay:
            rows = _stage_block(torch, dev, [parameters_updates[k] for k in range(k0, k1)], layout,
                                torch_dtype(kind), lo, hi)
            parts.append(FedAvgShard(kind, rows, w_all[k0:k1], k0, K, hi - lo,
                                     (pw[(pw >= lo) & (pw < hi)] - lo).astype(np.uint64)))
        out = torch.empty(layout.ld, dtype=out_dtype(torch, kind), device=dev)
        if not client_shard_fedavg_striped(parts, [(lo, hi, a) for lo, hi, a, *_ in lay], out, trs, GpuShardOps(),
                                           pw):
            return None
        flat = out[: layout.M].cpu().numpy()
        return [a for _, a in layout.unpack(np.array(flat, copy=True))]
    k0, k1 = client_blocks(K, G)[block_of(rank, G)]
    rows = _stage_block(torch, dev, [parameters_updates[k] for k in range(k0, k1)], layout, torch_dtype(kind))
    w = fedavg_weights(n_samples, kind)[k0:k1]
    out = torch.empty(layout.ld, dtype=out_dtype(torch, kind), device=dev)
    sh = FedAvgShard(kind, rows, w, k0, K, layout.M, layout.pairwise_idx)
    if not client_shard_fedavg(sh, out, tr, GpuShardOps(), combine):
        return None
    flat = out[: layout.M].cpu().numpy()
    return [a for _, a in layout.unpack(np.array(flat, copy=True))]


def client_sharded_scaffold(parameters_updates, control_variate_updates, server_control_variates, n_samples,
                            aggregation_lr, group=None, combine: str = "relay", transport=None,
                            stripes: Optional[int] = None, transports=None):
    """Scaffold (scaffold.py:193-196, 297-337) with the clients sharded over the process group.
    Every rank checks its block's server control variates against client 0's on the host while
    staging (one device copy of ``c``, needed by the root only).  Returns
    ``(mismatches, new_server_control_variate, avg_parameters_update)`` on the root, None
    elsewhere.  fp32 or fp64 buckets (one dtype for all three lists)."""
    import torch

    from . import runtime
    from .engine import scaffold_weights, torch_dtype

    if combine == "striped":
        trs = _stripe_transports(transport, group, stripes, transports)
        tr = trs[0]
    else:
        tr = transport or DistTransport(group)
    G, rank = tr.world, tr.rank
    K, L = len(parameters_updates), len(parameters_updates[0])
    # fp32 buckets when every list is fp32 (NEP 50: the sums are fp64 either way), else fp64 with
    # exact widening on the device; each list one dtype
    dts = [_one_dtype(lst, "Scaffold") for lst in (parameters_updates, control_variate_updates,
                                                   server_control_variates)]
    if any(d not in (np.float32, np.float64) for d in dts):
        raise NotImplementedError("client-sharded Scaffold takes float32 / float64 lists")
    sdt = np.dtype(np.float32 if all(d == np.float32 for d in dts) else np.float64)
    kind = "f32" if sdt == np.float32 else "f64"
    layout = BucketLayout(range(L), [a.shape for a in parameters_updates[0]], sdt)
    dev = _rank_device(torch)
    td = torch_dtype(kind)
    if combine == "striped":
        return _client_sharded_scaffold_striped(torch, runtime, trs, layout, kind, td, dts[2], dev, parameters_updates,
                                                control_variate_updates, server_control_variates,
                                                scaffold_weights(n_samples), float(aggregation_lr))
    k0, k1 = client_blocks(K, G)[block_of(rank, G)]
    delta = _stage_block(torch, dev, [parameters_updates[k] for k in range(k0, k1)], layout, td)
    cv = _stage_block(torch, dev, [control_variate_updates[k] for k in range(k0, k1)], layout, td)
    # c: client 0's copy staged once (used by the root), this block's copies checked against it
    s = runtime.session(dev.index)
    check_rows = [list(server_control_variates[0])] + [list(server_control_variates[k]) for k in range(k0, k1)
                                                      if k != 0]
    mism = s.check(check_rows, dts[2])
    c = _stage_block(torch, dev, [list(server_control_variates[0])], layout, td)[0]
    mism = tr.all_sum_int(mism)
    dout = torch.empty(layout.ld, dtype=torch.float64, device=dev)
    cout = torch.empty(layout.ld, dtype=torch.float64, device=dev)
    sh = ScaffoldShard(kind, delta, cv, c, scaffold_weights(n_samples)[k0:k1], k0, K, layout.M,
                       float(aggregation_lr), layout.pairwise_idx)
    if not client_shard_scaffold(sh, dout, cout, tr, GpuShardOps(), combine):
        return None
    d = dout[: layout.M].cpu().numpy().copy()
    cc = cout[: layout.M].cpu().numpy().copy()
    return mism, [a for _, a in layout.unpack(cc)], [a for _, a in layout.unpack(d)]


def _client_sharded_scaffold_striped(torch, runtime, trs, layout, kind, td, c_dtype, dev, pus, cvs, cs, w_all, lr):
    """client_sharded_scaffold's striped form: per stripe this rank stages its block's delta and
    control-variate slices, checks the block's server control variates against client 0's on the
    host over the stripe's bytes, and the root stages c once."""
    tr = trs[0]
    G, rank = tr.world, tr.rank
    K = len(pus)
    pw = layout.pairwise_idx.astype(np.int64)
    lay = stripe_layout(layout.M, K, G, rank, len(trs))
    s = runtime.session(dev.index)
    isz = np.dtype(c_dtype).itemsize
    c = _stage_block(torch, dev, [list(cs[0])], layout, td)[0] if rank == 0 else None
    mism = 0
    parts = []
    for lo, hi, a, b, k0, k1 in lay:
        delta = _stage_block(torch, dev, [pus[k] for k in range(k0, k1)], layout, td, lo, hi)
        cv = _stage_block(torch, dev, [cvs[k] for k in range(k0, k1)], layout, td, lo, hi)
        check_rows = [list(cs[0])] + [list(cs[k]) for k in range(k0, k1) if k != 0]
        if len(check_rows) > 1 and hi > lo:
            mism += s.stage_check(0, check_rows, c_dtype, byte_range=(lo * isz, hi * isz))
        parts.append(ScaffoldShard(kind, delta, cv, c[lo:hi] if c is not None else None, w_all[k0:k1], k0, K, hi - lo,
                                   lr, (pw[(pw >= lo) & (pw < hi)] - lo).astype(np.uint64)))
    mism = tr.all_sum_int(mism)
    dout = torch.empty(layout.ld, dtype=torch.float64, device=dev)
    cout = torch.empty(layout.ld, dtype=torch.float64, device=dev)
    if not client_shard_scaffold_striped(parts, [(lo, hi, a) for lo, hi, a, *_ in lay], dout, cout, trs,
                                         GpuShardOps(), pw, c=c):
        return None
    d = dout[: layout.M].cpu().numpy().copy()
    cc = cout[: layout.M].cpu().numpy().copy()
    return mism, [a for _, a in layout.unpack(cc)], [a for _, a in layout.unpack(d)]


# ======================================================================================
# parameter-range sharding (primary, bit-exact, no arithmetic collective)
# ======================================================================================
# reducer(rows [K, n] host array of the slice, n_samples, pairwise_idx (slice-local)) -> [n] array
Reducer = Callable[[np.ndarray, Sequence[int], np.ndarray], np.ndarray]


def param_range_fedavg(
    parameters_updates: List[List[np.ndarray]],
    n_samples: Sequence[int],
    group=None,
    reducer: Optional[Reducer] = None,
    gather: bool = True,
):
    """FedAvg over a process group with parameter-range sharding (bit-exact).

    Every rank passes the same host shared states (as every rank of a node would read the same
    task inputs); rank ``r`` stages bytes ``[lo_r, hi_r)`` of every client's row straight from
    the layer arrays into its HBM (``fedagg_session_stage_range``) and reduces them with the
    single-GPU kernel.  With ``gather=True`` every rank returns the full list of averaged layers
    (RCCL all-gather of the device slices); otherwise ``(lo, hi, slice)``.  Layers must share one
    floating dtype (the single-GPU engine handles mixed dtypes).  ``reducer``: CPU tests only
    (host rows in, host slice out)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    L = len(parameters_updates[0])
    dtype = _one_dtype(parameters_updates, "FedAvg")
    layout = BucketLayout(range(L), [a.shape for a in parameters_updates[0]], dtype)
    bounds = shard_bounds(layout.M, world)
    lo, hi = bounds[rank]
    K = len(parameters_updates)
    pw = layout.pairwise_idx.astype(np.int64)
    pw_local = (pw[(pw >= lo) & (pw < hi)] - lo).astype(np.uint64)
    chunk = bounds[0][1] - bounds[0][0]
    on_gpu = dist.get_backend(group) == "nccl" or reducer is None
    if reducer is not None:  # CPU test path: host rows, injected reducer
        rows = np.zeros((K, max(1, hi - lo)), dtype=dtype)
        for k in range(K):
            pack_range(layout, parameters_updates[k], rows[k], lo, hi)
        part_h = reducer(rows[:, : hi - lo], n_samples, pw_local) if hi > lo else np.zeros(0, dtype)
        if not gather:
            return lo, hi, part_h
        send = torch.zeros(chunk, dtype=torch.from_numpy(np.zeros(0, dtype)).dtype)
        send[: hi - lo] = torch.from_numpy(np.ascontiguousarray(part_h))
    else:
        from .engine import FedAvgPlan, fedavg_weights, kind_of, torch_dtype

        kind = kind_of(dtype)
        dev = _rank_device(torch)
        n = hi - lo
        isz = np.dtype(dtype).itemsize
        ld = max(4, -(-max(1, n) // 64) * 64)
        x = torch.empty((K, ld), dtype=torch_dtype(kind), device=dev)
        send = torch.zeros(chunk, dtype=torch_dtype(kind), device=dev)
        if n > 0:
            from . import runtime

            s = runtime.session(dev.index)
            s.stage(x.data_ptr(), ld * isz, [[np.ascontiguousarray(a) for a in pu] for pu in parameters_updates],
                    byte_range=(lo * isz, hi * isz))
            s.sync()
            FedAvgPlan(kind, x, fedavg_weights(n_samples, kind), n, send, pw_local).launch()
        if not gather:
            torch.cuda.synchronize(dev)
            return lo, hi, send[:n].cpu().numpy()
        if not on_gpu:
            send = send.cpu()
    recv = torch.empty(chunk * world, dtype=send.dtype, device=send.device)
    if dist.get_backend(group) != "nccl" and send.is_cuda:
        # gloo rehearsal (ranks sharing one GPU): the exchange bounces through host memory
        r = torch.empty(chunk * world, dtype=send.dtype)
        dist.all_gather_into_tensor(r, send.cpu(), group=group)
        recv = r
    else:
        dist.all_gather_into_tensor(recv, send, group=group)
    flat = recv[: layout.M].cpu().numpy()
    return [a for _, a in layout.unpack(np.array(flat, copy=True))]
