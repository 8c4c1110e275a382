"""Multi-GPU aggregation, one process per GPU over ``torch.distributed`` (RCCL on ROCm).

Two layouts:

* **Parameter-range sharding (primary, bit-exact).**  The reduction is independent per element,
  so rank ``r`` owns elements ``[lo_r, hi_r)`` of every client's flat bucket, stages only that
  slice over its own PCIe link, and reduces it with the same kernel and the same client order as
  one GPU.  No arithmetic crosses GPUs; results are bit-identical to the single-GPU path and to
  the reference.  The optional final gather to every rank is a plain all-gather of the result
  slices (RCCL over xGMI), not a reduction.
* **Client sharding (the north-star mode).**  The K clients are cut into G contiguous blocks
  whose buckets live in different GPUs' HBM, and the reference's sequential client sum
  (fed_avg.py:221-222; scaffold.py:262-263, 293) is completed across the ranks, device-resident
  (partial sums stay in HBM, the exchange is RCCL over xGMI, the result lands on the root):

  ``combine="relay"`` (default, **bit-exact**): rank ``(b + 1) % G`` holds block b for every
  element; the bucket is cut into chunks whose accumulators travel down the chain of blocks
  0..G-1 (each rank CONTINUES the accumulator it receives), so every element sees exactly the
  reference's rounding sequence.  The last block is on the root, which applies Scaffold's final
  step (+ c, then ``aggregation_lr``) inside its last kernel.
  ``combine="striped"`` (**bit-exact**): the same chains, over pieces scheduled so that every
  rank runs one block of one piece per ring at every step and sends on several xGMI links at
  once (:mod:`lockstep`); a stripe's final chunk goes from its last rank to the root.
  Both run as a :mod:`lockstep` schedule: ONE host thread, ONE communicator, exchange group t on
  every rank pairing only with group t on its peers -- deadlock-free by construction.
  ``combine="rccl"``: every block sums from +0.0, the partials are summed by ``dist.reduce``
  (RCCL's order) and the root applies the final scale.  Re-associates the client sum: a few ulp
  off the reference (DESIGN.md §6 drift table).
  ``combine="ordered"``: the partials are gathered on the root and added in block order by the
  bucket kernel (weight 1.0 per partial; Scaffold: lr and + c in the same launch).
  Deterministic, same drift class as ``rccl``.

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

from . import lockstep
from .layout import BucketLayout
from .lockstep import SLOTS, chain_rank, ring_multipliers, striped_pieces

SHARD_ALIGN = 512  # elements (2 KiB of fp32): every shard starts on a 256-B boundary
RELAY_CHUNK_ELEMS = 2 << 20  # pipelined relay: >= 2M elements (8 MB fp32) per P2P message
COMBINES = ("relay", "rccl", "ordered", "striped")


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
    """Block b = clients ``[k0, k1)`` (contiguous, list order): sizes differ by at most one, so
    every block holds a client once K >= world (the native executor's condition); with fewer
    clients than ranks, one client per block and the trailing blocks empty."""
    if K < world:
        return [(min(K, b), min(K, b + 1)) for b in range(world)]
    return [(b * K // world, (b + 1) * K // world) for b in range(world)]


def block_of(rank: int, world: int) -> int:
    """The block a rank holds in the plain relay (inverse of :func:`lockstep.chain_rank`)."""
    return (rank - 1) % world


def relay_chunks(M: int, chunk_elems: int = RELAY_CHUNK_ELEMS) -> List[Tuple[int, int]]:
    """Pipelining chunks of ``[0, M)`` (SHARD_ALIGN multiples; at least one)."""
    step = max(SHARD_ALIGN, -(-chunk_elems // SHARD_ALIGN) * SHARD_ALIGN)
    if M <= 0:
        return [(0, 0)]
    return [(a, min(M, a + step)) for a in range(0, M, step)]


def relay_plan(M: int, world: int, rank: int, chunk_elems: int = RELAY_CHUNK_ELEMS) -> lockstep.RankPlan:
    """This rank's part of the plain relay (its one block's buffer is indexed by global element)."""
    return lockstep.rank_plan(lockstep.relay_pieces(M, world, chunk_elems), world, rank, cols="global")


def striped_plan(M: int, world: int, rank: int, rings: Optional[int] = None,
                 rounds: Optional[Sequence[float]] = None) -> lockstep.RankPlan:
    """This rank's part of the striped relay: per client block, the element ranges it holds
    (``plan.blocks[b]``: ``(lo, hi, col)``, packed into a ``[Kb, plan.block_len[b]]`` buffer)."""
    return lockstep.rank_plan(striped_pieces(M, world, rings, rounds or lockstep.DEFAULT_ROUNDS), world, rank,
                              cols="packed")


def default_rounds(transport) -> Sequence[float]:
    """The striped schedule's round split for a transport: three rounds for the native RCCL
    executor over more than one rank, else one (lockstep.DEFAULT_ROUNDS / NATIVE_ROUNDS).  The push
    executor takes one: its finished pieces reach the root inside the final runs' own stores, so
    there is no gather tail for more rounds to hide."""
    native = getattr(transport, "native", False) and not getattr(transport, "push", False)
    return lockstep.default_rounds(getattr(transport, "world", 1), native)


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
    (the server control variate, ``[ld]``) is read where a block's final step runs."""

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


class TiledView:
    """One run's operand in the tile-interleaved layout (``engine.tiled_*``: tile t of client k at
    tile ``t * K + k`` of ``base``): K clients x n elements, tiles of ``tv`` 16-B vectors."""

    def __init__(self, kind: str, base, K: int, n: int, tv: int):
        self.kind, self.base, self.K, self.n, self.tv = kind, base, int(K), int(n), int(tv)
        self.shape = (self.K, self.n)


class TiledBlock:
    """A rank's buffer for one client block of a lockstep schedule in the tile-interleaved layout:
    ONE tiled bucket per run of the plan (the run is the unit of a launch), so each workgroup step
    of the chain kernel reads one contiguous Kb x tile region instead of Kb streams a row apart.
    ``block[:, col:col + n]`` is the :class:`TiledView` of the run starting at ``col``."""

    def __init__(self, kind: str, K: int, width: int, tv: int, buckets: Dict[int, Tuple[object, int]]):
        self.kind, self.K, self.tv = kind, int(K), int(tv)
        self.buckets = dict(buckets)  # col -> (flat device tensor, n)
        self.shape = (self.K, int(width))

    def __getitem__(self, idx):
        _, sl = idx
        t, n = self.buckets[sl.start]
        if sl.stop - sl.start != n:
            raise IndexError("a tiled block is sliced by whole runs")
        return TiledView(self.kind, t, self.K, n, self.tv)

    def locate(self, col: int) -> Tuple[object, int]:
        """(bucket tensor, element offset in its run) of block column ``col``."""
        for c0, (t, n) in self.buckets.items():
            if c0 <= col < c0 + n:
                return t, col - c0
        raise IndexError(col)

    @staticmethod
    def run_extents(plan: lockstep.RankPlan, block: int) -> List[Tuple[int, int]]:
        """(col, n) of every run of ``block`` in ``plan`` (the buckets a tiled block holds)."""
        return sorted({(r.col, r.n) for runs in plan.runs for r in runs if r.block == block})

    @classmethod
    def empty(cls, torch, kind: str, K: int, width: int, tv: int, extents, device):
        from .engine import tiled_elems, torch_dtype

        return cls(kind, K, width, tv, {c: (torch.zeros(tiled_elems(kind, K, n, tv), dtype=torch_dtype(kind),
                                                        device=device), n) for c, n in extents})

    @classmethod
    def from_rows(cls, torch, kind: str, rows, tv: int, extents):
        """Re-tile a ``[Kb, width]`` rows buffer run by run on the device (one strided copy each)."""
        from .engine import _ELEMS_PER_VEC

        K, width = int(rows.shape[0]), int(rows.shape[1])
        blk = cls.empty(torch, kind, K, width, tv, extents, rows.device)
        TL = int(tv) * _ELEMS_PER_VEC[kind]
        for c, (t, n) in blk.buckets.items():
            tiles = -(-n // TL)
            src = torch.zeros((K, tiles * TL), dtype=rows.dtype, device=rows.device)
            src[:, :n] = rows[:, c: c + n]
            t.view(tiles, K, TL).copy_(src.view(K, tiles, TL).permute(1, 0, 2))
        return blk


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
    against them).  Operands are tensor views: ``rows`` ``[Kb, n]`` (row stride free),
    accumulators ``[n]``."""

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

    def fedavg_run(self, kind, rows, w, seed: bool, acc) -> None:
        """acc = (seed ? +0 : acc) + the clients of ``rows`` (``[Kb, n]``) in order."""
        n = int(acc.shape[0])
        if n == 0:
            return
        if rows.shape[0] == 0:  # an empty block passes the accumulator on (or starts it at +0)
            if seed:
                acc.zero_()
            return
        if isinstance(rows, TiledView):
            fn = getattr(self.lib, f"fedagg_fedavg_chain_tiled_{kind}")
            rc = fn(rows.base.data_ptr(), self._weights(kind, w), rows.K, n, rows.tv, int(bool(seed)), acc.data_ptr(),
                    _stream())
            self._n.check(rc, "fedavg_chain_tiled")
            return
        fn = getattr(self.lib, f"fedagg_fedavg_chain_{kind}")
        rc = fn(self._n.ptr_array(self._rows(rows)), self._weights(kind, w), int(rows.shape[0]), n, int(bool(seed)),
                acc.data_ptr(), _stream())
        self._n.check(rc, "fedavg_chain")

    def fedavg_chain(self, kind, rows, w, a: int, b: int, seed: bool, out) -> None:
        """out[a:b] = (seed ? +0 : out[a:b]) + the clients of ``rows`` in order."""
        if b > a:
            self.fedavg_run(kind, rows[:, a:b], w, seed, out[a:b])

    def fedavg_products_at(self, kind, rows, w, kbase: int, K: int, idx, ws) -> None:
        """ws[p, kbase + k] = fl(rows[k, idx[p]] * w[k]) (numel == 1 products of this block)."""
        P = int(np.asarray(idx).size)
        if not P or not rows.shape[0]:
            return
        fn = getattr(self.lib, f"fedagg_pairwise_products_{kind}")
        if isinstance(rows, TiledBlock):  # client k's tile 0 as its base, indices mapped into the tiles
            from .engine import tiled_index

            for p, col in enumerate(np.asarray(idx, np.int64)):
                t, e = rows.locate(int(col))
                ptrs = [t.data_ptr() + k * rows.tv * 16 for k in range(rows.K)]
                ia = (ctypes.c_uint64 * 1)(int(tiled_index(kind, rows.K, 0, e, rows.tv)))
                rc = fn(self._n.ptr_array(ptrs), self._weights(kind, w), rows.K, ia, 1, K, kbase,
                        ws[p:].data_ptr(), _stream())
                self._n.check(rc, "pairwise_products")
            return
        ia = (ctypes.c_uint64 * P)(*[int(v) for v in np.asarray(idx)])
        rc = fn(self._n.ptr_array(self._rows(rows)), self._weights(kind, w), int(rows.shape[0]), ia, P, K, kbase,
                ws.data_ptr(), _stream())
        self._n.check(rc, "pairwise_products")

    def fedavg_products(self, sh: FedAvgShard, ws) -> None:
        self.fedavg_products_at(sh.kind, sh.rows, sh.w, sh.kbase, sh.K, sh.pairwise_idx, ws)

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
    def scaffold_run(self, kind, delta, cv, w, seed: bool, finish: bool, c, lr: float, dacc, cacc) -> None:
        """dacc/cacc = (seed ? +0 : themselves) + this block's clients, in order; ``finish`` (the
        last block): then ``+ c`` (``c``: the same elements of the server control variate) and
        ``* lr``."""
        n = int(dacc.shape[0])
        if n == 0:
            return
        if delta.shape[0] == 0:  # an empty block: pass the accumulators on (start them at +0), finish them
            if seed:
                dacc.zero_()
                cacc.zero_()
            if finish:
                self._scaffold_final(c, lr, dacc, cacc)
            return
        fn = getattr(self.lib, f"fedagg_scaffold_chain_{kind}")
        wa = (ctypes.c_double * delta.shape[0])(*[float(v) for v in w])
        rc = fn(self._n.ptr_array(self._rows(delta)), self._n.ptr_array(self._rows(cv)),
                c.data_ptr() if finish else None, wa, int(delta.shape[0]), n, int(bool(seed)), int(bool(finish)),
                float(lr), dacc.data_ptr(), cacc.data_ptr(), _stream())
        self._n.check(rc, "scaffold_chain")

    def scaffold_chain(self, sh: ScaffoldShard, a: int, b: int, seed: bool, finish: bool, dout, cout) -> None:
        """dout/cout[a:b] = (seed ? +0 : themselves) + this block's clients, in order; ``finish``
        (last block): then ``+ c`` and ``* lr``."""
        if b > a:
            self.scaffold_run(sh.kind, sh.delta[:, a:b], sh.cv[:, a:b], sh.w, seed, finish,
                              sh.c[a:b] if finish else None, sh.lr, dout[a:b], cout[a:b])

    def scaffold_products_at(self, kind, delta, cv, w, kbase: int, K: int, idx, ws) -> None:
        P = int(np.asarray(idx).size)
        if not P or not delta.shape[0]:
            return
        fn = getattr(self.lib, f"fedagg_scaffold_products_{kind}")
        ia = (ctypes.c_uint64 * P)(*[int(v) for v in np.asarray(idx)])
        wa = (ctypes.c_double * delta.shape[0])(*[float(v) for v in w])
        rc = fn(self._n.ptr_array(self._rows(delta)), self._n.ptr_array(self._rows(cv)), wa, int(delta.shape[0]),
                kbase, K, ia, P, ws.data_ptr(), _stream())
        self._n.check(rc, "scaffold_products")

    def scaffold_products(self, sh: ScaffoldShard, ws) -> None:
        self.scaffold_products_at(sh.kind, sh.delta, sh.cv, sh.w, sh.kbase, sh.K, sh.pairwise_idx, ws)

    def scaffold_finish(self, sh: ScaffoldShard, ws, dout, cout) -> None:
        P = int(sh.pairwise_idx.size)
        if not P:
            return
        fn = getattr(self.lib, f"fedagg_scaffold_finish_{sh.kind}")
        idx = (ctypes.c_uint64 * P)(*[int(v) for v in sh.pairwise_idx])
        rc = fn(ws.data_ptr(), sh.K, sh.c.data_ptr(), idx, P, float(sh.lr), dout.data_ptr(), cout.data_ptr(),
                _stream())
        self._n.check(rc, "scaffold_finish")

    def _scaffold_final(self, c, lr, dacc, cacc) -> None:
        """dacc = lr * (+0 + 1.0 * dacc), cacc = +0 + 1.0 * cacc + c: the final step of
        scaffold.py:262-263,293 on accumulators that never hold -0.0, so exact."""
        import torch

        n = int(dacc.shape[0])
        c64 = c[:n].to(torch.float64)
        w = (ctypes.c_double * 1)(1.0)
        d_in, c_in = dacc.clone().unsqueeze(0), cacc.clone().unsqueeze(0)
        rc = self.lib.fedagg_scaffold_chain_f64(self._n.ptr_array(self._rows(d_in)), self._n.ptr_array(self._rows(c_in)),
                                                c64.data_ptr(), w, 1, n, 1, 1, float(lr), dacc.data_ptr(),
                                                cacc.data_ptr(), _stream())
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
_WARMED: set = set()


class DistTransport:
    """The exchange steps over a ``torch.distributed`` group: RCCL (backend "nccl") on device
    tensors in the product; gloo on CPU tensors in the CPU tests.  Ranks are group ranks.  One
    transport = one communicator; the lockstep combines issue everything through it from the
    calling thread."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 1:
            # a group-wide collective before the first point-to-point call (NCCL's batched P2P
            # must not be the first operation a communicator sees on only some of its ranks),
            # then every peer pair's P2P connection, once per process and communicator
            self.all_sum_int(0)
            key = (id(dist.group.WORLD), None if group is None else tuple(dist.get_process_group_ranks(group)))
            if key not in _WARMED:
                self.warm_p2p()
                _WARMED.add(key)

    def _g(self, r: int) -> int:
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def _device(self):
        import torch

        # RCCL carries device tensors ("nccl", or the cuda half of "cpu:gloo,cuda:nccl")
        return torch.device("cuda", torch.cuda.current_device()) if "nccl" in str(self.dist.get_backend(self.group)) \
            else torch.device("cpu")

    def warm_p2p(self) -> None:
        """One element to and from every peer in ONE batched group, on every rank at once: RCCL
        connects a peer pair at its first send/recv, so this keeps the connection set-up out of
        the lockstep schedule's first groups."""
        import torch

        dev = self._device()
        peers = [p for p in range(self.world) if p != self.rank]
        sends = [torch.zeros(1, device=dev) for _ in peers]
        recvs = [torch.empty(1, device=dev) for _ in peers]
        ops = [("send", s, p) for s, p in zip(sends, peers)] + [("recv", r, p) for r, p in zip(recvs, peers)]
        for w in self.exchange(ops):
            w.wait()
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()

    def exchange(self, ops: Sequence[Tuple[str, object, int]]) -> list:
        """Batched point-to-point (``("send"|"recv", tensor, peer)``), one NCCL group; returns the
        works (``wait()`` orders the current stream after them).  With NCCL the whole batch may
        come back as ONE work (torch's coalescing manager): callers wait on every work returned."""
        if not ops:
            return []
        d = self.dist
        p2p = [d.P2POp(d.isend if kind == "send" else d.irecv, t, self._g(peer), self.group) for kind, t, peer in ops]
        return list(d.batch_isend_irecv(p2p) or [])

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

        t = torch.tensor([int(v)], dtype=torch.int64, device=self._device())
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
    A send posts a snapshot of the tensor (the sender may reuse its buffer at once, as after an
    RCCL send completes); device tensors are handed over with an event recorded on the sender's
    current stream and ``record_stream`` on the receiver's, so the ranks' streams stay ordered
    like RCCL's."""

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
                snap = t.clone()
                self._put((self.rank, peer), (snap, _event(snap)))
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
def _reduce_async(transport, t, root):
    """transport.reduce_sum_async when the transport has it (else the blocking form)."""
    fn = getattr(transport, "reduce_sum_async", None)
    if fn is not None:
        return fn(t, root)
    transport.reduce_sum(t, root)
    return _Done()


def _slots(torch, plan, like, n_acc: int = 1, slots=None):
    """The schedule's accumulator slots: ``[n_acc, SLOTS, slot_elems]`` of ``like``'s dtype."""
    need = max(1, plan.slot_elems)
    if slots is not None and slots.numel() >= n_acc * SLOTS * need and slots.dtype == like.dtype:
        return slots.reshape(-1)[: n_acc * SLOTS * need].view(n_acc, SLOTS, need)
    return torch.empty((n_acc, SLOTS, need), dtype=like.dtype, device=like.device)


def lockstep_fedavg(plan: lockstep.RankPlan, blocks: Dict[int, FedAvgShard], out, transport, ops, pairwise_idx,
                    ws=None, slots=None) -> bool:
    """Run one rank's part of a relay / striped FedAvg schedule (fed_avg.py:217-222, bit-exact).
    ``blocks[b]``: this rank's buffer for client block b (``rows`` ``[Kb, plan.block_len[b]]``
    in the plan's columns, the block's GLOBAL weights, ``kbase``, ``K``); ``out``: ``[>= M]``
    result on the root, which this returns True on; ``pairwise_idx``: the global numel == 1
    indices (sorted).  ``ws`` / ``slots``: optional reusable workspaces."""
    import torch

    sh0 = next(iter(blocks.values()))
    kind, K = sh0.kind, sh0.K
    acc = _slots(torch, plan, out, 1, slots)[0]
    pw = np.asarray(pairwise_idx, np.int64)
    if pw.size:
        if ws is None:
            ws = torch.zeros((pw.size, K), dtype=ws_dtype(torch, kind), device=out.device)
        else:
            ws.zero_()
    native = _native_schedule(transport, K, plan.world)
    if not native:
        transport = _python_transport(transport)
    if native:  # rccl.RcclTransport: the whole schedule issued from C++ (csrc/lockstep.hip)
        prog = transport.program(plan=plan, blocks=blocks, accs=[acc], outs=[out], kind=kind, scaffold=False)
        for b, p0, p1, cols in lockstep.pairwise_segments(plan, pw):  # before the schedule, same stream
            sh = blocks[b]
            ops.fedavg_products_at(kind, sh.rows, sh.w, sh.kbase, K, cols, ws[p0:p1])
        transport.execute(prog, _stream(), ws=ws if pw.size else None, ws_kind="f64" if kind == "f64" else "f32")
    else:
        def region(loc, n):
            where, slot, off = loc
            return [(out if where == "out" else acc[slot])[off: off + n]]

        def launch(r):
            sh = blocks[r.block]
            ops.fedavg_run(kind, sh.rows[:, r.col: r.col + r.n], sh.w, r.seed, region(r.acc, r.n)[0])

        lockstep.run(plan, transport, region, launch)
        for b, p0, p1, cols in lockstep.pairwise_segments(plan, pw):
            sh = blocks[b]
            ops.fedavg_products_at(kind, sh.rows, sh.w, sh.kbase, K, cols, ws[p0:p1])
        if pw.size and plan.world > 1:
            transport.reduce_sum(ws, plan.root)  # columns of other blocks are zeros: the sum is exact
    if pw.size and plan.rank == plan.root:
        ops.fedavg_finish(kind, ws, K, pw.astype(np.uint64), out)
    return plan.rank == plan.root


def lockstep_scaffold(plan: lockstep.RankPlan, blocks: Dict[int, ScaffoldShard], dout, cout, transport, ops,
                      pairwise_idx, c, lr: float, ws=None, slots=None) -> bool:
    """One rank's part of a relay / striped Scaffold schedule (scaffold.py:262-263, 293; fp64,
    bit-exact): the averaged update ``lr * sum_k w_k delta_k`` into ``dout`` and the new server
    control variate ``sum_k w_k cv_k + c`` into ``cout`` on the root (True there).  ``c``: the
    whole server control variate (global indexing), read where a stripe's last block runs (the
    root, and for ``striped`` every rank) and on the root for the numel == 1 elements."""
    import torch

    sh0 = next(iter(blocks.values()))
    kind, K = sh0.kind, sh0.K
    acc = _slots(torch, plan, dout, 2, slots)
    pw = np.asarray(pairwise_idx, np.int64)
    P = int(pw.size)
    if P:
        n = P * (2 * K + 1)
        if ws is None:
            ws = torch.zeros(n, dtype=torch.float64, device=dout.device)
        else:
            ws.zero_()

    def products():
        wd, wc = ws[: P * K].view(P, K), ws[P * K:].view(P, K + 1)
        for b, p0, p1, cols in lockstep.pairwise_segments(plan, pw):
            sh = blocks[b]
            if not sh.Kr:
                continue
            tmp = torch.zeros((p1 - p0) * (2 * K + 1), dtype=torch.float64, device=dout.device)
            ops.scaffold_products_at(kind, sh.delta, sh.cv, sh.w, sh.kbase, K, cols, tmp)
            wd[p0:p1] += tmp[: (p1 - p0) * K].view(p1 - p0, K)
            wc[p0:p1] += tmp[(p1 - p0) * K:].view(p1 - p0, K + 1)

    native = _native_schedule(transport, K, plan.world)
    if not native:
        transport = _python_transport(transport)
    if native:  # rccl.RcclTransport: the whole schedule issued from C++ (csrc/lockstep.hip)
        prog = transport.program(plan=plan, blocks=blocks, accs=[acc[0], acc[1]], outs=[dout, cout], kind=kind,
                                 scaffold=True, c=c, lr=lr)
        if P:
            products()
        transport.execute(prog, _stream(), ws=ws if P else None, ws_kind="f64")
    else:
        def region(loc, n):
            where, slot, off = loc
            if where == "out":
                return [dout[off: off + n], cout[off: off + n]]
            return [acc[0, slot, off: off + n], acc[1, slot, off: off + n]]

        def launch(r):
            sh = blocks[r.block]
            d, cc = region(r.acc, r.n)
            ops.scaffold_run(kind, sh.delta[:, r.col: r.col + r.n], sh.cv[:, r.col: r.col + r.n], sh.w, r.seed,
                             r.final, c[r.lo: r.lo + r.n] if r.final else None, lr, d, cc)

        lockstep.run(plan, transport, region, launch)
        if P:
            products()
            if plan.world > 1:
                transport.reduce_sum(ws, plan.root)
    if P:
        if plan.rank == plan.root:
            glob = ScaffoldShard(kind, None, None, c, np.zeros(0), 0, K, int(dout.shape[0]), lr, pw.astype(np.uint64))
            ops.scaffold_finish(glob, ws, dout, cout)
    return plan.rank == plan.root


def client_shard_fedavg(sh: FedAvgShard, out, transport, ops, combine: str = "relay", ws=None,
                        chunk_elems: int = RELAY_CHUNK_ELEMS) -> bool:
    """Client-sharded FedAvg (fed_avg.py:217-222) over ``transport``'s ranks with one client block
    per rank (rank ``(b + 1) % G`` holds block b, :func:`block_of`): every rank passes its
    :class:`FedAvgShard`; the result lands in ``out`` (``[>= M]``, fp32 for f32/bf16) on the root
    (rank 0), which this returns True on.  ``ws``: optional ``[P, K]`` workspace.  (``striped``
    holds a block per stripe instead: :func:`lockstep_fedavg` with :func:`striped_plan`.)"""
    import torch

    if combine not in ("relay", "rccl", "ordered"):
        raise ValueError("combine must be one of ('relay', 'rccl', 'ordered') (striped: lockstep_fedavg)")
    rank, G = transport.rank, transport.world
    root = 0
    if combine == "relay" or G == 1:
        plan = relay_plan(sh.M, G, rank, chunk_elems)
        return lockstep_fedavg(plan, {block_of(rank, G): sh}, out, transport, ops, sh.pairwise_idx, ws=ws)
    transport = _python_transport(transport)
    P = int(sh.pairwise_idx.size)
    if P:
        if ws is None:
            ws = torch.zeros((P, sh.K), dtype=ws_dtype(torch, sh.kind), device=out.device)
        else:
            ws.zero_()
        ops.fedavg_products(sh, ws)
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
    if P:
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

    if combine not in ("relay", "rccl", "ordered"):
        raise ValueError("combine must be one of ('relay', 'rccl', 'ordered') (striped: lockstep_scaffold)")
    rank, G = transport.rank, transport.world
    root = 0
    if combine == "relay" or G == 1:
        plan = relay_plan(sh.M, G, rank, chunk_elems)
        return lockstep_scaffold(plan, {block_of(rank, G): sh}, dout, cout, transport, ops, sh.pairwise_idx, sh.c,
                                 sh.lr, ws=ws)
    transport = _python_transport(transport)
    P = int(sh.pairwise_idx.size)
    if P:
        n = P * (2 * sh.K + 1)
        if ws is None:
            ws = torch.zeros(n, dtype=torch.float64, device=dout.device)
        else:
            ws.zero_()
        ops.scaffold_products(sh, ws)
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
    if P:
        transport.reduce_sum(ws, root)
    if rank == root and P:
        ops.scaffold_finish(sh, ws, dout, cout)
    return rank == root


# ======================================================================================
# host entry points (every rank reads the same K host shared states, stages its blocks)
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
                 segs: Optional[Sequence[Tuple[int, int, int]]] = None, ncols: Optional[int] = None):
    """The rows of a client block, staged through the native session's pinned ring into a
    ``[Kb, ld]`` device tensor of ``dtype`` (no host-side packing; stream-ordered before torch's
    work).  Rows of another float dtype are staged raw and widened exactly on the device
    (``fedagg_cast``: Scaffold's fp32 deltas beside fp64 control variates from round 2 on).
    ``segs``: only elements ``[lo, hi)`` of every row, each at column ``col`` of a
    ``[Kb, ncols]`` buffer (a striped block, ``plan.blocks[b]``)."""
    from . import runtime
    from .engine import torch_dtype

    full = segs is None
    width = layout.M if full else int(ncols)
    ld = layout.ld if full else max(64, -(-width // 64) * 64)
    t = torch.empty((max(1, len(rows)), ld), dtype=dtype, device=device)
    todo = [(0, layout.M, 0)] if full else [(lo, hi, c) for lo, hi, c in segs if hi > lo]
    if rows and todo:
        s = runtime.session(device.index)
        src = {a.dtype for r in rows for a in r}
        arrays = [[np.ascontiguousarray(a) for a in r] for r in rows]
        sdt = next(iter(src))
        isz = np.dtype(sdt).itemsize
        raw = t
        if len(src) == 1 and torch_dtype(sdt) != dtype:
            raw = torch.empty((len(rows), ld), dtype=torch_dtype(sdt), device=device)
        for lo, hi, col in todo:
            rng = None if full else (lo * isz, hi * isz)
            s.stage(raw.data_ptr() + col * raw.element_size(), ld * raw.element_size(), arrays, byte_range=rng)
        if raw is not t:
            s.cast(raw.data_ptr(), sdt, t.data_ptr(), np.dtype(str(dtype).replace("torch.", "")), len(rows) * ld)
        s.sync()
        del raw
    return t[: len(rows)] if full else t[: len(rows), :width]


def _transport(transport, group):
    return transport or DistTransport(group)


def _native_schedule(transport, K: int, world: int) -> bool:
    """Whether the native executor runs this schedule: a native transport and no empty client block
    in the whole partition (client_blocks(K, world)).  A function of (K, world) alone, so every
    rank takes the same executor -- a rank on the native communicator and a peer on the Python
    transport would never meet."""
    return getattr(transport, "native", False) and all(k1 > k0 for k0, k1 in client_blocks(K, world))


def _python_transport(transport):
    """The transport for the Python-issued paths: a native transport (rccl.RcclTransport) hands over
    its torch.distributed counterpart for what its executor does not run (schedules with empty
    client blocks, the re-associating combines)."""
    return transport.python_transport() if getattr(transport, "native", False) else transport


def _block_layout(torch, kind: str, Kb: int, extents, tiled) -> int:
    """The tile (16-B vectors) a client block is re-tiled with, 0 for rows: ``tiled`` True/False,
    or "auto" -- where the library recommends the tile-interleaved layout for EVERY run of the
    block (its kernel for such a run walks the tiled kernel's tile)."""
    from .engine import TILED_KINDS, tiled_recommended, tiled_tile

    if tiled is False or kind not in TILED_KINDS or Kb == 0 or not extents:
        return 0
    if tiled == "auto" and not all(tiled_recommended(kind, Kb, n) for _c, n in extents):
        return 0
    return tiled_tile(kind, Kb, max(n for _c, n in extents))


def client_sharded_fedavg(parameters_updates: List[List[np.ndarray]], n_samples: Sequence[int], group=None,
                          combine: str = "relay", transport=None, rings: Optional[int] = None,
                          rounds: Optional[Sequence[float]] = None, tiled="auto",
                          chunk_elems: int = RELAY_CHUNK_ELEMS):
    """FedAvg (fed_avg.py:217-222) with the clients sharded over the process group: rank r stages
    only its blocks' buckets (to its own GPU), the chain / reduce runs over RCCL and the root
    (rank 0) returns the averaged layers; other ranks return None.  Layers must share one float
    dtype.  ``combine="relay"`` and ``"striped"`` are bit-identical to the reference
    (``striped``: ``rings`` hop lengths and ``rounds`` of :func:`lockstep.striped_pieces`);
    ``tiled``: their client blocks re-tiled per run (:class:`TiledBlock`; "auto": where the
    library recommends it, fp32 / bf16)."""
    import torch

    from .engine import fedavg_weights, kind_of, torch_dtype

    if combine not in COMBINES:
        raise ValueError(f"combine must be one of {COMBINES}")
    tr = _transport(transport, group)
    G, rank = tr.world, tr.rank
    K, L = len(parameters_updates), len(parameters_updates[0])
    dtype = _one_dtype(parameters_updates, "FedAvg")
    kind = kind_of(dtype)
    layout = BucketLayout(range(L), [a.shape for a in parameters_updates[0]], dtype)
    dev = _rank_device(torch)
    w_all = fedavg_weights(n_samples, kind)
    out = torch.empty(layout.ld, dtype=out_dtype(torch, kind), device=dev)
    if combine in ("relay", "striped"):
        plan = (striped_plan(layout.M, G, rank, rings, rounds or default_rounds(tr)) if combine == "striped"
                else relay_plan(layout.M, G, rank, chunk_elems))
        blocks = {}
        for b, segs in plan.blocks.items():
            k0, k1 = client_blocks(K, G)[b]
            rows = _stage_block(torch, dev, [parameters_updates[k] for k in range(k0, k1)], layout,
                                torch_dtype(kind), segs if combine == "striped" else None, plan.block_len[b])
            ext = TiledBlock.run_extents(plan, b)
            tv = _block_layout(torch, kind, k1 - k0, ext, tiled)
            if tv:
                rows = TiledBlock.from_rows(torch, kind, rows, tv, ext)
            blocks[b] = FedAvgShard(kind, rows, w_all[k0:k1], k0, K, plan.block_len[b], np.zeros(0, np.uint64))
        root = lockstep_fedavg(plan, blocks, out, tr, GpuShardOps(), layout.pairwise_idx)
    else:
        k0, k1 = client_blocks(K, G)[block_of(rank, G)]
        rows = _stage_block(torch, dev, [parameters_updates[k] for k in range(k0, k1)], layout, torch_dtype(kind))
        sh = FedAvgShard(kind, rows, w_all[k0:k1], k0, K, layout.M, layout.pairwise_idx)
        root = client_shard_fedavg(sh, out, tr, GpuShardOps(), combine, chunk_elems=chunk_elems)
    if not root:
        return _finish_peer(torch, tr)
    flat = out[: layout.M].cpu().numpy()
    try:
        _raise_transport_errors(tr)  # after the copy's synchronisation: a push wait that gave up is an error
    finally:
        _release_programs(tr)  # collective: the peers release in _finish_peer, error or not
    return [a for _, a in layout.unpack(np.array(flat, copy=True))]


def _finish_peer(torch, transport) -> None:
    """A non-root rank's end of a sharded call: with a transport that records failed exchanges
    (push), wait for this rank's stream and raise if any rank's wait gave up -- the call failed for
    the whole group, not only on the root.  Returns None (the result lives on the root)."""
    try:
        if getattr(transport, "raise_errors", None) is not None:
            torch.cuda.current_stream().synchronize()
            settle = getattr(transport, "settle", None)
            if settle is not None:  # this rank's part is done: did the group's call succeed?
                settle()
            _raise_transport_errors(transport)
    finally:
        _release_programs(transport)
    return None


def _release_programs(transport) -> None:
    """The host entry points stage new client blocks every call, so a compiled program never
    repeats: free it (and the peers' mappings of its buffers) before returning, so nothing of one
    aggregation stays on the GPUs into the next FL round.  Collective: root and peers both call it."""
    fn = getattr(transport, "release_programs", None)
    if fn is not None:
        fn()


def _raise_transport_errors(transport) -> None:
    """A transport's own record of a failed exchange (push.PushTransport: a wait kernel that timed
    out and let its rank go on without the data), checked once the result is synchronised."""
    fn = getattr(transport, "raise_errors", None)
    if fn is not None:
        fn()


def client_sharded_scaffold(parameters_updates, control_variate_updates, server_control_variates, n_samples,
                            aggregation_lr, group=None, combine: str = "relay", transport=None,
                            rings: Optional[int] = None, rounds: Optional[Sequence[float]] = None):
    """Scaffold (scaffold.py:193-196, 297-337) with the clients sharded over the process group.
    Every rank checks its blocks' server control variates against client 0's on the host while
    staging (``c`` itself is staged once per rank that runs a final step).  Returns
    ``(mismatches, new_server_control_variate, avg_parameters_update)`` on the root, None
    elsewhere.  fp32 or fp64 buckets (one dtype for all three lists)."""
    import torch

    from . import runtime
    from .engine import scaffold_weights, torch_dtype

    if combine not in COMBINES:
        raise ValueError(f"combine must be one of {COMBINES}")
    tr = _transport(transport, group)
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
    w_all = scaffold_weights(n_samples)
    lr = float(aggregation_lr)
    s = runtime.session(dev.index)
    c = _stage_block(torch, dev, [list(server_control_variates[0])], layout, td)[0]
    dout = torch.empty(layout.ld, dtype=torch.float64, device=dev)
    cout = torch.empty(layout.ld, dtype=torch.float64, device=dev)
    isz = np.dtype(dts[2]).itemsize
    mism = 0
    if combine == "striped":
        plan = striped_plan(layout.M, G, rank, rings, rounds or default_rounds(tr))
        blocks = {}
        for b, segs in plan.blocks.items():
            k0, k1 = client_blocks(K, G)[b]
            sel = [pu for pu in range(k0, k1)]
            delta = _stage_block(torch, dev, [parameters_updates[k] for k in sel], layout, td, segs, plan.block_len[b])
            cv = _stage_block(torch, dev, [control_variate_updates[k] for k in sel], layout, td, segs,
                              plan.block_len[b])
            check_rows = [list(server_control_variates[0])] + [list(server_control_variates[k]) for k in sel if k != 0]
            if len(check_rows) > 1:  # this block's copies of c over the elements this rank holds for it
                for lo, hi, _col in segs:
                    if hi > lo:
                        mism += s.stage_check(0, check_rows, dts[2], byte_range=(lo * isz, hi * isz))
            blocks[b] = ScaffoldShard(kind, delta, cv, None, w_all[k0:k1], k0, K, plan.block_len[b], lr,
                                      np.zeros(0, np.uint64))
        mism = tr.all_sum_int(mism)
        root = lockstep_scaffold(plan, blocks, dout, cout, tr, GpuShardOps(), layout.pairwise_idx, c, lr)
    else:
        k0, k1 = client_blocks(K, G)[block_of(rank, G)]
        delta = _stage_block(torch, dev, [parameters_updates[k] for k in range(k0, k1)], layout, td)
        cv = _stage_block(torch, dev, [control_variate_updates[k] for k in range(k0, k1)], layout, td)
        # this block's copies of c checked against client 0's on the host (pack workers)
        check_rows = [list(server_control_variates[0])] + [list(server_control_variates[k]) for k in range(k0, k1)
                                                          if k != 0]
        mism = tr.all_sum_int(s.check(check_rows, dts[2]))
        sh = ScaffoldShard(kind, delta, cv, c, w_all[k0:k1], k0, K, layout.M, lr, layout.pairwise_idx)
        root = client_shard_scaffold(sh, dout, cout, tr, GpuShardOps(), combine)
    if not root:
        return _finish_peer(torch, tr)
    d = dout[: layout.M].cpu().numpy().copy()
    cc = cout[: layout.M].cpu().numpy().copy()
    try:
        _raise_transport_errors(tr)
    finally:
        _release_programs(tr)
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
