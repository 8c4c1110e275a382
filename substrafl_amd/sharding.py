"""Multi-GPU aggregation, one process per GPU over ``torch.distributed`` (RCCL on ROCm).

Two layouts:

* **Parameter-range sharding (primary, bit-exact).**  The reduction is independent per element,
  so rank ``r`` owns elements ``[lo_r, hi_r)`` of every client's flat bucket, stages only that
  slice over its own PCIe link, and reduces it with the same kernel and the same client order as
  one GPU.  No arithmetic crosses GPUs; results are bit-identical to the single-GPU path and to
  the reference.  The optional final gather to one rank is a plain all-gather of fp32 slices
  (RCCL over xGMI), not a reduction.
* **Client sharding + reduce + final scale on rank 0 (north-star mode, NOT bit-exact).**  Rank
  ``r`` sums its contiguous block of clients, the partial sums are combined across ranks and the
  root applies the final scale.  Combining partial sums re-associates the client sum, so results
  drift from the reference by a few ulp (~34 % of elements > 2 ulp on N(0,1)
  data); the drift is measured and reported, never hidden.  ``combine="ordered"`` gathers the
  partials and adds them in rank order (deterministic); ``combine="rccl"`` uses ``dist.reduce``
  (order chosen by RCCL).

The per-shard reducer is injectable (``reducer=``): the product path uses the GPU engine; the CPU
``gloo`` tests of the distributed plumbing inject the oracle instead (tests only).
"""

from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .layout import BucketLayout

SHARD_ALIGN = 512  # elements (2 KiB of fp32): every shard starts on a 256-B boundary


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


# reducer(rows [K, n] host array of the slice, n_samples, pairwise_idx (slice-local)) -> [n] array
Reducer = Callable[[np.ndarray, Sequence[int], np.ndarray], np.ndarray]


def gpu_slice_reducer(device: Optional[int] = None) -> Reducer:
    """The product reducer: stage the slice to HBM and run libfedagg's FedAvg kernels."""

    def reduce(rows: np.ndarray, n_samples, pairwise_idx):
        import torch

        from .engine import FedAvgPlan, fedavg_weights, kind_of, torch_dtype

        kind = kind_of(rows.dtype)
        dev = torch.device("cuda", device if device is not None else torch.cuda.current_device())
        x = torch.from_numpy(np.ascontiguousarray(rows)).to(dev)
        out = torch.empty(rows.shape[1], dtype=torch_dtype(kind), device=dev)
        # rows of a [K, n] tensor are 16-B aligned only when n is a multiple of 4: the library
        # checks every pointer and takes its scalar path otherwise
        FedAvgPlan(kind, x, fedavg_weights(n_samples, kind), rows.shape[1], out, pairwise_idx).launch()
        torch.cuda.synchronize(dev)
        return out.cpu().numpy()

    return reduce


def param_range_fedavg(
    parameters_updates: List[List[np.ndarray]],
    n_samples: Sequence[int],
    group=None,
    reducer: Optional[Reducer] = None,
    gather: bool = True,
):
    """FedAvg over a process group with parameter-range sharding (bit-exact).

    Every rank passes the same host shared states (as every rank of a node would read the same
    task inputs); rank ``r`` reduces only its slice.  With ``gather=True`` every rank returns the
    full list of averaged layers (all-gather of slices); otherwise ``(lo, hi, slice)``.
    Layers must share one floating dtype (the single-GPU engine handles mixed dtypes)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    L = len(parameters_updates[0])
    dtype = np.result_type(*[np.result_type(a.dtype, 1.0) for a in parameters_updates[0]])
    layout = BucketLayout(range(L), [a.shape for a in parameters_updates[0]], dtype)
    bounds = shard_bounds(layout.M, world)
    lo, hi = bounds[rank]
    K = len(parameters_updates)
    rows = np.zeros((K, max(1, hi - lo)), dtype=dtype)
    for k in range(K):
        pack_range(layout, parameters_updates[k], rows[k], lo, hi)
    pw = layout.pairwise_idx.astype(np.int64)
    pw_local = (pw[(pw >= lo) & (pw < hi)] - lo).astype(np.uint64)
    red = reducer or gpu_slice_reducer()
    part = red(rows[:, : hi - lo], n_samples, pw_local) if hi > lo else np.zeros(0, dtype)
    if not gather:
        return lo, hi, part
    chunk = bounds[0][1] - bounds[0][0]
    backend = dist.get_backend(group)
    on_gpu = backend == "nccl"
    tdev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    send = torch.zeros(chunk, dtype=torch.from_numpy(np.zeros(0, dtype)).dtype, device=tdev)
    send[: hi - lo] = torch.from_numpy(np.ascontiguousarray(part)).to(tdev)
    recv = torch.empty(chunk * world, dtype=send.dtype, device=tdev)
    dist.all_gather_into_tensor(recv, send, group=group)
    flat = recv[: layout.M].cpu().numpy()
    return [a for _, a in layout.unpack(np.array(flat, copy=True))]


def client_sharded_fedavg(
    parameters_updates: List[List[np.ndarray]],
    n_samples: Sequence[int],
    group=None,
    reducer: Optional[Reducer] = None,
    combine: str = "ordered",
    root: int = 0,
):
    """North-star mode: contiguous client blocks per rank, partial sums combined on ``root``
    (NOT bit-exact with the reference; see module docstring).  Returns the averaged layers on
    ``root`` and ``None`` elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    K = len(parameters_updates)
    L = len(parameters_updates[0])
    dtype = np.result_type(*[np.result_type(a.dtype, 1.0) for a in parameters_updates[0]])
    layout = BucketLayout(range(L), [a.shape for a in parameters_updates[0]], dtype)
    per = -(-K // world)
    mine = list(range(rank * per, min(K, (rank + 1) * per)))
    n_all = sum(int(n) for n in n_samples)
    # each rank's weights are the GLOBAL weights fl(n_k / n) of its clients; the final scale is 1
    # for FedAvg (weights are pre-normalised) -- Scaffold would apply aggregation_lr here.
    rows = np.zeros((max(1, len(mine)), layout.M), dtype=dtype)
    for j, k in enumerate(mine):
        layout.pack_row(parameters_updates[k], rows[j])
    red = reducer or gpu_slice_reducer()
    if mine:
        # the reducer normalises by the sum of the n it gets: pass n_k scaled so that its
        # weights equal the global fl(n_k / n) -- done by giving it the global weights directly
        part = _weighted_partial(red, rows[: len(mine)], [n_samples[k] for k in mine], n_all, layout)
    else:
        part = np.zeros(layout.M, dtype)
    backend = dist.get_backend(group)
    tdev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.from_numpy(np.ascontiguousarray(part)).to(tdev)
    if combine == "rccl":
        dist.reduce(t, dst=root, op=dist.ReduceOp.SUM, group=group)
        total = t.cpu().numpy() if rank == root else None
    elif combine == "ordered":
        gathered = [torch.empty_like(t) for _ in range(world)] if rank == root else None
        dist.gather(t, gather_list=gathered, dst=root, group=group)
        if rank == root:
            total = gathered[0].cpu().numpy().copy()
            for g in gathered[1:]:
                total = (total + g.cpu().numpy()).astype(dtype)
        else:
            total = None
    else:
        raise ValueError(combine)
    if rank != root:
        return None
    return [a for _, a in layout.unpack(total)]


def _weighted_partial(red: Reducer, rows, local_n, n_all, layout):
    # A reducer computes weights from the n_samples it is given (fl(n_k / sum)).  To get the
    # global weights fl(n_k / n_all) we append a virtual zero-row client carrying the remaining
    # samples: its products are exactly 0 and do not change any partial sum (x + 0 == x).
    rest = n_all - sum(int(n) for n in local_n)
    if rest:
        rows = np.concatenate([rows, np.zeros((1, rows.shape[1]), rows.dtype)], axis=0)
        local_n = list(local_n) + [rest]
    return red(rows, local_n, layout.pairwise_idx)
