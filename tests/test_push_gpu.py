"""Push executor (substrafl_amd/push.py, fedagg_push_execute): G rank PROCESSES on the one GPU
(IPC-mapped slots between processes, the node-shared progress page, gloo for the set-up), each
running its part of a relay / striped FedAvg schedule three times through the cached program;
the root's result bit-identical to the reference (fed_avg.py:217-222).  On the 8-GPU node the
same protocol crosses xGMI (bench.py's client_shard_push leg)."""

from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

# (G, K, rounds, relay, shapes[, kind])
# (the relay case once gave the numel == 1 elements only the root's products in the second of
# three calls, while the root's staging sum was a torch reduction between the executor and the
# pairwise finish (tools/push_tail_probe.py); the sum and the landing copies run
# inside the executor since, so no torch op sits between libfedagg launches on this path)
CASES = [
    (2, 5, (1.0,), False, "default"),
    (3, 7, (0.5, 0.3, 0.2), False, "default"),
    (4, 9, (0.75, 0.25), True, "default"),
    (3, 40, (0.5, 0.5), False, "wide"),
    (3, 7, (0.5, 0.5), False, "default", "bf16"),  # C5's kind: bf16 buckets, fp32 accumulators
    (4, 9, (0.75, 0.25), True, "default", "bf16"),
]
CASES = [c if len(c) == 6 else c + ("f32",) for c in CASES]
CASES = [c + ("fedavg",) for c in CASES] + [
    # Scaffold: two fp64 accumulators per element, each run two launches (delta, control variate)
    (3, 7, (0.5, 0.3, 0.2), False, "default", "f32", "scaffold"),
    (4, 9, (0.75, 0.25), True, "default", "f32", "scaffold"),
    (2, 5, (1.0,), False, "wide", "f64", "scaffold"),
    # ragged: the ranks' slot sizes differ (root 512, the others 1024 elements per slot), so a
    # producer must address a consumer's slots with the CONSUMER's slot size
    (4, 9, (0.5, 0.3, 0.2), False, "ragged", "f32", "fedavg"),
    (4, 6, (0.5, 0.3, 0.2), False, "ragged", "f32", "scaffold"),
]
SHAPE_SETS = {"wide": [(1,), (130001,), (1, 1), (77777,)], "ragged": [(4097,), (1,), (1, 1)],
              "c4": [(24_999_998,), (1,), (1, 1)]}  # BASELINE's C4 bucket: 25M parameters


def _random_cases(n, seed=31):
    """Seeded random schedules (2-4 rank processes share the one GPU): plan, sizes, strategy, kind."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        G = int(rng.integers(2, 5))
        scaffold = i % 2 == 1
        kind = ("f32", "f64")[int(rng.integers(0, 2))] if scaffold else ("f32", "bf16")[int(rng.integers(0, 2))]
        rounds = [(1.0,), (0.75, 0.25), (0.5, 0.3, 0.2)][int(rng.integers(0, 3))]
        out.append((G, G + int(rng.integers(0, 6)), rounds, bool(rng.random() < 0.3), f"rand{int(rng.integers(1 << 20))}",
                    kind, "scaffold" if scaffold else "fedavg"))
    return out


def _shapes(name):
    if name in SHAPE_SETS:
        return SHAPE_SETS[name]
    rng = np.random.default_rng(int(name[4:]))  # "rand<seed>": ragged layers around numel == 1 ones
    shapes = [(int(rng.integers(1, 40_000)),) for _ in range(int(rng.integers(1, 4)))] + [(1,), (1, 1)]
    rng.shuffle(shapes)
    return shapes


CASES += _random_cases(6)
CASES.append((2, 16, (1.0,), False, "c4", "f32", "scaffold"))  # C4 (16 x 25M) over two rank processes


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, G, K, rounds, relay, shapes_name, kind, strategy, port, q):
    import faulthandler

    faulthandler.dump_traceback_later(100, exit=True)
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from datetime import timedelta

    import torch
    import torch.distributed as dist

    from oracle import fedavg_reference_structure, scaffold_reference_structure
    from substrafl_amd.engine import fedavg_weights, scaffold_weights
    from substrafl_amd.layout import BucketLayout
    from substrafl_amd.push import PushTransport
    from substrafl_amd.sharding import (SLOTS, FedAvgShard, GpuShardOps, ScaffoldShard, client_blocks,
                                        lockstep_fedavg, lockstep_scaffold, relay_plan, striped_plan)
    from test_client_shard_gpu import SHAPES, _data, _rows

    try:
        dist.init_process_group("gloo", rank=rank, world_size=G, timeout=timedelta(seconds=90))
        torch.cuda.set_device(0)
        shapes = SHAPES + [(5000,), (1,)] if shapes_name == "default" else _shapes(shapes_name)
        scaffold = strategy == "scaffold"
        npdt = np.float64 if kind == "f64" else np.float32
        pus, ns = _data(K, seed=17 + G, shapes=shapes)
        pus = [[a.astype(npdt) for a in c] for c in pus]
        if kind == "bf16":  # bf16-representable values: the reference runs on the exact upcast
            pus = [[(a.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32) for a in c] for c in pus]
        rng = np.random.default_rng(5 + G)
        cvs = [[rng.standard_normal(a.shape).astype(npdt) for a in pu] for pu in pus]
        c = [rng.standard_normal(a.shape).astype(npdt) for a in pus[0]]
        lr = 0.7
        layout = BucketLayout(range(len(shapes)), shapes, npdt)
        plan = relay_plan(layout.M, G, rank, 4096) if relay else striped_plan(layout.M, G, rank, None, rounds)
        tdt = torch.bfloat16 if kind == "bf16" else (torch.float64 if kind == "f64" else torch.float32)

        def packed(lists, b, segs):
            k0, k1 = client_blocks(K, G)[b]
            full = _rows(torch, lists[k0:k1], layout, dtype=npdt, tdtype=tdt)
            t = torch.zeros((k1 - k0, plan.block_len[b]), dtype=tdt, device="cuda")
            for lo, hi, col in segs:
                t[:, col: col + hi - lo] = full[:, lo:hi]
            return t

        blocks = {}
        for b, segs in plan.blocks.items():
            k0, k1 = client_blocks(K, G)[b]
            if scaffold:
                blocks[b] = ScaffoldShard(kind, packed(pus, b, segs), packed(cvs, b, segs), None,
                                          scaffold_weights(ns)[k0:k1], k0, K, plan.block_len[b], lr,
                                          np.zeros(0, np.uint64))
            else:
                blocks[b] = FedAvgShard(kind, packed(pus, b, segs), fedavg_weights(ns, kind)[k0:k1], k0, K,
                                        plan.block_len[b], np.zeros(0, np.uint64))
        tr = PushTransport(timeout_s=30)
        bad, calls = [], 0
        ref = None
        if rank == plan.root:
            if scaffold:
                rc, ra = scaffold_reference_structure(pus, cvs, c, ns, lr)
                ref = ra + rc  # the averaged update, then the new server control variate
            else:
                ref = fedavg_reference_structure(pus, ns)
        odt = torch.float64 if scaffold else torch.float32
        outs = [torch.empty((layout.ld,), dtype=odt, device="cuda") for _ in range(2 if scaffold else 1)]
        slots = torch.empty((2 if scaffold else 1) * SLOTS * max(1, plan.slot_elems), dtype=odt, device="cuda")
        full_c = _rows(torch, [c], layout, dtype=npdt)[0] if scaffold else None
        lay_out = BucketLayout(range(len(shapes)), shapes, np.float64 if scaffold else np.float32)
        ubits = np.uint64 if scaffold else np.uint32
        held = []
        for call in range(3):  # the cached program, and counters that keep climbing across calls
            if call == 2:  # fresh outputs at new addresses (the old ones held): the program is reused, rebased
                held.append(outs)
                outs = [torch.empty_like(o) for o in outs]
            for o in outs:
                o.fill_(float("nan"))
            if scaffold:
                is_root = lockstep_scaffold(plan, blocks, outs[0], outs[1], tr, GpuShardOps(), layout.pairwise_idx,
                                            full_c, lr, slots=slots)
            else:
                is_root = lockstep_fedavg(plan, blocks, outs[0], tr, GpuShardOps(), layout.pairwise_idx, slots=slots)
            torch.cuda.synchronize()
            calls += 1
            if is_root:
                got = [a for o in outs for _, a in lay_out.unpack(o[: layout.M].cpu().numpy())]
                nb = sum(int(np.count_nonzero(g.view(ubits) != r.view(ubits))) for g, r in zip(got, ref))
                if nb and os.environ.get("PUSH_DEBUG"):
                    print(f"[push debug] call {calls}: " + "; ".join(
                        f"layer {i} {g.shape}: idx {np.nonzero(g.reshape(-1).view(ubits) != r.reshape(-1).view(ubits))[0][:4]} "
                        f"got {g.reshape(-1)[np.nonzero(g.reshape(-1).view(ubits) != r.reshape(-1).view(ubits))[0][:2]]} "
                        f"ref {r.reshape(-1)[np.nonzero(g.reshape(-1).view(ubits) != r.reshape(-1).view(ubits))[0][:2]]}"
                        for i, (g, r) in enumerate(zip(got, ref)) if np.any(g.view(ubits) != r.view(ubits))),
                        file=sys.stderr, flush=True)
                bad.append(nb)
        errs = tr.errors()
        programs = len(tr._programs)
        prog = tr._programs[0]
        # every rank writes landing tags (at least the root's staging tag) and the root waits for them
        assert prog.ntags > 0 if rank != plan.root else sum(1 for w in prog.tag_waits) > 0, (rank, prog.ntags)
        print(f"[push] rank {rank}: late landing tags {tr.late_tags()[rank]}", file=sys.stderr, flush=True)
        tr.close()
        dist.destroy_process_group()
        q.put((rank, bad, errs, programs, calls, None))
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        import traceback

        q.put((rank, None, None, 0, 0, traceback.format_exc()[-2000:]))


@pytest.mark.parametrize("G,K,rounds,relay,shapes,kind,strategy", CASES)
def test_push_executor_processes_bit_exact(G, K, rounds, relay, shapes, kind, strategy):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, G, K, rounds, relay, shapes, kind, strategy, port, q))
             for r in range(G)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(G):
            rank, bad, errs, programs, calls, tb = q.get(timeout=110)
            res[rank] = (bad, errs, programs, calls, tb)
    finally:
        for p in procs:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()  # our own child, by handle
    for rank, (bad, errs, programs, calls, tb) in sorted(res.items()):
        assert tb is None, f"rank {rank}:\n{tb}"
        assert errs == {} and programs == 1 and calls == 3, (rank, errs, programs, calls, bad)
    assert res[0][0] == [0, 0, 0], res[0][0]  # root: every element, every call


@pytest.mark.parametrize("kind", ["f32", "bf16"])
@pytest.mark.parametrize("K,M", [(9, 4096 * 3 + 5), (65, 2_000_000), (130, 70_001)])
def test_push_run_continues_its_input_accumulator(kind, K, M):
    """fedagg_fedavg_chain_push_{f32,bf16} (one process): d_in continued by the block's clients into
    a separate d_out, bit-identical to the chain kernel continuing the same accumulator in place;
    d_in NULL is the chain from +0.0.  Also across client chunks (K > 128) and element remainders."""
    import ctypes

    import torch

    from substrafl_amd import _native
    from substrafl_amd.engine import fedavg_weights

    lib = _native.load()
    torch.manual_seed(K + M)
    tdt = torch.bfloat16 if kind == "bf16" else torch.float32
    rows = torch.randn((K, M), dtype=torch.float32, device="cuda").to(tdt)
    w = (ctypes.c_float * K)(*[float(v) for v in fedavg_weights(list(range(1, K + 1)), "f32")])
    ptrs = _native.ptr_array([rows[k].data_ptr() for k in range(K)])
    acc_in = torch.randn(M, dtype=torch.float32, device="cuda")
    chain = getattr(lib, f"fedagg_fedavg_chain_{kind}")
    push = getattr(lib, f"fedagg_fedavg_chain_push_{kind}")
    s = torch.cuda.current_stream().cuda_stream
    ref = acc_in.clone()
    _native.check(chain(ptrs, w, K, M, 0, ref.data_ptr(), s), "chain")
    out = torch.full((M,), float("nan"), device="cuda")
    _native.check(push(ptrs, w, K, M, acc_in.data_ptr(), out.data_ptr(), s), "chain_push")
    ref0 = torch.empty(M, device="cuda")
    _native.check(chain(ptrs, w, K, M, 1, ref0.data_ptr(), s), "chain seed")
    out0 = torch.full((M,), float("nan"), device="cuda")
    _native.check(push(ptrs, w, K, M, None, out0.data_ptr(), s), "chain_push seed")
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    assert torch.equal(out0.view(torch.int32), ref0.view(torch.int32))


@pytest.mark.parametrize("kind", ["f32", "f64"])
@pytest.mark.parametrize("K,M,finish", [(9, 4096 * 3 + 5, True), (70, 1_000_003, False), (5, 77_777, True)])
def test_scaffold_push_run_continues_its_input_accumulator(kind, K, M, finish):
    """fedagg_scaffold_chain_push_{f32,f64} (one process): per bucket, d_in continued by the block's
    rows into a separate d_out (x lr / + c at the finish), bit-identical to fedagg_scaffold_chain_*
    continuing the same two accumulators in place; d_in NULL is the chain from +0.0.  Also across
    client chunks (K > 64) and element remainders."""
    import ctypes

    import torch

    from substrafl_amd import _native
    from substrafl_amd.engine import scaffold_weights

    lib = _native.load()
    torch.manual_seed(K + M)
    tdt = torch.float64 if kind == "f64" else torch.float32
    delta = torch.randn((K, M), dtype=tdt, device="cuda")
    cv = torch.randn((K, M), dtype=tdt, device="cuda")
    c = torch.randn(M, dtype=tdt, device="cuda")
    lr = 0.3
    w = (ctypes.c_double * K)(*[float(v) for v in scaffold_weights(list(range(3, K + 3)))])
    dp = _native.ptr_array([delta[k].data_ptr() for k in range(K)])
    cp = _native.ptr_array([cv[k].data_ptr() for k in range(K)])
    chain = getattr(lib, f"fedagg_scaffold_chain_{kind}")
    push = getattr(lib, f"fedagg_scaffold_chain_push_{kind}")
    s = torch.cuda.current_stream().cuda_stream
    for seed in (False, True):
        d_in = torch.randn(M, dtype=torch.float64, device="cuda")
        c_in = torch.randn(M, dtype=torch.float64, device="cuda")
        ref_d, ref_c = d_in.clone(), c_in.clone()
        _native.check(chain(dp, cp, c.data_ptr(), w, K, M, int(seed), int(finish), lr, ref_d.data_ptr(),
                            ref_c.data_ptr(), s), "chain")
        got = []
        for ph, (rows, acc_in) in enumerate(((dp, d_in), (cp, c_in))):
            out = torch.full((M,), float("nan"), dtype=torch.float64, device="cuda")
            _native.check(push(rows, w, K, M, ph, c.data_ptr(), lr, int(finish), None if seed else acc_in.data_ptr(),
                               out.data_ptr(), s), "chain_push")
            got.append(out)
        torch.cuda.synchronize()
        assert torch.equal(got[0].view(torch.int64), ref_d.view(torch.int64)), (seed, "delta")
        assert torch.equal(got[1].view(torch.int64), ref_c.view(torch.int64)), (seed, "control variate")


# ---------------------------------------------------------------------------- the failure path
FAULT_TIMEOUT_S = 3.0
FAULT_SHAPES = [(37, 29), (1,), (3_000_000,), (1, 1)]  # 2-3 relay chunks: several steps


def _fault_worker(rank, G, K, fault, strategy, port, q):
    """One rank of a client-sharded call through a PushTransport with ``fault`` injected (on rank
    ``fault[1]``); reports (rank, error text or None, returned a result, seconds, errors(), tb)."""
    import faulthandler
    import time

    faulthandler.dump_traceback_later(100, exit=True)
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from datetime import timedelta

    import torch
    import torch.distributed as dist

    from substrafl_amd._native import NativeLibraryError
    from substrafl_amd.push import PushTransport
    from substrafl_amd.sharding import client_sharded_fedavg, client_sharded_scaffold
    from test_client_shard_gpu import _data

    tr = None
    try:
        dist.init_process_group("gloo", rank=rank, world_size=G, timeout=timedelta(seconds=90))
        torch.cuda.set_device(0)
        pus, ns = _data(K, seed=3, shapes=FAULT_SHAPES)
        tr = PushTransport(timeout_s=FAULT_TIMEOUT_S, fault=fault)
        t0 = time.perf_counter()
        err, res = None, None
        try:
            if strategy == "scaffold":
                rng = np.random.default_rng(9)
                cvs = [[rng.standard_normal(a.shape).astype(np.float32) for a in pu] for pu in pus]
                c = [rng.standard_normal(a.shape).astype(np.float32) for a in pus[0]]
                res = client_sharded_scaffold(pus, cvs, [c] * K, ns, 0.7, transport=tr)
            else:
                res = client_sharded_fedavg(pus, ns, transport=tr, chunk_elems=1 << 20)
        except NativeLibraryError as e:
            err = str(e)
        torch.cuda.synchronize()
        q.put((rank, err, res is not None, time.perf_counter() - t0, tr.errors(), None))
    except Exception:  # noqa: BLE001 -- reported to the parent
        import traceback

        q.put((rank, None, False, 0.0, None, traceback.format_exc()[-2000:]))
    finally:
        if tr is not None:
            tr.close()
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("strategy", ["fedavg", "scaffold"])
@pytest.mark.parametrize("fault,expect", [(("signal", 1, 1), "counter of rank 1"),
                                          (("exit", 1, 1), "counter of rank 1"),
                                          (("tag", 1, 0), "landing tag of rank 1")])
def test_push_executor_fails_cleanly(fault, expect, strategy):
    """VERDICT r04 "Next 3": a rank that withholds its step signal (a peer stuck mid-call), whose
    process exits mid-call without releasing anything (a peer that died), or that
    withholds one landing tag makes the ROOT's client_sharded_* raise, naming the counter or the
    tag, within about one timeout (every other wait gives up on the first failure instead of
    timing out in turn; no collective runs after the failure, so the dead peer costs no backend
    timeout); the root's output is never returned; every process exits."""
    import torch.multiprocessing as mp

    from substrafl_amd.push import FAULT_EXIT_CODE

    G, K = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_fault_worker, args=(r, G, K, fault, strategy, port, q)) for r in range(G)]
    for p in procs:
        p.start()
    res = {}
    dead = {fault[1]} if fault[0] == "exit" else set()  # the rank that dies reports nothing
    try:
        for _ in range(G - len(dead)):
            rank, err, returned, secs, errs, tb = q.get(timeout=110)
            res[rank] = (err, returned, secs, errs, tb)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()  # our own child, by handle
    assert all(not p.is_alive() for p in procs)
    for r in dead:
        assert procs[r].exitcode == FAULT_EXIT_CODE, procs[r].exitcode
    for rank, (err, returned, secs, errs, tb) in sorted(res.items()):
        assert tb is None, f"rank {rank}:\n{tb}"
    err, returned, secs, errs, _ = res[0]
    assert err is not None and "a wait timed out" in err and expect in err, res[0]
    assert not returned  # the root's output never comes back as a result
    assert errs and expect in errs[0], errs
    assert secs < FAULT_TIMEOUT_S + 15, secs  # one timeout, not one per wait
    print(f"[push fault] {fault} {strategy}: root raised after {secs:.2f} s: {err}", file=sys.stderr)


def _memory_worker(rank, G, K, strategy, calls, port, q):
    """Repeated host-entry calls through one PushTransport (new client blocks every call, as in an
    FL run): reports per call the programs / peer mappings held after it and the device's free
    memory."""
    import faulthandler

    faulthandler.dump_traceback_later(100, exit=True)
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from datetime import timedelta

    import torch
    import torch.distributed as dist

    from substrafl_amd import runtime
    from substrafl_amd.push import PushTransport
    from substrafl_amd.sharding import client_sharded_fedavg, client_sharded_scaffold
    from test_client_shard_gpu import _data

    tr = None
    try:
        dist.init_process_group("gloo", rank=rank, world_size=G, timeout=timedelta(seconds=90))
        torch.cuda.set_device(0)
        tr = PushTransport(timeout_s=30)
        rec = []
        for i in range(calls):
            pus, ns = _data(K, seed=40 + i, shapes=FAULT_SHAPES)
            if strategy == "scaffold":
                rng = np.random.default_rng(i)
                cvs = [[rng.standard_normal(a.shape).astype(np.float32) for a in pu] for pu in pus]
                c = [rng.standard_normal(a.shape).astype(np.float32) for a in pus[0]]
                client_sharded_scaffold(pus, cvs, [c] * K, ns, 0.7, transport=tr)
            else:
                client_sharded_fedavg(pus, ns, transport=tr, chunk_elems=1 << 20)
            torch.cuda.synchronize()
            dist.barrier()
            rec.append((len(tr._programs), len(tr._maps), runtime.device_memory(0)[0]))
        q.put((rank, rec, None))
    except Exception:  # noqa: BLE001 -- reported to the parent
        import traceback

        q.put((rank, None, traceback.format_exc()[-2000:]))
    finally:
        if tr is not None:
            tr.close()
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("strategy", ["scaffold", "fedavg"])
def test_repeated_host_calls_keep_memory_flat(strategy):
    """client_sharded_* stage new blocks every call, so the push program never repeats;
    each call releases its program (uncached buffers, the peers' IPC mappings of them) before it
    returns, and the device's free memory stays flat over repeated calls."""
    import torch.multiprocessing as mp

    G, K, calls = 2, 6, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_memory_worker, args=(r, G, K, strategy, calls, port, q)) for r in range(G)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(G):
            rank, rec, tb = q.get(timeout=110)
            res[rank] = (rec, tb)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()  # our own child, by handle
    for rank, (rec, tb) in sorted(res.items()):
        assert tb is None, f"rank {rank}:\n{tb}"
        assert all(n_prog == 0 and n_maps == 0 for n_prog, n_maps, _f in rec), rec
        free = [f for _p, _m, f in rec]
        # from the second call on (torch's caching allocator holds the staged blocks' memory for reuse)
        assert min(free[1:]) >= free[1] - (64 << 20), [f >> 20 for f in free]
    print(f"[push memory] {strategy}: free MiB per call {[f >> 20 for _p, _m, f in res[0][0]]}", file=sys.stderr)
