"""Bisect of the round-3 push-executor failure (relay, G = 4, K = 9, second of three calls: the
root's numel == 1 outputs held only part of the products; gpurun_out/push_dbg3.log).

Until 8f2eb26 the root's tail ran AFTER fedagg_push_execute, on the same stream:
    fedagg_copy_async(stage_t <- stage_u)          a runtime hipMemcpyAsync (device to device) out
                                                   of the uncached staging rows the peers wrote
    with torch.cuda.stream(ExternalStream(s)):
        ws.copy_(stage_t.view(G, P, K).sum(0))     a torch reduction, then torch's copy_ (another
                                                   runtime device-to-device copy) into ws
Since then a kernel sums the staging rows into ws inside the executor.  (Run on the ABI-12
library of round 3, profiles/r04_push_tail*.jsonl; it passes the landing tags of ABI 13 through.)  This probe runs the
relay case with each combination of those mechanisms on the product kernels and records, per
call, the root's numel == 1 result against the reference AND, after a full synchronize, what the
staging rows hold against what the tail read from them -- so a stale read, a late write and a
copy that raced the sum can be told apart:

    kernel   the product: the executor's own stage-sum kernel
    legacy   hipMemcpyAsync out of the staging rows, torch sum, torch copy_       (round-3 code)
    kcopy    a KERNEL copy out of the staging rows (fedagg_flat_gather_f32), torch sum, torch copy_
    tcopyk   hipMemcpyAsync out of the staging rows, torch sum, KERNEL copy into ws

    python3 tools/push_tail_probe.py --modes kernel,legacy,kcopy,tcopyk --reps 3

One GPU: the G ranks are processes on it (IPC-mapped staging rows, as in tests/test_push_gpu.py).
Prints one JSON line per (mode, repetition).
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# fedagg_copy_async (the "legacy" / "tcopyk" modes) is exported by the FEDAGG_TUNING build only
os.environ.setdefault("FEDAGG_LIB", os.path.join(ROOT, "substrafl_amd", "libfedagg_tuning.so"))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, G, K, mode, calls, port, q):
    import faulthandler

    faulthandler.dump_traceback_later(100, exit=True)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from datetime import timedelta

    import torch
    import torch.distributed as dist

    from substrafl_amd import _native
    from substrafl_amd.engine import fedavg_weights
    from substrafl_amd.layout import BucketLayout
    from substrafl_amd.push import PushTransport, _check
    from substrafl_amd.sharding import SLOTS, FedAvgShard, GpuShardOps, client_blocks, lockstep_fedavg, relay_plan
    from test_client_shard_gpu import SHAPES, _data, _rows

    try:
        dist.init_process_group("gloo", rank=rank, world_size=G, timeout=timedelta(seconds=90))
        torch.cuda.set_device(0)
        shapes = SHAPES + [(5000,), (1,)]
        pus, ns = _data(K, seed=17 + G, shapes=shapes)
        pus = [[a.astype(np.float32) for a in c] for c in pus]
        layout = BucketLayout(range(len(shapes)), shapes, np.float32)
        plan = relay_plan(layout.M, G, rank, 4096)
        blocks = {}
        for b, segs in plan.blocks.items():
            k0, k1 = client_blocks(K, G)[b]
            full = _rows(torch, pus[k0:k1], layout, dtype=np.float32)
            t = torch.zeros((k1 - k0, plan.block_len[b]), dtype=torch.float32, device="cuda")
            for lo, hi, col in segs:
                t[:, col: col + hi - lo] = full[:, lo:hi]
            blocks[b] = FedAvgShard("f32", t, fedavg_weights(ns, "f32")[k0:k1], k0, K, plan.block_len[b],
                                    np.zeros(0, np.uint64))
        tr = PushTransport(timeout_s=30)
        lib = _native.load()
        diag = []
        diag_streams = []
        snaps = {k: torch.full((4096,), float("nan"), device="cuda") for k in ("tmp", "ws", "ws_fin", "out_fin")}

        def snap(dst, t):  # a stream-ordered kernel copy of t, taken where the tail stands
            cnt = (ctypes.c_uint64 * 1)(t.numel())
            _check(lib.fedagg_flat_gather_f32(_native.ptr_array([t.data_ptr()]), cnt, 1, dst.data_ptr(),
                                              int(torch.cuda.current_stream().cuda_stream)), "snap")

        if mode != "kernel":
            def execute(prog, stream, ws=None, ws_kind="f32"):
                """PushTransport.execute without the in-executor tail, then the round-3 tail."""
                ws_bytes = ws.numel() * ws.element_size() if ws is not None else 0
                ws_src, ws_dst = (ws.data_ptr(), prog.ws_dst(ws_bytes)) if ws_bytes else (None, None)
                root = tr.rank == prog.plan.root
                _check(lib.fedagg_push_execute(ctypes.byref(prog.runs) if prog.nruns else None, prog.nruns,
                                               ctypes.byref(prog.waits) if prog.nwaits else None, prog.nwaits,
                                               ctypes.byref(prog.tags) if prog.ntags else None, prog.ntags,
                                               prog.nsteps, tr._dev, tr.rank, tr.world, tr.base, tr._timeout,
                                               ws_src, ws_dst, ws_bytes, _native.FEDAGG_F32, None, None, 0,
                                               tr._aux_ptrs, len(tr._aux), int(stream)), "fedagg_push_execute")
                tr.base += prog.nsteps + 1
                if not root:
                    return

                def copy(dst, src, nbytes):  # the mode's device-to-device copy
                    if mode.startswith("legacy") or mode == "tcopyk":
                        _check(lib.fedagg_copy_async(dst, src, nbytes, int(stream)), "fedagg_copy_async")
                    else:
                        cnt = (ctypes.c_uint64 * 1)(nbytes // 4)
                        _check(lib.fedagg_flat_gather_f32(_native.ptr_array([src]), cnt, 1, dst, int(stream)),
                               "fedagg_flat_gather_f32")

                out_t = prog.outs[0]
                for lo, hi in prog.land_ranges:  # the landed pieces into the output (round 3: land_to_out)
                    copy(out_t.data_ptr() + lo * 4, prog.land_u.ptr + lo * 4, (hi - lo) * 4)
                if not ws_bytes:
                    return
                if not hasattr(prog, "stage_t"):
                    prog.stage_t = torch.empty(tr.world * ws_bytes // 4, dtype=torch.float32, device=ws.device)
                copy(prog.stage_t.data_ptr(), prog.stage_u.ptr, tr.world * ws_bytes)
                if mode == "legacy_sync":
                    torch.cuda.synchronize()
                import contextlib

                ctxm = contextlib.nullcontext() if mode == "legacy_noctx" else \
                    torch.cuda.stream(torch.cuda.ExternalStream(int(stream)))
                with ctxm:
                    tmp = prog.stage_t.view(tr.world, *ws.shape).sum(0)
                    snap(snaps["tmp"], tmp)
                    if mode == "tcopyk":
                        src = _native.ptr_array([tmp.data_ptr()])
                        cnt = (ctypes.c_uint64 * 1)(tmp.numel())
                        _check(lib.fedagg_flat_gather_f32(src, cnt, 1, ws.data_ptr(), int(stream)),
                               "fedagg_flat_gather_f32")
                    else:
                        ws.copy_(tmp)
                    snap(snaps["ws"], ws)
                if mode == "legacy_sync":
                    torch.cuda.synchronize()
                diag_streams.append([int(stream), int(torch.cuda.current_stream().cuda_stream),
                                     tmp.data_ptr() == ws.data_ptr()])

            tr.execute = execute

        ops = GpuShardOps()
        finish0 = ops.fedavg_finish

        def finish(kind, ws, K_, pairwise_idx, out_):  # ws as the finish reads it, out as it leaves it
            snap(snaps["ws_fin"], ws)
            finish0(kind, ws, K_, pairwise_idx, out_)
            for j, e in enumerate(np.asarray(pairwise_idx, np.int64)):
                snap(snaps["out_fin"][j:], out_[int(e): int(e) + 1])

        ops.fedavg_finish = finish
        # the reference's own expression (fed_avg.py:217-222): per layer, np.sum of the weighted list
        total = sum(int(n) for n in ns)
        ref = [np.sum([c[i] * (int(n) / total) for c, n in zip(pus, ns)], axis=0)
               for i in range(len(shapes))] if rank == plan.root else None
        out = torch.empty((layout.ld,), dtype=torch.float32, device="cuda")
        slots = torch.empty(SLOTS * max(1, plan.slot_elems), dtype=torch.float32, device="cuda")
        bad = []
        for call in range(calls):
            out.fill_(float("nan"))
            for v in snaps.values():
                v.fill_(float("nan"))
            is_root = lockstep_fedavg(plan, blocks, out, tr, ops, layout.pairwise_idx, slots=slots)
            torch.cuda.synchronize()
            if is_root:
                got = [a for _, a in layout.unpack(out[: layout.M].cpu().numpy())]
                nb = sum(int(np.count_nonzero(g.view(np.uint32) != r.view(np.uint32))) for g, r in zip(got, ref))
                bad.append(nb)
                prog = tr._programs[0]
                rec = {"call": call + 1, "wrong_elements": nb}
                if prog.stage_u is not None:  # what the staging rows hold now (every peer done)
                    now = np.empty(prog.stage_u.bytes // 4, np.float32)
                    lib_hip = torch.empty(now.size, dtype=torch.float32, device="cuda")
                    src = _native.ptr_array([prog.stage_u.ptr])
                    cnt = (ctypes.c_uint64 * 1)(now.size)
                    _check(lib.fedagg_flat_gather_f32(src, cnt, 1, lib_hip.data_ptr(), 0), "gather")
                    torch.cuda.synchronize()
                    now = lib_hip.cpu().numpy().reshape(G, -1)
                    if hasattr(prog, "stage_t"):  # what the tail read, and what it computed from it
                        full = now.sum(0)
                        nws = full.size
                        rec["tmp_snapshot_wrong"] = int(np.count_nonzero(
                            snaps["tmp"][:nws].cpu().numpy().view(np.uint32) != full.view(np.uint32)))
                        rec["ws_snapshot_wrong"] = int(np.count_nonzero(
                            snaps["ws"][:nws].cpu().numpy().view(np.uint32) != full.view(np.uint32)))
                        rec["streams"] = diag_streams[-1] if diag_streams else None
                        read = prog.stage_t.cpu().numpy().reshape(G, -1)
                        rec["rows_read_stale"] = [int(np.count_nonzero(read[r].view(np.uint32) != now[r].view(np.uint32)))
                                                  for r in range(G)]
                        rec["rows_read_zero"] = [int(np.count_nonzero((read[r] == 0) & (now[r] != 0))) for r in range(G)]
                    rec["rows_nonzero_now"] = [int(np.count_nonzero(now[r])) for r in range(G)]
                    full = now.sum(0)
                    rec["ws_at_finish_wrong"] = int(np.count_nonzero(
                        snaps["ws_fin"][:full.size].cpu().numpy().view(np.uint32) != full.view(np.uint32)))
                    got_out = out.cpu().numpy()
                    fin = snaps["out_fin"][: layout.pairwise_idx.size].cpu().numpy()
                    rec["out_at_finish_vs_final_differ"] = int(np.count_nonzero(
                        fin.view(np.uint32) != got_out[layout.pairwise_idx.astype(np.int64)].view(np.uint32)))
                diag.append(rec)
        errs = tr.errors()
        tr.close()
        dist.destroy_process_group()
        q.put((rank, bad, diag, errs, None))
    except Exception:  # noqa: BLE001 -- reported to the parent
        import traceback

        q.put((rank, None, None, None, traceback.format_exc()[-2000:]))


def run(mode: str, G: int, K: int, calls: int) -> dict:
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, G, K, mode, calls, port, q)) for r in range(G)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(G):
            rank, bad, diag, errs, tb = q.get(timeout=110)
            res[rank] = (bad, diag, errs, tb)
    finally:
        for p in procs:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()  # our own child, by handle
    tbs = {r: v[3] for r, v in res.items() if v[3]}
    return {"mode": mode, "G": G, "K": K, "calls": calls, "root_wrong_per_call": res[0][0],
            "diag": res[0][1], "wait_errors": {r: v[2] for r, v in res.items() if v[2]}, "tracebacks": tbs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="kernel,legacy,kcopy,tcopyk,legacy_noctx,legacy_sync")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--G", type=int, default=4)
    ap.add_argument("--K", type=int, default=9)
    ap.add_argument("--calls", type=int, default=3)
    a = ap.parse_args()
    for rep in range(a.reps):
        for mode in a.modes.split(","):
            r = run(mode, a.G, a.K, a.calls)
            r["rep"] = rep
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
