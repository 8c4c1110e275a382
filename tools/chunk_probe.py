#!/usr/bin/env python3
"""The chain kernel at the run sizes of the client-sharded schedules (substrafl_amd/lockstep.py).

The striped schedule launches one chain kernel per step over a rank's client block: for C3 in the
weak form (64 clients per rank, 125M params) a run is M / (2 G rounds) elements -- 7.8M at G = 8,
one round.  This probe times ``fedagg_fedavg_chain_*`` (rows) and ``fedagg_fedavg_chain_tiled_*``
(tile-interleaved, both fp32 tiles) at such sizes with HIP events, and the host cost of issuing one
run through ``GpuShardOps.fedavg_run`` (ctypes + pointer table), which bounds how short a step may
be when the schedule is issued from Python.

    python3 tools/chunk_probe.py [--clients 64] [--sizes 2e6,3.9e6,7.8e6,15.6e6,31.25e6,62.5e6,125e6]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--sizes", default="2e6,3.90625e6,7.8125e6,15.625e6,31.25e6,62.5e6,125e6")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--knobs", default="", help="tuning build only: rows under each knob set, "
                    "e.g. 'vpt=4,unroll=4;vpt=2,unroll=8' (FEDAGG_LIB=substrafl_amd/libfedagg_tuning.so)")
    ap.add_argument("--no-tiled", action="store_true")
    args = ap.parse_args()

    import torch

    from substrafl_amd.engine import fedavg_weights, tiled_elems
    from substrafl_amd.sharding import GpuShardOps, TiledView

    dev = torch.device("cuda", 0)
    ops = GpuShardOps()
    K = args.clients
    w = fedavg_weights(list(range(1, K + 1)), "f32")
    sizes = [int(float(x)) // 512 * 512 for x in args.sizes.split(",")]
    Mmax = max(sizes)
    rows = torch.empty((K, Mmax), dtype=torch.float32, device=dev).normal_()
    acc = torch.empty(Mmax, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev)

    def timeit(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / args.reps

    res = []
    for n in sizes:
        nbytes = K * n * 4 + n * 4 * 2  # client reads + accumulator read and write (seed = 0)
        line = {"clients": K, "elems": n, "GB": round(nbytes / 1e9, 3)}
        r = rows[:, :n]
        ms = timeit(lambda: ops.fedavg_run("f32", r, w, False, acc[:n]))
        line["rows_ms"], line["rows_TBps"] = round(ms, 4), round(nbytes / ms / 1e9, 3)
        for ks in [k for k in args.knobs.split(";") if k]:
            from substrafl_amd import _native

            kv = {a: int(b) for a, b in (x.split("=") for x in ks.split(","))}
            _native.tune(**kv)
            ms = timeit(lambda: ops.fedavg_run("f32", r, w, False, acc[:n]))
            _native.tune(vpt=0, unroll=8)
            line[f"rows[{ks}]_TBps"] = round(nbytes / ms / 1e9, 3)
        for tv in (() if args.no_tiled else (2048, 8192)):
            buf = torch.empty(tiled_elems("f32", K, n, tv), dtype=torch.float32, device=dev).normal_()
            view = TiledView("f32", buf, K, n, tv)
            ms = timeit(lambda: ops.fedavg_run("f32", view, w, False, acc[:n]))
            line[f"tiled{tv}_ms"], line[f"tiled{tv}_TBps"] = round(ms, 4), round(nbytes / ms / 1e9, 3)
            del buf
        res.append(line)
        print(json.dumps(line), flush=True)
    # host cost of one run issued from Python (kernel queue kept short by syncing every 20)
    n = sizes[0]
    t0 = time.perf_counter()
    for i in range(200):
        ops.fedavg_run("f32", rows[:, :n], w, False, acc[:n])
        if i % 20 == 19:
            torch.cuda.synchronize(dev)
    host_us = (time.perf_counter() - t0) / 200 * 1e6
    print(json.dumps({"host_us_per_run_incl_gpu": round(host_us, 1), "note": "upper bound: includes the GPU time "
                      "of the smallest run when the queue drains"}), flush=True)


if __name__ == "__main__":
    main()
