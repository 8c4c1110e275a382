"""Why a client round's one host->device staging of the averaged update runs at ~20 GB/s when
back-to-back stagings run at ~50 (tools/accelerate_algo_bench.py --breakdown,
profiles/r05i_accel_breakdown_25M.jsonl: 100 MB fp32 in 5.0 ms, 200 MB fp64 in 5.3 ms).
``weight_manager._stage_host_layers`` of L host layers, timed per call (wall, and the session's
own stage time), in four settings: back to back; after a 50 ms idle gap; after a burst of
torch GPU work on the current stream (a training step stand-in); and on fresh host arrays each
call (first touch paid before the timer).  One JSON line per setting.

    python3 tools/stage_gap_probe.py --mb 100 --layers 24 --reps 8
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=100)
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--dtype", default="float32")
    args = ap.parse_args()

    import torch

    from substrafl_amd import runtime
    from substrafl_amd.algorithms import weight_manager as wm

    dev = torch.device("cuda", 0)
    dt = np.dtype(args.dtype)
    per = args.mb * 1_000_000 // dt.itemsize // args.layers
    rng = np.random.default_rng(0)
    arrays = [rng.standard_normal(per).astype(dt) for _ in range(args.layers)]
    a = torch.randn(4096, 4096, device=dev)

    def gpu_work():
        for _ in range(20):
            torch.mm(a, a)

    def one(setting, arrs):
        torch.cuda.synchronize()
        if setting == "idle_gap":
            time.sleep(0.05)
        elif setting == "after_gpu_work":
            gpu_work()  # queued, not waited for: _stage_host_layers synchronises torch's stream
        t0 = time.perf_counter()
        flat = wm._stage_host_layers(arrs, dev)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        return t1 - t0, runtime.session(0).timing()["stage_s"], flat

    one("warm", arrays)
    for setting in ("back_to_back", "idle_gap", "after_gpu_work", "fresh_arrays"):
        walls, stages = [], []
        for _ in range(args.reps):
            arrs = [x.copy() for x in arrays] if setting == "fresh_arrays" else arrays
            w, st, flat = one(setting, arrs)
            del flat
            walls.append(w)
            stages.append(st)
        gb = args.mb / 1e3
        print(json.dumps({"setting": setting, "mb": args.mb, "layers": args.layers, "dtype": args.dtype,
                          "wall_ms": [round(1e3 * w, 2) for w in walls],
                          "stage_ms": [round(1e3 * s, 2) if s is not None else None for s in stages],
                          "median_GBps": round(gb / float(np.median(walls)), 1)}), flush=True)


if __name__ == "__main__":
    main()
