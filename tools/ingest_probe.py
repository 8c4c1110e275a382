#!/usr/bin/env python3
"""Host ingest probe for SURVEY.md §8(f) rows 1-2: how fast can an aggregate task get K shared-state
pickles (reference format: PickleSerializer, protocol 4) into host memory?

  seq      -- the reference's loop (substratools_methods.py:61-64), one pickle.load per file
  threads  -- the same pickle.load calls on a thread pool (file reads release the GIL)
  readinto -- raw file bytes into one preallocated buffer per file (fresh / reused), the floor
Prints one JSON line per (K, M)."""

import argparse
import json
import os
import pickle
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def best(fn, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t)
        del r
    return min(ts), ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=8)
    ap.add_argument("--M", type=int, default=25_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from substrafl_amd.layout import synthetic_state_dict_shapes
    from substrafl_amd.schemas import FedAvgSharedState

    shapes = synthetic_state_dict_shapes(args.M)
    tmp = Path(tempfile.mkdtemp(prefix="ingest_", dir=os.environ.get("TMPDIR", "/tmp")))
    rng = np.random.default_rng(0)
    paths = []
    for k in range(args.K):
        st = FedAvgSharedState(n_samples=100 + k, parameters_update=[rng.standard_normal(s, dtype=np.float32) for s in shapes])
        p = tmp / f"s{k}"
        with open(p, "wb") as f:
            pickle.dump(st, f)
        paths.append(p)
    nbytes = sum(p.stat().st_size for p in paths)

    def load(p):
        with open(p, "rb") as f:
            return pickle.load(f)

    out = dict(K=args.K, M=args.M, file_bytes=nbytes, cpus=os.cpu_count())
    out["seq_s"], _ = best(lambda: [load(p) for p in paths], args.reps)
    for th in (4, 8, 16):
        with ThreadPoolExecutor(th) as ex:
            out[f"threads{th}_s"], _ = best(lambda: list(ex.map(load, paths)), args.reps)

    def readinto(bufs):
        for p, b in zip(paths, bufs):
            with open(p, "rb", buffering=0) as f:
                f.readinto(memoryview(b))
        return bufs

    sizes = [p.stat().st_size for p in paths]
    out["readinto_fresh_s"], _ = best(lambda: readinto([np.empty(n, np.uint8) for n in sizes]), args.reps)
    reused = [np.ones(n, np.uint8) for n in sizes]
    out["readinto_reused_s"], _ = best(lambda: readinto(reused), args.reps)
    t = time.perf_counter()
    faulted = [np.ones(n, np.uint8) for n in sizes]
    out["fault_only_s"] = time.perf_counter() - t
    del faulted
    with ThreadPoolExecutor(8) as ex:
        def one(i):
            b = np.empty(sizes[i], np.uint8)
            with open(paths[i], "rb", buffering=0) as f:
                f.readinto(memoryview(b))
            return b
        out["readinto_fresh_threads8_s"], _ = best(lambda: list(ex.map(one, range(len(paths)))), args.reps)
    for k, v in list(out.items()):
        if k.endswith("_s"):
            out[k.replace("_s", "_GBps")] = round(nbytes / v / 1e9, 2)
            out[k] = round(v, 4)
    print(json.dumps(out), flush=True)
    for p in paths:
        p.unlink()


if __name__ == "__main__":
    main()
