#!/usr/bin/env python3
"""Fresh-process load of K shared-state pickles: pickle.load vs the mapped loader
(substrafl_amd/remote/mapped_pickle.py), each followed by one read pass over every array (what
staging does).  The parent writes the files once (page cache warm) and times each child."""

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def child(mode, d, K, threads):
    from concurrent.futures import ThreadPoolExecutor

    import pickle

    from substrafl_amd.remote import mapped_pickle

    paths = [Path(d) / f"s{k}" for k in range(K)]
    if mode == "pickle":
        def load(p):
            with open(p, "rb") as f:
                return pickle.load(f)
    else:
        mapped_pickle.POPULATE = mode == "mapped_populate"
        load = mapped_pickle.load_mapped
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        states = list(ex.map(load, paths))
    t1 = time.perf_counter()
    s = 0.0
    for st in states:  # one read pass (staging reads every byte once)
        for a in st.parameters_update:
            s += float(a.reshape(-1)[:: max(1, a.size // 4096)].sum()) if a.size else 0.0
            if a.size:
                np.asarray(a).view(np.uint8).sum(dtype=np.uint64)
    t2 = time.perf_counter()
    print(json.dumps({"mode": mode, "threads": threads, "load_s": round(t1 - t0, 4), "touch_s": round(t2 - t1, 4)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=8)
    ap.add_argument("--M", type=int, default=25_000_000)
    ap.add_argument("--child", default="")
    ap.add_argument("--dir", default="")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    if a.child:
        return child(a.child, a.dir, a.K, a.threads)
    from substrafl_amd.layout import synthetic_state_dict_shapes
    from substrafl_amd.remote import PickleSerializer
    from substrafl_amd.schemas import FedAvgSharedState

    d = Path(tempfile.mkdtemp(prefix="mapload_", dir=os.environ.get("TMPDIR", "/tmp")))
    rng = np.random.default_rng(0)
    shapes = synthetic_state_dict_shapes(a.M)
    for k in range(a.K):
        PickleSerializer.save(FedAvgSharedState(n_samples=k + 1, parameters_update=[
            rng.standard_normal(s, dtype=np.float32) for s in shapes]), d / f"s{k}")
    for rep in range(3):
        for mode in ("pickle", "mapped", "mapped_populate"):
            for th in (1, a.threads):
                t0 = time.perf_counter()
                r = subprocess.run([sys.executable, __file__, "--child", mode, "--dir", str(d), "--K", str(a.K),
                                    "--threads", str(th)], capture_output=True, text=True, check=True)
                print(r.stdout.strip()[:-1] + f', "process_s": {time.perf_counter() - t0:.4f}, "rep": {rep}}}',
                      flush=True)


if __name__ == "__main__":
    main()
