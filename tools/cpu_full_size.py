#!/usr/bin/env python3
"""The reference's CPU path at a BASELINE config's full size (bench.py's cpu_baseline
leg times a bounded sample).  Times the oracle's reference-call-structure FedAvg
(oracle/aggregation.py, the same NumPy calls as fed_avg.py:217-222) once or twice over the full
K x M host state -- C3 is 64 x 125M fp32 = 32 GB of client states, ~40 GB peak -- and prints one
JSON line.  C5 (128 x 350M, which the reference can only hold as fp32: 179 GB of inputs plus the
per-layer temporaries) does not fit a GPU box's host memory budget and is not run."""

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3", choices=["c2", "c3", "c4"])
    ap.add_argument("--runs", type=int, default=2)
    args = ap.parse_args()
    from oracle import fedavg_reference_structure, scaffold_reference_structure
    from substrafl_amd.layout import synthetic_state_dict_shapes

    K, M = {"c2": (8, 25_000_000), "c3": (64, 125_000_000), "c4": (16, 25_000_000)}[args.workload]
    shapes = synthetic_state_dict_shapes(M)
    rng = np.random.default_rng(1)
    t0 = time.perf_counter()
    base = [rng.standard_normal(s, dtype=np.float32) for s in shapes]

    def clients():  # distinct clients without K x M random draws: per-client scaled copies
        return [[(a * np.float32(1 + 1e-3 * k)).astype(np.float32) for a in base] for k in range(K)]

    pus = clients()
    n_samples = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    if args.workload == "c4":
        cvs = clients()
        fn = lambda: scaffold_reference_structure(pus, cvs, base, n_samples, 1.0)  # noqa: E731
        nbytes = 2 * K * M * 4 + M * 4 + 2 * M * 8
    else:
        fn = lambda: fedavg_reference_structure(pus, n_samples)  # noqa: E731
        nbytes = K * M * 4 + M * 4
    gen_s = time.perf_counter() - t0
    times = []
    for _ in range(args.runs):
        t = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t)
    best = min(times)
    print(json.dumps({"workload": args.workload, "clients": K, "params": M, "layers": len(shapes),
                      "kind": "port (oracle/aggregation.py reference call structure, full size)",
                      "cores": 1, "runs_s": [round(x, 3) for x in times], "GBps": round(nbytes / best / 1e9, 3),
                      "data_generation_s": round(gen_s, 1), "host_cpus": os.cpu_count()}), flush=True)


if __name__ == "__main__":
    main()
