"""Staging rate of one GPU's native session against its pack thread count (VERDICT r04 "Next 4").

``fedagg_session_stage`` of the BASELINE C2 (8 x 25M fp32) and C3 (64 x 125M fp32) client rows --
per-layer host arrays of the synthetic state dict, as unpickled -- into HBM with 2, 4, 8 and 16
pack workers, unbound and bound to the GPU's NUMA node (multi_device.host_placement).  Best of
--reps; one JSON line per (workload, threads, binding).  The 1-GPU box grants this process 16
CPUs, so 16 is the top of the sweep.

    python3 tools/stage_threads_probe.py --workloads c2,c3 --threads 2,4,8,16
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

WL = {"c2": (8, 25_000_000), "c3": (64, 125_000_000)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c2,c3")
    ap.add_argument("--threads", default="2,4,8,16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args()

    from substrafl_amd import runtime
    from substrafl_amd.layout import synthetic_state_dict_shapes
    from substrafl_amd.multi_device import host_placement

    dev = args.device
    bus = runtime.device_pci_bus_id(dev)
    (place,) = host_placement([bus])
    allowed = sorted(os.sched_getaffinity(0))
    print(json.dumps({"device": dev, "bus_id": bus, "numa_node": place["numa_node"],
                      "node_cpus_allowed": len(place["cpus"]), "cpus_allowed": len(allowed),
                      "os_cpu_count": os.cpu_count()}), flush=True)
    s = runtime.Session(dev)
    for wl in args.workloads.split(","):
        K, M = WL[wl]
        shapes = synthetic_state_dict_shapes(M)
        t0 = time.perf_counter()
        rows = []
        for k in range(K):  # distinct, faulted-in per-layer arrays (no cache reuse between clients)
            rows.append([np.full(sh, np.float32(k + 1)) for sh in shapes])
        gen_s = time.perf_counter() - t0
        nbytes = K * M * 4
        d = s.buffer(0, nbytes)
        for binding in ("unbound", "numa"):
            if binding == "numa" and not place["cpus"]:
                continue
            s.affinity(place["cpus"] if binding == "numa" else None)
            for T in [int(v) for v in args.threads.split(",")]:
                s.set("threads", T)
                s.stage(d, M * 4, rows)  # warm: ring, pool
                s.sync()
                best = float("inf")
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    s.stage(d, M * 4, rows)
                    s.sync()
                    best = min(best, time.perf_counter() - t0)
                print(json.dumps({"workload": wl, "clients": K, "params": M, "bytes": nbytes, "threads": T,
                                  "binding": binding, "ring_node": s.ring_node(), "stage_s": round(best, 4),
                                  "stage_GBps": round(nbytes / best / 1e9, 2), "host_arrays_gen_s": round(gen_s, 1)}),
                      flush=True)
        del rows
    s.close()


if __name__ == "__main__":
    main()
