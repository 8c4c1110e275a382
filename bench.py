#!/usr/bin/env python3
"""Device-resident aggregation throughput (BASELINE.json metric:
"aggregated-param GB/s (device-resident) FedAvg reduce, N clients x M params").

One step = one pass of the hot path (the FedAvg bucket kernel + the numel == 1 pairwise
patch) over one batch of synthetic client buckets already resident in HBM.  Default workload
is BASELINE.json configs[1]: FedAvg, 8 clients x 25M fp32 params on one MI355X.

N > 1 (torchrun, one process per GPU): the buckets are sharded by PARAMETER RANGE (SURVEY.md
§8(e) primary mode): every rank owns its own 25M-param slice of an N x 25M-param model for all
8 clients, so there is no data-path collective and results are bit-identical to one GPU
(weak scaling).  value = algorithmic bytes of all ranks / max-over-ranks time.

Algorithmic bytes: FedAvg K*M*s_in + M*s_out; Scaffold
2*K*M*s_in + M*s_in + 2*M*8.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

WORKLOADS = {
    "c2": dict(name="fedavg_fp32_8x25M", strategy="fedavg", K=8, M=25_000_000, kind="f32"),
    "c3": dict(name="fedavg_fp32_64x125M", strategy="fedavg", K=64, M=125_000_000, kind="f32"),
    "c4": dict(name="scaffold_fp32_16x25M", strategy="scaffold", K=16, M=25_000_000, kind="f32"),
    "c5": dict(name="fedavg_bf16_128x350M", strategy="fedavg", K=128, M=350_000_000, kind="bf16"),
}
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "aggregated-param GB/s (device-resident) FedAvg reduce, N clients × M params"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--grid-cap", type=int, default=0)
    ap.add_argument("--nontemporal", type=int, default=-1)
    ap.add_argument("--traffic", default="", help="JSON with PMC-derived bytes per launch (profiles/)")
    return ap.parse_args()


def synth_clients(torch, K, ld, M, kind, device, rank):
    """Client k's bucket: N(0,1) from torch's device Philox stream seeded 20241016 + k (+rank salt)."""
    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f64": torch.float64}[kind]
    buf = torch.empty((K, ld), dtype=dt, device=device)
    g = torch.Generator(device=device)
    for k in range(K):
        g.manual_seed(20241016 + k + 1_000_003 * rank)
        if kind == "bf16":
            buf[k, :M].copy_(torch.randn(M, generator=g, device=device, dtype=torch.float32))
        else:
            buf[k, :M].normal_(generator=g)
        buf[k, M:].zero_()
    return buf


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from substrafl_amd import _native
    from substrafl_amd.engine import FedAvgPlan, ScaffoldPlan, fedavg_weights, scaffold_weights
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # Parameter-range sharding has no data-path collective: the process group only carries
        # the barrier and the max-over-ranks timing, on the host (gloo).
        dist.init_process_group("gloo")
    ndev = torch.cuda.device_count()
    local = local % max(1, ndev)  # lets a 1-GPU box rehearse N > 1 (ranks then share the GPU)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    lib = _native.load()
    if args.grid_cap:
        _native.tune(grid_cap=args.grid_cap)
    if args.nontemporal >= 0:
        _native.tune(nt_load=args.nontemporal)

    wl = WORKLOADS[args.workload]
    K, M, kind = wl["K"], wl["M"], wl["kind"]
    shapes = synthetic_state_dict_shapes(M)
    layout = BucketLayout(list(range(len(shapes))), shapes, np.float32)
    ld = layout.ld
    n_samples = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]

    def barrier():
        if world > 1:
            dist.barrier()

    if wl["strategy"] == "fedavg":
        clients = synth_clients(torch, K, ld, M, kind, device, rank)
        out = torch.empty(ld, dtype=torch.float32, device=device)
        w = fedavg_weights(n_samples, kind)
        plan = FedAvgPlan(kind, clients, w, M, out, layout.pairwise_idx)
        s_in = 2 if kind == "bf16" else 4
    else:
        delta = synth_clients(torch, K, ld, M, kind, device, rank)
        cv = synth_clients(torch, K, ld, M, kind, device, rank + 7919)
        c = torch.randn(ld, dtype=torch.float32, device=device)
        dout = torch.empty(ld, dtype=torch.float64, device=device)
        cout = torch.empty(ld, dtype=torch.float64, device=device)
        w = scaffold_weights(n_samples)
        plan = ScaffoldPlan(kind, delta, cv, c, w, M, 1.0, dout, cout, layout.pairwise_idx)
        s_in = 4
    bytes_alg = plan.bytes_alg()
    stream = torch.cuda.current_stream(device)

    # ---- warmup (untimed) ----
    for _ in range(args.warmup):
        plan.launch(stream)
    torch.cuda.synchronize(device)

    # ---- timed region: exactly `steps` steps, barrier + sync on both sides ----
    # HIP events on the launch stream bracket the region: kern_ms = region / steps is the
    # average launch duration of the bucket kernel (back-to-back launches, so it includes the
    # ~1-2 us inter-kernel boundary: an upper bound; rocprofv3 gives the exact duration).
    ev_start, ev_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    ev_start.record(stream)
    for _ in range(args.steps):
        plan.launch(stream)
    ev_end.record(stream)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0  # this rank's region; the job's time is the max over ranks
    barrier()
    kern_ms = ev_start.elapsed_time(ev_end) / args.steps

    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    ms_per_step = elapsed / args.steps * 1e3
    value = bytes_alg * world / (elapsed / args.steps) / 1e9

    # ---- per-launch distribution (after the timed region): one event pair per launch ----
    n_each = max(5, min(args.steps, 20))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_each)]
    for a, b in evs:
        a.record(stream)
        plan.launch(stream)
        b.record(stream)
    torch.cuda.synchronize(device)
    each_ms = np.array([a.elapsed_time(b) for a, b in evs])

    # ---- parity spot check (outside the timed region): sampled elements vs the sequential order ----
    parity = None
    if wl["strategy"] == "fedavg":
        g = np.random.default_rng(123)
        idx = np.setdiff1d(np.unique(g.integers(0, M, 4096)), layout.pairwise_idx.astype(np.int64))
        tidx = torch.from_numpy(idx).to(device)
        xs = clients[:, tidx].float().cpu().numpy()  # exact upcast for bf16
        got = out[tidx].cpu().numpy()
        w32 = fedavg_weights(n_samples, "f32")
        acc = np.zeros(idx.size, np.float32)
        for k in range(K):
            acc = (acc + (xs[k] * w32[k]).astype(np.float32)).astype(np.float32)
        # (the numel == 1 element is reduced in NumPy's pairwise order: tests/ check it against the oracle)
        parity = {"sampled": int(idx.size), "mismatches": int(np.sum(acc.view(np.uint32) != got.view(np.uint32)))}
    else:  # Scaffold (scaffold.py:262-263,293): fp64 products and sums, c added last, lr after the sum
        g = np.random.default_rng(123)
        idx = np.setdiff1d(np.unique(g.integers(0, M, 4096)), layout.pairwise_idx.astype(np.int64))
        tidx = torch.from_numpy(idx).to(device)
        xd = delta[:, tidx].double().cpu().numpy()
        xc = cv[:, tidx].double().cpu().numpy()
        cc = c[tidx].double().cpu().numpy()
        w64 = scaffold_weights(n_samples)
        ad = np.zeros(idx.size, np.float64)
        ac = np.zeros(idx.size, np.float64)
        for k in range(K):
            ad = ad + xd[k] * w64[k]
            ac = ac + xc[k] * w64[k]
        ad = 1.0 * ad
        ac = ac + cc
        gd = dout[tidx].cpu().numpy()
        gc = cout[tidx].cpu().numpy()
        parity = {"sampled": int(idx.size),
                  "mismatches": int(np.sum(ad.view(np.uint64) != gd.view(np.uint64))
                                    + np.sum(ac.view(np.uint64) != gc.view(np.uint64)))}

    # ---- read-stream ceiling on the same box (same 16-B nt load path) ----
    probe_n = min(clients.numel() if wl["strategy"] == "fedavg" else delta.numel(), 2_000_000_000)
    src = clients if wl["strategy"] == "fedavg" else delta
    nbytes_probe = probe_n * src.element_size()
    floats = nbytes_probe // 4 // 4 * 4
    full = int(min(floats // 4 // 256, 1 << 20))  # one 16-B vector per thread, like the bucket kernel
    sink = torch.empty(full, dtype=torch.float32, device=device)
    read_ceiling = 0.0
    for pgrid in sorted({min(g, full) for g in (2048, 4096, 8192, 16384, 65536)} | {full}):  # best grid = the ceiling
        for _ in range(3):
            _native.check(lib.fedagg_read_probe_f32(src.data_ptr(), floats, sink.data_ptr(), pgrid,
                                                    stream.cuda_stream), "probe")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            lib.fedagg_read_probe_f32(src.data_ptr(), floats, sink.data_ptr(), pgrid, stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize(device)
        read_ceiling = max(read_ceiling, floats * 4 / (e0.elapsed_time(e1) / 10 / 1e3) / 1e9)

    # ---- CPU baseline (rank 0, N == 1): the reference call structure timed on host cores ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(wl, args.cpu_seconds)

    traffic = None
    tpath = Path(args.traffic) if args.traffic else ROOT / "profiles" / f"traffic_{args.workload}.json"
    if tpath.exists():
        try:
            tj = json.loads(tpath.read_text())
            traffic = tj.get("hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None

    achieved = bytes_alg / (kern_ms / 1e3) / 1e9
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16-in/f32-acc" if kind == "bf16" else ("f32-in/f64-acc" if wl["strategy"] == "scaffold" else "f32"),
            "data": "synthetic (N(0,1) client buckets generated on device, torch Philox seeds 20241016+k; "
                    "n_samples = default_rng(7).integers(100, 10000, K))",
            "config": {
                "workload": wl["name"],
                "strategy": wl["strategy"],
                "clients": K,
                "params_per_gpu": M,
                "global_params": M * world,
                "layers": len(shapes),
                "parallelism": f"param-range x{world}" if world > 1 else "single-gpu",
                "bytes_alg_per_step_per_gpu": bytes_alg,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "kernel": (f"fedavg_kernel<{'BF16' if kind == 'bf16' else 'F32'}>" if wl["strategy"] == "fedavg"
                           else "scaffold_kernel<float>"),
                "kernel_ms": round(kern_ms, 5),
                "kernel_ms_median": round(float(np.median(each_ms)), 5),
                "kernel_ms_min": round(float(each_ms.min()), 5),
                "read_stream_ceiling_GBps": round(read_ceiling, 1),
                "frac_of_read_ceiling": round(achieved / read_ceiling, 4),
            },
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(wl, budget_s):
    """Time the oracle's reference-call-structure FedAvg/Scaffold (list of products, np.sum) on a
    bounded host sample of the same workload shape.  NumPy's ufuncs are single-threaded here,
    so the reference path uses one core whatever the machine has."""
    from oracle import fedavg_reference_structure, scaffold_reference_structure
    from substrafl_amd.layout import synthetic_state_dict_shapes

    K = wl["K"]
    M_s = min(wl["M"], 25_000_000 if K <= 16 else 4_000_000)
    shapes = synthetic_state_dict_shapes(M_s)
    rng = np.random.default_rng(1)

    def client():
        return [rng.standard_normal(s, dtype=np.float32) for s in shapes]

    n_samples = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    if wl["strategy"] == "fedavg":
        pus = [client() for _ in range(K)]
        if wl["kind"] == "bf16":  # exact bf16 values, upcast (the reference cannot carry bf16)
            pus = [[(a.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32) for a in c] for c in pus]
        fn = lambda: fedavg_reference_structure(pus, n_samples)  # noqa: E731
        s_in = 2 if wl["kind"] == "bf16" else 4
        nbytes = K * M_s * s_in + M_s * 4
    else:
        pus = [client() for _ in range(K)]
        cvs = [client() for _ in range(K)]
        c = client()
        fn = lambda: scaffold_reference_structure(pus, cvs, c, n_samples, 1.0)  # noqa: E731
        nbytes = 2 * K * M_s * 4 + M_s * 4 + 2 * M_s * 8
    times = []
    t_end = time.perf_counter() + budget_s
    while len(times) < 3 or (time.perf_counter() < t_end and len(times) < 50):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() > t_end and len(times) >= 1:
            break
    best = min(times)
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:  # noqa: BLE001
        aff = os.cpu_count()
    return {
        "value": round(nbytes / best / 1e9, 3),
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{K} clients x {M_s} fp32 params ({len(shapes)} layers), best of {len(times)} runs "
                  f"({best * 1e3:.1f} ms); oracle/aggregation.py reference call structure; "
                  f"host has {os.cpu_count()} cpus, affinity {aff}, NumPy ufuncs single-threaded",
    }


if __name__ == "__main__":
    main()
