#!/usr/bin/env python3
"""Device-resident aggregation throughput (BASELINE.json metric:
"aggregated-param GB/s (device-resident) FedAvg reduce, N clients x M params").

One step = one pass of the hot path over one batch of synthetic client buckets already resident
in HBM.  The default workload is BASELINE.json configs[2] on one MI355X: FedAvg, 64 clients x
125M fp32 params (C3) -- the configuration north_star's ">= 80 % of the single-GPU HBM-read
roofline" target is stated on.

Multi-GPU (one process per GPU).  ``--gpus N`` from a plain ``python3 bench.py`` starts the N rank
processes itself (before anything touches a GPU); under torchrun the ranks come from the
environment, and a WORLD_SIZE that differs from --gpus is an error.  Modes:

* ``--mode param-range`` (default; SURVEY.md §8(e) primary, bit-exact): every rank reduces its own
  parameter range of all K clients -- no data-path collective.  ``--scaling weak`` (default): each
  rank owns a full M-param slice of an N*M-param model; ``--scaling strong``: the workload's own M
  is split over the N ranks (C3 at 64 x 125M over 8 GPUs = 15.6M params per GPU).
* ``--mode client-shard --combine relay|rccl|ordered|striped`` (the north-star mode): the clients
  are split over the ranks, partial sums stay in HBM and are combined over RCCL/xGMI on the root
  (``relay`` and ``striped`` bit-exact; ``striped``: the relay over up to four parameter stripes
  whose chains hop over disjoint xGMI links, one communicator each; see
  substrafl_amd/sharding.py).  ``--scaling weak``: every rank holds the
  workload's K clients (N*K clients of M params in all -- the "buckets overflow one GPU" case);
  ``--scaling strong``: the workload's K clients are split over the N ranks.  Needs one GPU per
  rank.
* ``--engine multi-device``: the drop-in's own multi-GPU path, ONE process driving N GPUs
  (MultiDeviceEngine: host buckets staged over each GPU's PCIe link, per-shard kernel time from
  HIP events on the session streams) -- an end-to-end line, not the device-resident metric.

value = algorithmic bytes of the whole job / max-over-ranks time.  Algorithmic bytes (SURVEY.md
§8(d)): FedAvg K*M*s_in + M*s_out; Scaffold 2*K*M*s_in + M*s_in + 2*M*8.
"""

from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
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
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--mode", default="param-range", choices=["param-range", "client-shard"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--combine", default="relay", choices=["relay", "rccl", "ordered", "striped"])
    ap.add_argument("--engine", default="rank", choices=["rank", "multi-device"])
    ap.add_argument("--tile", type=int, default=0, help="tiles layout: 16-B vectors per client tile "
                    "(0: the library's choice; FEDAGG_TILE_VECTORS_*)")
    ap.add_argument("--layout", default="auto", choices=["rows", "tiles", "auto"],
                    help="client buckets in HBM: [K, ld] rows, tile-interleaved (fedagg_fedavg_tiled_*; "
                         "FedAvg fp32/bf16), or (default) tiles where the library recommends them -- the "
                         "layout the drop-in host path stages (AggregationEngine.tiled)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--grid-cap", type=int, default=0)
    ap.add_argument("--tune", default="", help="library launch knobs for experiments, key=value[,key=value] "
                    "(fedagg_tune; the default run sets none)")
    ap.add_argument("--nontemporal", type=int, default=-1)
    ap.add_argument("--traffic", default="", help="JSON with PMC-derived bytes per launch (profiles/)")
    ap.add_argument("--cpu-only", action="store_true",
                    help="run only the cpu_baseline leg (no GPU) and print its JSON")
    ap.add_argument("--cpu-full-size", action="store_true",
                    help="cpu_baseline over the workload's full K x M instead of a bounded sample (C3: ~40 GB host)")
    ap.add_argument("--rehearse-cpu", action="store_true",
                    help="tests only: run the launcher / rank / timing plumbing with no GPU (no measurement)")
    return ap.parse_args()


# ======================================================================================
# launcher: --gpus N from a plain `python3 bench.py`
# ======================================================================================
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int) -> int:
    """Start ranks 0..n-1 of this very command as child processes (torchrun's environment
    contract: RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT), before any GPU call in this
    process; wait for all of them and return the first failure's code (0 if all succeeded).
    A failed rank takes the others down (exact PIDs, no pattern kill)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]], env=env))
    rc = 0
    alive = set(range(n))
    while alive:
        for r in sorted(alive):
            code = procs[r].poll()
            if code is None:
                continue
            alive.discard(r)
            if code != 0 and rc == 0:
                rc = code
                print(f"bench.py: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr)
                for o in alive:
                    procs[o].terminate()
        time.sleep(0.05)
    return rc


# ======================================================================================
# synthetic device-resident buckets
# ======================================================================================
def synth_clients(torch, K, ld, M, kind, device, seed0):
    """Client k's bucket: N(0,1) from torch's device Philox stream seeded seed0 + k."""
    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f64": torch.float64}[kind]
    buf = torch.empty((max(1, K), ld), dtype=dt, device=device)
    g = torch.Generator(device=device)
    for k in range(K):
        g.manual_seed(seed0 + k)
        if kind == "bf16":
            buf[k, :M].copy_(torch.randn(M, generator=g, device=device, dtype=torch.float32))
        else:
            buf[k, :M].normal_(generator=g)
        buf[k, M:].zero_()
    return buf[:K]


def synth_tiled(torch, K, M, kind, device, seed0, tv):
    """The same client buckets as synth_clients (client k: Philox seed seed0 + k), laid out
    tile-interleaved with tiles of tv vectors (engine.tiled_client_view): tile t of client k is
    tile t * K + k."""
    from substrafl_amd.engine import tiled_client_view, tiled_elems

    dt = torch.bfloat16 if kind == "bf16" else torch.float32
    buf = torch.zeros(tiled_elems(kind, K, M, tv), dtype=dt, device=device)
    g = torch.Generator(device=device)
    row = None
    for k in range(K):
        view = tiled_client_view(buf, kind, K, k, tv)
        if row is None:
            row = torch.zeros(view.numel(), dtype=torch.float32, device=device)
        g.manual_seed(seed0 + k)
        row[:M].normal_(generator=g)
        view.copy_(row.view(view.shape))
    return buf


def lib_sha256() -> str:
    p = ROOT / "substrafl_amd" / "libfedagg.so"
    return hashlib.sha256(p.read_bytes()).hexdigest()[:16] if p.exists() else ""


def read_traffic(args, sha):
    """PMC-derived HBM bytes per launch from a rocprofv3 --pmc session (tools/pmc_traffic.py),
    with its source file and whether it was collected on this very build of libfedagg.so."""
    tpath = Path(args.traffic) if args.traffic else ROOT / "profiles" / f"traffic_{args.workload}.json"
    if not tpath.exists():
        return None, None
    try:
        tj = json.loads(tpath.read_text())
    except Exception:  # noqa: BLE001
        return None, None
    src = {"file": str(tpath.relative_to(ROOT)) if tpath.is_relative_to(ROOT) else str(tpath),
           "lib_sha256": tj.get("lib_sha256"), "same_build": tj.get("lib_sha256") == sha,
           "collected": tj.get("collected", "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes")}
    return tj.get("hbm_bytes_per_launch"), src


# ======================================================================================
# the rank path (device-resident metric)
# ======================================================================================
def main():
    args = parse()
    if args.cpu_only:
        print(json.dumps(cpu_baseline(WORKLOADS[args.workload], args.cpu_seconds, full=args.cpu_full_size)),
              flush=True)
        return None
    if args.engine == "multi-device":
        return multi_device_bench(args)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; refusing to report a mislabelled line",
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if args.rehearse_cpu:
        return rehearse(args, world, rank)

    import torch
    import torch.distributed as dist

    from substrafl_amd import _native
    from substrafl_amd.engine import FedAvgPlan, ScaffoldPlan, fedavg_weights, scaffold_weights
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes
    from substrafl_amd.sharding import (DistTransport, FedAvgShard, GpuShardOps, ScaffoldShard, block_of,
                                        client_blocks, client_shard_fedavg, client_shard_fedavg_striped,
                                        client_shard_scaffold, client_shard_scaffold_striped, shard_bounds,
                                        stripe_layout)

    ndev = torch.cuda.device_count()
    if ndev == 0:
        print("bench.py: no GPU visible", file=sys.stderr)
        sys.exit(3)
    client_shard = args.mode == "client-shard"
    if client_shard and world > ndev:
        print(f"bench.py: --mode client-shard needs one GPU per rank (RCCL); {world} ranks, {ndev} GPUs",
              file=sys.stderr)
        sys.exit(2)
    dev_index = local % ndev  # param-range: a 1-GPU box can rehearse N > 1 (the ranks share the GPU)
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        if client_shard:  # the exchange is RCCL over xGMI
            dist.init_process_group("nccl", device_id=device)
        else:  # parameter ranges need no data-path collective: barrier + max-over-ranks only
            dist.init_process_group("gloo")
    lib = _native.load()
    if args.grid_cap:
        _native.tune(grid_cap=args.grid_cap)
    if args.nontemporal >= 0:
        _native.tune(nt_load=args.nontemporal)
    if args.tune:
        _native.tune(**{k: int(v) for k, v in (kv.split("=") for kv in args.tune.split(","))})

    wl = WORKLOADS[args.workload]
    K, M_glob, kind = wl["K"], wl["M"], wl["kind"]
    if client_shard and args.scaling == "weak":
        K *= world  # every rank holds the workload's K clients
    scaffold = wl["strategy"] == "scaffold"
    n_samples = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    s_in = 2 if kind == "bf16" else 4

    # ---- this rank's share of the job ----
    if client_shard:
        M = M_glob
        k0, k1 = client_blocks(K, world)[block_of(rank, world)]
        parallelism = f"client-shard x{world} ({args.combine})" if world > 1 else "single-gpu"
        scaling = args.scaling
    elif args.scaling == "strong":
        lo, hi = shard_bounds(M_glob, world)[rank]
        M = hi - lo
        k0, k1 = 0, K
        parallelism = f"param-range x{world} (strong)" if world > 1 else "single-gpu"
        scaling = "strong"
    else:
        M = M_glob
        k0, k1 = 0, K
        parallelism = f"param-range x{world}" if world > 1 else "single-gpu"
        scaling = "weak"
    Kr = k1 - k0
    shapes = synthetic_state_dict_shapes(M_glob if client_shard else max(M, 1))
    layout = BucketLayout(list(range(len(shapes))), shapes, np.float32)
    ld = layout.ld
    pw = layout.pairwise_idx
    seed0 = 20241016 + k0 + (1_000_003 * rank if not client_shard else 0)
    # striped relay: this rank's block per parameter stripe, one communicator per stripe
    striped = client_shard and args.combine == "striped" and world > 1
    stripes = stripe_layout(M, K, world, rank) if striped else []
    if striped:
        strs = [DistTransport()] + [DistTransport(dist.new_group()) for _ in range(len(stripes) - 1)]
        bounds = [(lo, hi, a) for lo, hi, a, *_ in stripes]
        pw64 = pw.astype(np.int64)

        def local_pw(lo, hi):
            return (pw64[(pw64 >= lo) & (pw64 < hi)] - lo).astype(np.uint64)

        def stripe_rows(si, lo, hi, k0s, k1s, salt=0):  # client k's stripe si: Philox seed per (k, stripe)
            n = hi - lo
            return synth_clients(torch, k1s - k0s, max(64, -(-n // 64) * 64), n, kind, device,
                                 20241016 + 7919 * salt + 104729 * si + k0s)

    class _Plans:  # the stripes' block kernels, back to back
        def __init__(self, plans):
            self.plans = plans

        def launch(self, st):
            for p in self.plans:
                p.launch(st)

        def bytes_alg(self):
            return sum(p.bytes_alg() for p in self.plans)

    def barrier():
        if world > 1:
            dist.barrier()

    stream = torch.cuda.current_stream(device)
    from substrafl_amd.engine import TiledFedAvgPlan, tiled_recommended, tiled_tile

    tiled = (not scaffold and not client_shard and kind in ("f32", "bf16")
             and (args.layout == "tiles" or (args.layout == "auto" and tiled_recommended(kind, K, M))))
    tv = (args.tile or tiled_tile(kind, K, M)) if tiled else 0
    if args.layout == "tiles" and not tiled:
        print("bench.py: --layout tiles takes the FedAvg fp32/bf16 workloads in param-range mode", file=sys.stderr)
        sys.exit(2)
    if not scaffold:
        clients = synth_tiled(torch, K, M, kind, device, seed0, tv) if tiled else \
            synth_clients(torch, Kr, ld, M, kind, device, seed0)
        out = torch.empty(ld, dtype=torch.float32, device=device)
        w_all = fedavg_weights(n_samples, kind)
        if tiled:
            plan = TiledFedAvgPlan(kind, clients, K, w_all, M, out, pw, tv=tv)
            kplan = plan

            def step():
                plan.launch(stream)
        elif striped:
            del clients
            parts = [FedAvgShard(kind, stripe_rows(si, lo, hi, k0s, k1s), w_all[k0s:k1s], k0s, K, hi - lo,
                                 local_pw(lo, hi)) for si, (lo, hi, a, b, k0s, k1s) in enumerate(stripes)]
            clients = parts  # spot check
            ops = GpuShardOps()
            ws = torch.zeros((max(1, pw.size), K), dtype=torch.float32, device=device)

            def step():
                client_shard_fedavg_striped(parts, bounds, out, strs, ops, pw, ws=ws)

            kplan = _Plans([FedAvgPlan(kind, sh.rows, sh.w, sh.M, out[lo:], None)
                            for sh, (lo, hi, a) in zip(parts, bounds) if sh.Kr and sh.M])
        elif client_shard:
            sh = FedAvgShard(kind, clients, w_all[k0:k1], k0, K, M, pw)
            ops, tr = GpuShardOps(), DistTransport() if world > 1 else None
            ws = torch.zeros((max(1, pw.size), K), dtype=torch.float32, device=device)

            def step():
                if world > 1:
                    client_shard_fedavg(sh, out, tr, ops, args.combine, ws=ws)
                else:
                    FedAvgPlan(kind, clients, w_all, M, out, pw).launch(stream)

            # this block's partial kernel (a rank with no clients, K < N, has none)
            kplan = FedAvgPlan(kind, clients, w_all[k0:k1], M, out, None) if Kr else None
        else:
            plan = FedAvgPlan(kind, clients, w_all, M, out, pw)
            kplan = plan

            def step():
                plan.launch(stream)
        bytes_job = K * M_glob * s_in + M_glob * 4
        bytes_kernel = kplan.bytes_alg() if kplan else 0
    else:
        delta = synth_clients(torch, Kr, ld, M, kind, device, seed0)
        cv = synth_clients(torch, Kr, ld, M, kind, device, seed0 + 7919)
        gc = torch.Generator(device=device)
        gc.manual_seed(4242)
        c = torch.randn(ld, dtype=torch.float32, device=device, generator=gc)
        dout = torch.empty(ld, dtype=torch.float64, device=device)
        cout = torch.empty(ld, dtype=torch.float64, device=device)
        w_all = scaffold_weights(n_samples)
        if striped:
            del delta, cv
            parts = [ScaffoldShard(kind, stripe_rows(si, lo, hi, k0s, k1s), stripe_rows(si, lo, hi, k0s, k1s, salt=1),
                                   c[lo:hi], w_all[k0s:k1s], k0s, K, hi - lo, 1.0, local_pw(lo, hi))
                     for si, (lo, hi, a, b, k0s, k1s) in enumerate(stripes)]
            delta, cv = parts, parts  # spot check
            ops = GpuShardOps()

            def step():
                client_shard_scaffold_striped(parts, bounds, dout, cout, strs, ops, pw, c=c)

            kplan = _Plans([ScaffoldPlan(kind, sh.delta, sh.cv, sh.c, sh.w, sh.M, 1.0, dout[lo:], cout[lo:], None)
                            for sh, (lo, hi, a) in zip(parts, bounds) if sh.Kr and sh.M])
        elif client_shard:
            sh = ScaffoldShard(kind, delta, cv, c, w_all[k0:k1], k0, K, M, 1.0, pw)
            ops, tr = GpuShardOps(), DistTransport() if world > 1 else None

            def step():
                if world > 1:
                    client_shard_scaffold(sh, dout, cout, tr, ops, args.combine)
                else:
                    ScaffoldPlan(kind, delta, cv, c, w_all, M, 1.0, dout, cout, pw).launch(stream)

            kplan = ScaffoldPlan(kind, delta, cv, c, w_all[k0:k1], M, 1.0, dout, cout, None) if Kr else None
        else:
            plan = ScaffoldPlan(kind, delta, cv, c, w_all, M, 1.0, dout, cout, pw)
            kplan = plan

            def step():
                plan.launch(stream)
        bytes_job = 2 * K * M_glob * 4 + M_glob * 4 + 2 * M_glob * 8
        bytes_kernel = kplan.bytes_alg() if kplan else 0
    if not client_shard and args.scaling == "weak":  # every rank reduces a full M-param slice
        bytes_job = bytes_kernel * world

    # ---- warmup (untimed) ----
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)

    # ---- timed region: exactly `steps` steps, barrier + sync on both sides ----
    ev_start, ev_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    ev_start.record(stream)
    for _ in range(args.steps):
        step()
    ev_end.record(stream)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0  # this rank's region; the job's time is the max over ranks
    barrier()
    step_ms_dev = ev_start.elapsed_time(ev_end) / args.steps

    # ---- the dominant kernel alone, HIP events on its launch stream (after the timed region) ----
    n_each = max(5, min(args.steps, 20))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_each)]
    for a, b in evs:
        a.record(stream)
        if kplan:
            kplan.launch(stream)
        b.record(stream)
    torch.cuda.synchronize(device)
    each_ms = np.array([a.elapsed_time(b) for a, b in evs])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(max(5, min(args.steps, 50))):
        if kplan:
            kplan.launch(stream)
    e1.record(stream)
    torch.cuda.synchronize(device)
    kern_ms = e0.elapsed_time(e1) / max(5, min(args.steps, 50))
    if not client_shard:  # the step IS the one kernel, launched back to back: region / steps
        kern_ms = step_ms_dev

    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64,
                         device=device if client_shard else torch.device("cpu"))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
    else:
        kern_ms_max = kern_ms
    ms_per_step = elapsed / args.steps * 1e3
    value = bytes_job / (elapsed / args.steps) / 1e9

    # ---- parity spot check (outside the timed region) ----
    step()  # the kernel-alone launches above overwrote the outputs with a block's partial
    torch.cuda.synchronize(device)
    parity = spot_check(torch, dist, world, rank, client_shard, scaffold, K, k0, k1, M, layout, n_samples, kind,
                        device, locals())

    # ---- read-stream ceiling on the same box (same 16-B nt load path) ----
    src = clients if not scaffold else delta
    if isinstance(src, list):  # striped: this rank's largest stripe block
        src = max((p.rows if not scaffold else p.delta for p in src), key=lambda t: t.numel())
    read_ceiling = read_probe(torch, lib, src, stream, device, _native)

    # ---- CPU baseline (rank 0, N == 1): the reference call structure timed on host cores ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(wl, args.cpu_seconds, full=args.cpu_full_size)

    sha = lib_sha256()
    traffic, tsrc = read_traffic(args, sha) if (world == 1 or args.scaling == "weak") and not client_shard \
        else (None, None)

    achieved = bytes_kernel / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else 0.0
    if rank == 0:
        if not scaffold:
            kname = f"fedavg_kernel<{'BF16' if kind == 'bf16' else 'F32'}>"
        elif lib.fedagg_scaffold_launches(max(1, Kr), 4, M, 1) == 2:  # the library's own launch plan
            kname = "scaffold_bucket_kernel<float> x2 (delta bucket, then control variate + c)"
        else:
            kname = "scaffold_kernel<float>"
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "bf16-in/f32-acc" if kind == "bf16" else ("f32-in/f64-acc" if scaffold else "f32"),
            "data": "synthetic (N(0,1) client buckets generated on device, torch Philox seeds 20241016+k; "
                    "n_samples = default_rng(7).integers(100, 10000, K))",
            "config": {
                "workload": wl["name"],
                "strategy": wl["strategy"],
                "clients": K,
                "clients_per_gpu": Kr,
                "params_per_gpu": M,
                "global_params": M_glob if (client_shard or args.scaling == "strong") else M * world,
                "layers": len(shapes),
                "parallelism": parallelism,
                "layout": f"tile-interleaved ({tv} vectors per client tile)" if tiled else "rows",
                "bytes_alg_per_step_job": bytes_job,
                "bytes_alg_per_launch_rank0": bytes_kernel,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_source": tsrc,
                "kernel": kname,
                "kernel_ms": round(kern_ms, 5),
                "kernel_ms_max_over_ranks": round(kern_ms_max, 5),
                "kernel_ms_median": round(float(np.median(each_ms)), 5),
                "kernel_ms_min": round(float(each_ms.min()), 5),
                "kernel_timing": "HIP events on the launch stream: timed region / steps" if not client_shard else
                                 "HIP events on the launch stream: this rank's block kernel alone, back to back",
                "read_stream_ceiling_GBps": round(read_ceiling, 1) if read_ceiling > 0 else None,
                "frac_of_read_ceiling": round(achieved / read_ceiling, 4) if read_ceiling > 0 else None,
            },
            "cpu_baseline": cpu,
            "parity": parity,
            "build": {"lib_sha256": sha},
        }
        if client_shard and world > 1:
            line["combine"] = {"mode": args.combine, "step_ms": round(ms_per_step, 5),
                               "block_kernel_ms": round(kern_ms_max, 5),
                               "exchange_and_final_ms": round(max(0.0, ms_per_step - kern_ms_max), 5),
                               "bit_exact_by_construction": args.combine in ("relay", "striped")}
            if striped:
                line["combine"]["stripes"] = [{"params": hi - lo, "hop": a} for lo, hi, a in bounds]
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def spot_check(torch, dist, world, rank, client_shard, scaffold, K, k0, k1, M, layout, n_samples, kind, device, env):
    """Sampled output elements against the reference's sequential order (fp32 FedAvg chain /
    fp64 Scaffold with c last and lr after the sum); client-sharded: every rank's sampled
    columns are gathered on the root.  numel == 1 elements are excluded here (pairwise order:
    tests/ check them against the oracle)."""
    from substrafl_amd.engine import fedavg_weights, scaffold_weights

    g = np.random.default_rng(123)
    idx = np.setdiff1d(np.unique(g.integers(0, M, 4096)), layout.pairwise_idx.astype(np.int64))
    tidx = torch.from_numpy(idx).to(device)
    Kr = k1 - k0

    def cols_striped(parts, field):
        """Striped relay: every rank holds a different block per stripe; gather each stripe's
        sampled columns from its holders and assemble [K, S] on the root."""
        from substrafl_amd.sharding import client_blocks, stripe_layout, stripe_rank

        lay = stripe_layout(M, K, world, rank)
        per = -(-K // world)
        sel = [np.nonzero((idx >= lo) & (idx < hi))[0] for lo, hi, *_ in lay]
        ni = max(1, max(len(x) for x in sel))
        pad = torch.zeros((len(lay), per, ni), dtype=torch.float64, device=device)
        for si, ((lo, hi, a, b, k0s, k1s), part) in enumerate(zip(lay, parts)):
            rows = getattr(part, field)
            if k1s > k0s and len(sel[si]):
                loc = torch.from_numpy(idx[sel[si]] - lo).to(device)
                pad[si, : k1s - k0s, : len(sel[si])] = rows[:, loc].to(torch.float64)
        got = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
        dist.gather(pad, gather_list=got, dst=0)
        if rank != 0:
            return None
        xs = np.zeros((K, idx.size))
        blocks = client_blocks(K, world)
        for si, (lo, hi, a, *_rest) in enumerate(lay):
            for b, (k0b, k1b) in enumerate(blocks):
                if k1b > k0b and len(sel[si]):
                    src = got[stripe_rank(b, world, a)][si, : k1b - k0b, : len(sel[si])].cpu().numpy()
                    xs[k0b:k1b, sel[si]] = src
        return xs

    def cols(x):  # [Kr, S] sampled columns of this rank's rows, gathered on the root in block order
        if isinstance(x, tuple):
            return cols_striped(*x)
        if env.get("tiled"):  # tile-interleaved buffer: gather each client's sampled elements
            from substrafl_amd.engine import tiled_index

            pos = tiled_index(kind, K, np.arange(K)[:, None], idx[None, :], env["tv"])
            return x[torch.from_numpy(pos.reshape(-1)).to(device)].view(K, -1).to(torch.float64).cpu().numpy()
        xs = x[:, tidx].to(torch.float64) if Kr else torch.zeros((0, idx.size), dtype=torch.float64, device=device)
        if not (client_shard and world > 1):
            return xs.cpu().numpy()
        from substrafl_amd.sharding import chain_rank, client_blocks

        per = -(-K // world)
        pad = torch.zeros((per, idx.size), dtype=torch.float64, device=device)
        pad[:Kr] = xs
        got = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
        dist.gather(pad, gather_list=got, dst=0)
        if rank != 0:
            return None
        blocks = client_blocks(K, world)
        return np.concatenate([got[chain_rank(b, world)][: blocks[b][1] - blocks[b][0]].cpu().numpy()
                               for b in range(world)], axis=0)

    def src(name, field):
        v = env[name]
        return (v, field) if isinstance(v, list) else v

    if not scaffold:
        xs = cols(src("clients", "rows"))
        if rank != 0 or xs is None:
            return None
        got = env["out"][tidx].cpu().numpy()
        w32 = fedavg_weights(n_samples, "f32")
        acc = np.zeros(idx.size, np.float32)
        for k in range(K if client_shard else xs.shape[0]):
            acc = (acc + (xs[k].astype(np.float32) * w32[k]).astype(np.float32)).astype(np.float32)
        bad = acc.view(np.uint32) != got.view(np.uint32)
        res = {"sampled": int(idx.size), "mismatches": int(np.sum(bad))}
        if bad.any():
            ia, ib = acc.view(np.int32).astype(np.int64), got.view(np.int32).astype(np.int64)
            res["max_ulp"] = int(np.max(np.abs(ia - ib)))
        return res
    xd, xc = cols(src("delta", "delta")), cols(src("cv", "cv"))
    if rank != 0 or xd is None:
        return None
    cc = env["c"][tidx].double().cpu().numpy()
    w64 = scaffold_weights(n_samples)
    ad = np.zeros(idx.size)
    ac = np.zeros(idx.size)
    for k in range(xd.shape[0]):
        ad = ad + xd[k] * w64[k]
        ac = ac + xc[k] * w64[k]
    ad = 1.0 * ad
    ac = ac + cc
    gd = env["dout"][tidx].cpu().numpy()
    gcv = env["cout"][tidx].cpu().numpy()
    return {"sampled": int(idx.size),
            "mismatches": int(np.sum(ad.view(np.uint64) != gd.view(np.uint64))
                              + np.sum(ac.view(np.uint64) != gcv.view(np.uint64)))}


def read_probe(torch, lib, src, stream, device, _native) -> float:
    """Best single-stream 16-B non-temporal read rate over the client buckets (up to 40 GB of
    them): the grid-strided probe at 2K..64K workgroups and the full grid, and the tile-walk probe
    (one workgroup per 4/8/16 x 256 contiguous vectors; tools/hbm_ceiling_probe.hip found it the
    fastest pattern, 7.1-7.2 TB/s over 32 GiB)."""
    probe_n = min(src.numel(), 40_000_000_000 // src.element_size())
    if probe_n < 4096:
        return 0.0
    nbytes_probe = probe_n * src.element_size()
    floats = nbytes_probe // 4 // 4 * 4
    full = int(min(floats // 4 // 256, 1 << 20))
    sink = torch.empty(max(1, full), dtype=torch.float32, device=device)
    ptr, sp, s = src.data_ptr(), sink.data_ptr(), stream.cuda_stream
    probes = [lambda g=g: lib.fedagg_read_probe_f32(ptr, floats, sp, g, s)
              for g in sorted({min(g, full) for g in (2048, 4096, 8192, 16384, 65536)} | {full}) if g > 0]
    probes += [lambda v=v: lib.fedagg_read_probe_tile_f32(ptr, floats, sp, v, s) for v in (4, 8, 16)]
    best = 0.0
    for probe in probes:
        for _ in range(3):
            _native.check(probe(), "probe")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            probe()
        e1.record(stream)
        torch.cuda.synchronize(device)
        best = max(best, floats * 4 / (e0.elapsed_time(e1) / 10 / 1e3) / 1e9)
    return best


# ======================================================================================
# --engine multi-device: the drop-in's one-process multi-GPU path (end-to-end line)
# ======================================================================================
def multi_device_bench(args):
    """MultiDeviceEngine over --gpus devices of ONE process (indices repeat on a box with fewer
    GPUs, one native session each): host buckets -> per-GPU pinned-ring staging over its PCIe
    link -> the bucket kernel -> D2H into the one output array.  Reports the PCIe-inclusive rate
    and, per shard, the stage / kernel / fetch split with the kernel timed by HIP events on the
    shard's session stream."""
    from substrafl_amd import _native
    from substrafl_amd.layout import synthetic_state_dict_shapes
    from substrafl_amd.multi_device import MultiDeviceEngine

    ndev = _native.load().fedagg_device_count()
    if ndev <= 0:
        print("bench.py: no GPU visible", file=sys.stderr)
        sys.exit(3)
    wl = WORKLOADS[args.workload]
    if wl["strategy"] != "fedavg" or wl["kind"] != "f32":
        print("bench.py: --engine multi-device runs the fp32 FedAvg workloads (c2, c3)", file=sys.stderr)
        sys.exit(2)
    K, M = wl["K"], wl["M"]
    devices = [g % ndev for g in range(args.gpus)]
    shapes = synthetic_state_dict_shapes(M)
    rng = np.random.default_rng(1)
    base = [rng.standard_normal(int(np.prod(s)), dtype=np.float32).reshape(s) for s in shapes]
    pus = [[(a * np.float32(1 + 0.01 * k)).astype(np.float32) for a in base] for k in range(K)]
    n_samples = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    eng = MultiDeviceEngine(devices)
    eng.kernel_events = True
    for _ in range(max(1, args.warmup)):
        eng.fedavg(pus, n_samples)
    walls, shards = [], []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        eng.fedavg(pus, n_samples)
        walls.append(time.perf_counter() - t0)
        shards.append(eng.last_timing["shards"])
    wall = float(np.median(walls))
    bytes_alg = K * M * 4 + M * 4
    per_shard = []
    for g in range(len(devices)):
        st = [s[g] for s in shards]
        lo, hi = eng.last_timing["ranges"][g][0][0], eng.last_timing["ranges"][g][-1][1]
        kms = float(np.median([s.get("kernel_ms", float("nan")) for s in st]))
        b = K * (hi - lo) * 4 + (hi - lo) * 4
        per_shard.append({"device": devices[g], "params": hi - lo, "layout": st[-1].get("layout"),
                          "stage_s": round(float(np.median([s["stage_s"] for s in st])), 5),
                          "kernel_fetch_s": round(float(np.median([s["kernel_fetch_s"] for s in st])), 5),
                          "kernel_ms": round(kms, 4),
                          "kernel_GBps_device_resident": round(b / (kms / 1e3) / 1e9, 1) if kms == kms else None})
    print(json.dumps({
        "metric": "aggregated-param GB/s (host buckets, PCIe-inclusive) FedAvg reduce, one process x N GPUs",
        "value": round(bytes_alg / wall / 1e9, 2), "unit": "GB/s", "n_gpus": len(devices),
        "distinct_gpus": len(set(devices)), "steps": args.steps, "warmup": args.warmup,
        "ms_per_call_median": round(wall * 1e3, 3), "higher_is_better": True, "dtype": "f32",
        "data": "synthetic host NumPy client states (per-layer arrays, N(0,1) scaled per client)",
        "config": {"workload": wl["name"], "clients": K, "params": M, "layers": len(shapes),
                   "engine": "MultiDeviceEngine (one process, one thread + native session per GPU)"},
        "shards": per_shard,
        "note": "end-to-end (pinned-ring pack + H2D + kernel + D2H); not the device-resident metric",
    }), flush=True)


# ======================================================================================
# --rehearse-cpu (tests): the launcher / rank / timing plumbing without a GPU
# ======================================================================================
def rehearse(args, world, rank):
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    x = np.ones(1 << 16, np.float32)
    for _ in range(args.warmup):
        x = x * np.float32(1.0)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x = x * np.float32(1.0)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
    if rank == 0:
        print(json.dumps({"metric": METRIC + " [CPU rehearsal of the launcher: not a measurement]",
                          "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 6),
                          "rehearsal": True, "ranks_seen": world}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(wl, budget_s, full=False):
    """Time the oracle's reference-call-structure FedAvg/Scaffold (list of products, np.sum) on a
    bounded host sample of the same workload shape (``full``: the workload's whole K x M; C3 is
    32 GB of client states, ~40 GB peak; C5 cannot be held by the reference on a box's host).
    NumPy's ufuncs are single-threaded here, so the reference path uses one core whatever the
    machine has."""
    from oracle import fedavg_reference_structure, scaffold_reference_structure
    from substrafl_amd.layout import synthetic_state_dict_shapes

    K = wl["K"]
    M_s = wl["M"] if full else min(wl["M"], 25_000_000 if K <= 16 else 4_000_000)
    shapes = synthetic_state_dict_shapes(M_s)
    rng = np.random.default_rng(1)
    base = [rng.standard_normal(s, dtype=np.float32) for s in shapes] if full else None
    counter = [0]

    def client():
        if base is not None:  # full size: distinct clients as scaled copies (no K x M random draws)
            counter[0] += 1
            return [(a * np.float32(1 + 1e-3 * counter[0])).astype(np.float32) for a in base]
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
    while len(times) < (2 if full else 3) or (time.perf_counter() < t_end and len(times) < 50):
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
        "sample": f"{'FULL SIZE: ' if full else ''}{K} clients x {M_s} fp32 params ({len(shapes)} layers), "
                  f"best of {len(times)} runs "
                  f"({best * 1e3:.1f} ms); oracle/aggregation.py reference call structure; "
                  f"host has {os.cpu_count()} cpus, affinity {aff}, NumPy ufuncs single-threaded",
    }


if __name__ == "__main__":
    main()
