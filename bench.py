#!/usr/bin/env python3
"""Device-resident aggregation throughput (BASELINE.json metric:
"aggregated-param GB/s (device-resident) FedAvg reduce, N clients x M params").

One step = one pass of the hot path over one batch of synthetic client buckets already resident
in HBM.  The default workload is BASELINE.json configs[2] on one MI355X: FedAvg, 64 clients x
125M fp32 params (C3) -- the configuration north_star's ">= 80 % of the single-GPU HBM-read
roofline" target is stated on.

Multi-GPU (one process per GPU).  ``--gpus N`` from a plain ``python3 bench.py`` starts the N rank
processes itself (before anything touches a GPU); under torchrun the ranks come from the
environment, and a WORLD_SIZE that differs from --gpus is an error.  The process group has a
finite timeout (``pg_kwargs``).  Modes:

* ``--mode param-range`` (default; SURVEY.md §8(e) primary, bit-exact): every rank reduces its own
  parameter range of all K clients -- no data-path collective.  ``--scaling weak`` (default): each
  rank owns a full M-param slice of an N*M-param model; ``--scaling strong``: the workload's own M
  is split over the N ranks (C3 at 64 x 125M over 8 GPUs = 15.6M params per GPU).  With N > 1 and
  one GPU per rank the SAME line also carries ``client_shard``: the north-star client-sharded
  mode timed right after, weak (every rank holds the workload's K clients, N*K in all), combine
  ``--combine`` (default striped) -- step time, block-kernel time, exchange time, GB/s, fraction
  of N x 8 TB/s, and weak efficiency against the parameter-range kernel time of one GPU -- and
  ``multi_device``: the drop-in's one-process MultiDeviceEngine over the same N GPUs (host
  buckets, PCIe-inclusive).
* ``--mode client-shard --combine relay|rccl|ordered|striped``: the client-sharded mode as the
  line itself.  ``relay`` and ``striped`` are bit-exact lockstep schedules over ONE communicator
  (substrafl_amd/lockstep.py); ``--scaling weak``: every rank holds the workload's K clients;
  ``--scaling strong``: the workload's K clients are split over the N ranks.  Needs one GPU per rank.
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
    ap.add_argument("--combine", default="striped", choices=["relay", "rccl", "ordered", "striped"],
                    help="client-shard combine (the N > 1 line's client_shard leg and --mode client-shard)")
    ap.add_argument("--client-shard", default="auto", choices=["auto", "off", "force"],
                    help="N > 1 param-range runs: also time the client-sharded (north-star) mode in the same "
                         "invocation (auto: when every rank has its own GPU; force: also at N = 1, a rehearsal "
                         "of the legs' plumbing on one GPU)")
    ap.add_argument("--client-shard-steps", type=int, default=50, help="timed steps of the client-shard leg")
    ap.add_argument("--multi-device-leg", default="auto", choices=["auto", "off", "force"],
                    help="N > 1: also time the drop-in's one-process MultiDeviceEngine over the N GPUs "
                         "(host buckets, PCIe-inclusive; rank 0 runs it in a child process)")
    ap.add_argument("--rings", type=int, default=0, help="striped: rings / chains (0 = the default: 6 Latin "
                    "chains at 8 ranks, 5 at 6, else up to 4 unit rings; lockstep.ring_chains)")
    ap.add_argument("--rounds", default="", help="striped: relative round sizes, e.g. 0.75,0.25 (default: three "
                    "rounds with the native executor, one with the Python one)")
    ap.add_argument("--variant-rounds", default="",
                    help="client-shard striped: also time these round splits (';'-separated, e.g. "
                         "'1.0;0.75,0.25') over the same communicator")
    ap.add_argument("--chunk", type=int, default=2 << 20, help="relay: elements per pipelined chunk")
    ap.add_argument("--gather-chunks", type=int, default=4,
                    help="gather leg: the pipelined variant cuts each rank's slice into this many chunks, "
                         "each gathered to rank 0 while the next is reduced (0: no pipelined variant)")
    ap.add_argument("--executor", default="native", choices=["native", "torch", "push", "gather"],
                    help="client-shard relay / striped: the native RCCL executor (csrc/lockstep.hip), the "
                         "Python schedule over torch.distributed's RCCL process group, or the push executor "
                         "(substrafl_amd/push.py: chain kernels storing into IPC-mapped peer slots, FedAvg fp32 / bf16 and Scaffold fp32 / fp64 rows); "
                         "gather (N > 1 line's param_range_strong_gather leg: the workload's M split over the ranks, "
                         "the result slices gathered to rank 0 over RCCL inside the timed step)")
    ap.add_argument("--client-shard-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--leg-key", default="", help=argparse.SUPPRESS)
    ap.add_argument("--md-pack-threads", type=int, default=0,
                    help="--engine multi-device: pack workers per GPU (0: CPUs allowed // GPUs, 2..32)")  # the leg a child runs (rehearsal)
    ap.add_argument("--rehearse-legs", action="store_true",
                    help="with --rehearse-cpu and N > 1: run the client-shard legs as child processes "
                         "(the N > 1 line's leg mechanism, its deadlines and failure handling) over gloo")
    ap.add_argument("--t1-ms", type=float, default=0.0, help=argparse.SUPPRESS)
    ap.add_argument("--engine", default="rank", choices=["rank", "multi-device"])
    ap.add_argument("--tile", type=int, default=0, help="tiles layout: 16-B vectors per client tile "
                    "(0: the library's choice; FEDAGG_TILE_VECTORS_*)")
    ap.add_argument("--layout", default="auto", choices=["rows", "tiles", "auto"],
                    help="client buckets in HBM: [K, ld] rows, tile-interleaved (fedagg_fedavg_tiled_*; "
                         "FedAvg fp32/bf16), or (default) tiles where the library recommends them -- the "
                         "layout the drop-in host path stages (AggregationEngine.tiled)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wait-quiet", action="store_true",
                    help="time at once, even while the driver still clears the previous process's freed device memory")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--grid-cap", type=int, default=0)
    ap.add_argument("--tune", default="", help="library launch knobs for experiments, key=value[,key=value] "
                    "(fedagg_tune; the default run sets none)")
    ap.add_argument("--nontemporal", type=int, default=-1)
    ap.add_argument("--traffic", default="", help="JSON with PMC-derived bytes per launch (profiles/)")
    ap.add_argument("--cpu-only", action="store_true",
                    help="run only the cpu_baseline leg (no GPU) and print its JSON")
    ap.add_argument("--cpu-full-size", action="store_true",
                    help="cpu_baseline over the workload's full K x M (default: when the host's free RAM holds it)")
    ap.add_argument("--cpu-sample", action="store_true",
                    help="cpu_baseline over a bounded sample (64/128 clients x 4M) even when the full size fits")
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
# process group (N > 1)
# ======================================================================================
PG_TIMEOUT_S = 300  # a stuck collective or exchange ends the rank instead of holding the lease
CLIENT_SHARD_DEADLINE_S = float(os.environ.get("BENCH_LEG_DEADLINE_S", "180"))  # one client-shard leg of an
# N > 1 line, set-up to spot check (normally 30-60 s)
# The whole N > 1 line (parameter-range value + its legs) finishes within this many seconds of the
# rank's start, under the driver's 600 s limit: each leg gets what is left of it (minus what the
# legs after it and the final line need), and a leg with too little left is skipped, not started.
LINE_BUDGET_S = float(os.environ.get("BENCH_LINE_BUDGET_S", "480"))
LEG_MIN_S = float(os.environ.get("BENCH_LEG_MIN_S", "45"))  # below this a leg cannot finish: skipped
# a leg's set-up (process group, RCCL communicator, IPC maps) through its warm-up steps (RCCL's lazy
# connect): its own deadline, apart from the timed part, so a leg stuck connecting costs this much
LEG_CONNECT_S = float(os.environ.get("BENCH_LEG_CONNECT_S", "90"))
LEG_READY = "BENCH_LEG_READY"  # a leg child's stdout line once its warm-up steps are done
_T_START = time.monotonic()


def line_time_left() -> float:
    """Seconds left of this rank's LINE_BUDGET_S."""
    return LINE_BUDGET_S - (time.monotonic() - _T_START)


def leg_deadline(cap: float, reserve: float) -> float:
    """The deadline of the next leg: at most ``cap``, and no later than the line budget minus
    ``reserve`` (what the legs after it and the final line need); 0 means skip the leg."""
    d = min(cap, line_time_left() - reserve)
    return d if d >= LEG_MIN_S else 0.0


def pg_kwargs() -> dict:
    """init_process_group options of every multi-rank run: a finite timeout (RCCL's watchdog
    aborts a communicator whose work exceeds it, with TORCH_NCCL_ASYNC_ERROR_HANDLING set below,
    so a hung rank fails instead of holding the GPUs until the driver's limit)."""
    from datetime import timedelta

    return {"timeout": timedelta(seconds=PG_TIMEOUT_S)}


def init_group(dist, world: int, device, nccl: bool) -> str:
    """gloo for the host-side barrier / max-over-ranks; with one GPU per rank also RCCL ("nccl")
    for device tensors -- the client-shard exchange (one communicator, sharding.DistTransport)."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")  # abort the communicators, raise in the rank
    backend = "cpu:gloo,cuda:nccl" if nccl else "gloo"
    kw = pg_kwargs()
    if nccl:
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)
    return backend


class _Ctx:
    """What every measurement of one rank needs."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, vals):
        if self.world == 1:
            return [float(v) for v in vals]
        t = self.torch.tensor([float(v) for v in vals], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return [float(v) for v in t]


QUIET_SOCCLK_MHZ = 200.0  # firmware-averaged SOC clock at or above this: the driver is clearing freed VRAM
QUIET_WAIT_MAX_S = 12.0  # a 288 GB clear at the measured ~38 GB/s takes ~7.5 s


def wait_device_quiet(dev_index: int, limit_s: float = QUIET_WAIT_MAX_S) -> dict:
    """Wait, bounded, until the kernel driver has finished clearing the device memory that the
    PREVIOUS process on this GPU freed.  The driver zeroes freed VRAM in the background at ~38 GB/s
    (a process that held 91 GB leaves ~2.5 s of it; 45 GB ~1 s; 8 GB ~0.1 s; none without device
    memory), and while it runs the SOC clock domain sits at its high level and HBM-bound launches
    are 2.0-2.5 % slower ("C5 per launch": profiles/r06s_*, r06q_*, r06r_*).  That is
    another process's cost, so the timed region starts after it; the line reports what was seen
    and waited (``device_quiet``).  The signal is amdsmi's gpu_metrics ``current_socclks``, the
    firmware's average (it decays over ~0.25 s once the clear ends); without amdsmi nothing is
    waited and the record says why."""
    rec = {"signal": "amdsmi gpu_metrics current_socclks (firmware-averaged MHz)", "threshold_mhz": QUIET_SOCCLK_MHZ}
    try:
        import amdsmi

        from substrafl_amd.runtime import device_pci_bus_id

        amdsmi.amdsmi_init()
    except Exception as e:  # noqa: BLE001 -- the measurement stands without it, labelled
        rec["skipped"] = f"{type(e).__name__}: {e}"[:200]
        return rec
    try:
        bdf = device_pci_bus_id(dev_index)
        handles = amdsmi.amdsmi_get_processor_handles()
        match = [h for h in handles if amdsmi.amdsmi_get_gpu_device_bdf(h).lower().endswith(bdf[-7:])]
        if not match:
            rec["skipped"] = f"no amdsmi handle for {bdf}"
            return rec

        def soc():
            v = amdsmi.amdsmi_get_gpu_metrics_info(match[0]).get("current_socclks")
            v = [x for x in v if isinstance(x, (int, float))] if isinstance(v, list) else [v]
            v = [float(x) for x in v if isinstance(x, (int, float)) and x < 0xFFFF]
            return sum(v) / len(v) if v else None

        t0 = time.perf_counter()
        first = cur = soc()
        while cur is not None and cur >= QUIET_SOCCLK_MHZ and time.perf_counter() - t0 < limit_s:
            time.sleep(0.02)
            cur = soc()
        rec.update(soc_clock_mhz_at_check=first, soc_clock_mhz_at_start=cur,
                   waited_s=round(time.perf_counter() - t0, 3),
                   gave_up=bool(cur is not None and cur >= QUIET_SOCCLK_MHZ))
    except Exception as e:  # noqa: BLE001
        rec["skipped"] = f"{type(e).__name__}: {e}"[:200]
    finally:
        try:
            amdsmi.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass
    return rec


def _timed(ctx, step, steps, warmup):
    """W untimed steps, then EXACTLY `steps` steps bracketed by a barrier + synchronize on both
    sides; returns this rank's wall time of the region and its HIP-event time.  Once per process,
    before the warm-up, waits for the driver's clear of the previous process's freed memory
    (wait_device_quiet; ``--no-wait-quiet`` skips it)."""
    torch = ctx.torch
    if getattr(ctx, "quiet", None) is None:
        ctx.quiet = wait_device_quiet(ctx.device.index) if getattr(ctx, "wait_quiet", True) else \
            {"skipped": "--no-wait-quiet"}
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(ctx.device)
    _leg_ready(ctx)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ctx.barrier()
    torch.cuda.synchronize(ctx.device)
    t0 = time.perf_counter()
    ev0.record(ctx.stream)
    for _ in range(steps):
        step()
    ev1.record(ctx.stream)
    torch.cuda.synchronize(ctx.device)
    elapsed = time.perf_counter() - t0
    ctx.barrier()
    return elapsed, ev0.elapsed_time(ev1)


def _leg_ready(ctx) -> None:
    """In a leg child (client_shard_legs): tell the parent the set-up and the warm-up steps are
    done (RCCL connected), once; the timed part has its own deadline from here."""
    if getattr(ctx, "leg_child", False) and not getattr(ctx, "_ready_sent", False):
        print(LEG_READY, flush=True)
        ctx._ready_sent = True


def run_leg_child(cmd, env, connect_s: float, deadline: float):
    """Run one leg child: it must print LEG_READY within ``connect_s`` (set-up + warm-up) and exit
    within ``deadline`` of its start; a child that misses either is killed (by PID) and the reason
    returned.  Returns (stdout, stderr, returncode, error or None, seconds to LEG_READY or None)."""
    import threading

    t_start = time.monotonic()
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    out, err, ready = [], [], threading.Event()
    ready_at = []

    def pump(stream, sink, watch):
        for ln in stream:
            sink.append(ln)
            if watch and ln.strip() == LEG_READY:
                ready_at.append(time.monotonic() - t_start)
                ready.set()

    th = [threading.Thread(target=pump, args=(p.stdout, out, True), daemon=True),
          threading.Thread(target=pump, args=(p.stderr, err, False), daemon=True)]
    for t in th:
        t.start()
    t0 = time.monotonic()
    why = None
    while p.poll() is None:
        if not ready.is_set() and time.monotonic() - t0 > min(connect_s, deadline):
            why = f"did not connect (set-up, RCCL connect, warm-up) within {min(connect_s, deadline):.0f} s"
        elif time.monotonic() - t0 > deadline:
            why = f"did not finish within {deadline:.0f} s"
        if why:
            p.kill()  # this rank's own child, by PID
            break
        time.sleep(0.05)
    p.wait()
    for t in th:
        t.join(timeout=5)
    return "".join(out), "".join(err), p.returncode, why, (round(ready_at[0], 2) if ready_at else None)


# ======================================================================================
# the rank path (device-resident metric)
# ======================================================================================
def main():
    args = parse()
    if args.cpu_only:
        print(json.dumps(cpu_baseline(WORKLOADS[args.workload], args.cpu_seconds, full=_cpu_full(args))), flush=True)
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
    own_gpus = world <= ndev
    # RCCL in the process group only where torch's process group carries the exchange itself
    torch_pg_exchange = (client_shard or args.client_shard_child) and args.executor in ("torch", "gather")
    backend = init_group(dist, world, device, world > 1 and own_gpus and torch_pg_exchange) if world > 1 else None
    lib = _native.load()
    if args.grid_cap:
        _native.tune(grid_cap=args.grid_cap)
    if args.nontemporal >= 0:
        _native.tune(nt_load=args.nontemporal)
    if args.tune:
        _native.tune(**{k: int(v) for k, v in (kv.split("=") for kv in args.tune.split(","))})
    ctx = _Ctx(torch=torch, dist=dist, world=world, rank=rank, device=device, lib=lib, native=_native,
               wl=WORKLOADS[args.workload], stream=torch.cuda.current_stream(device), backend=backend,
               leg_child=args.client_shard_child, physical_gpus=min(world, ndev), wait_quiet=not args.no_wait_quiet)

    if args.client_shard_child:  # one leg of an N > 1 line (see client_shard_legs)
        try:
            if args.executor == "gather":
                res = measure_param_range_gather(args, ctx, t1_ms=args.t1_ms or None)
            else:
                res = measure_client_shard(args, ctx, args.combine, args.scaling, t1_ms=args.t1_ms or None,
                                           t1_source="the parameter-range line's kernel (one GPU, the workload's K x M)")
        except Exception as e:  # noqa: BLE001 -- reported in the parent's line
            res = {"error": f"{type(e).__name__}: {e}"[:800]}
        if getattr(ctx, "quiet", None) is not None:
            res["device_quiet"] = ctx.quiet
        if args.executor == "torch" and world > 1 and "error" not in res:
            try:  # the xGMI rates the schedule model needs, measured on this node (tools/lockstep_model.py)
                res["xgmi_p2p"] = p2p_probe(torch, dist, rank, world, device, ctx.barrier, ctx.max_over_ranks)
            except Exception as e:  # noqa: BLE001
                res["xgmi_p2p"] = {"error": f"{type(e).__name__}: {e}"[:400]}
        if rank == 0:
            print(json.dumps(res), flush=True)
    elif client_shard:
        cs = measure_client_shard(args, ctx, args.combine or "relay", args.scaling)
        line = client_shard_line(args, ctx, cs)
    else:
        line, info = measure_param_range(args, ctx)
        if (world > 1 and args.client_shard == "auto") or args.client_shard == "force":
            if own_gpus:  # the north-star mode beside it: client buckets sharded, exchanged over xGMI
                line.update(client_shard_legs(args, ctx, info))
            else:
                line["client_shard"] = {"skipped": f"needs one GPU per rank for RCCL ({world} ranks, {ndev} GPUs)"}
                if args.client_shard == "force":  # the push leg needs no RCCL: rehearse it with ranks sharing GPUs
                    line.update(client_shard_legs(args, ctx, info, only_push=True))
        if own_gpus and ((world > 1 and args.multi_device_leg == "auto") or args.multi_device_leg == "force"):
            line["multi_device"] = multi_device_leg(args, ctx)
    if rank == 0 and not args.client_shard_child:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _cpu_full(args) -> bool:
    """The CPU baseline at the workload's full K x M when the host can hold it (the reference's
    NumPy path needs the K client lists plus a stacked copy: ~1.3 x K x M x 4 bytes)."""
    if args.cpu_full_size:
        return True
    if args.cpu_sample:
        return False
    wl = WORKLOADS[args.workload]
    if wl["kind"] == "bf16":  # C5: 179 GB of fp32 inputs for the reference; never on a host
        return False
    mult = 2 if wl["strategy"] == "scaffold" else 1
    need = int(1.5 * mult * wl["K"] * wl["M"] * 4) + (8 << 30)
    try:
        import psutil

        avail = psutil.virtual_memory().available
    except Exception:  # noqa: BLE001
        return False
    return avail > need


def measure_param_range(args, ctx):
    """The device-resident metric, one process per GPU, parameter-range sharding (no data-path
    collective): weak -- every rank reduces the workload's full K x M; strong -- the workload's
    M split over the ranks.  Returns (line, info)."""
    torch, world, rank, device = ctx.torch, ctx.world, ctx.rank, ctx.device
    from substrafl_amd.engine import (FedAvgPlan, ScaffoldPlan, TiledFedAvgPlan, fedavg_weights, scaffold_weights,
                                      tiled_recommended, tiled_tile)
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes
    from substrafl_amd.sharding import shard_bounds

    wl = ctx.wl
    K, M_glob, kind = wl["K"], wl["M"], wl["kind"]
    scaffold = wl["strategy"] == "scaffold"
    n_samples = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    s_in = 2 if kind == "bf16" else 4
    if args.scaling == "strong":
        lo, hi = shard_bounds(M_glob, world)[rank]
        M = hi - lo
        parallelism = f"param-range x{world} (strong)" if world > 1 else "single-gpu"
    else:
        M = M_glob
        parallelism = f"param-range x{world}" if world > 1 else "single-gpu"
    shapes = synthetic_state_dict_shapes(max(M, 1))
    layout = BucketLayout(list(range(len(shapes))), shapes, np.float32)
    ld = layout.ld
    pw = layout.pairwise_idx
    seed0 = 20241016 + 1_000_003 * rank
    stream = ctx.stream
    tiled = (not scaffold and kind in ("f32", "bf16")
             and (args.layout == "tiles" or (args.layout == "auto" and tiled_recommended(kind, K, M))))
    tv = (args.tile or tiled_tile(kind, K, M)) if tiled else 0
    if args.layout == "tiles" and not tiled:
        print("bench.py: --layout tiles takes the FedAvg fp32/bf16 workloads in param-range mode", file=sys.stderr)
        sys.exit(2)
    env = {"tiled": tiled, "tv": tv}
    if not scaffold:
        clients = synth_tiled(torch, K, M, kind, device, seed0, tv) if tiled else \
            synth_clients(torch, K, ld, M, kind, device, seed0)
        out = torch.empty(ld, dtype=torch.float32, device=device)
        w_all = fedavg_weights(n_samples, kind)
        plan = TiledFedAvgPlan(kind, clients, K, w_all, M, out, pw, tv=tv) if tiled else \
            FedAvgPlan(kind, clients, w_all, M, out, pw)
        env.update(clients=clients, out=out)
    else:
        delta = synth_clients(torch, K, ld, M, kind, device, seed0)
        cv = synth_clients(torch, K, ld, M, kind, device, seed0 + 7919)
        gc = torch.Generator(device=device)
        gc.manual_seed(4242)
        c = torch.randn(ld, dtype=torch.float32, device=device, generator=gc)
        dout = torch.empty(ld, dtype=torch.float64, device=device)
        cout = torch.empty(ld, dtype=torch.float64, device=device)
        plan = ScaffoldPlan(kind, delta, cv, c, scaffold_weights(n_samples), M, 1.0, dout, cout, pw)
        env.update(delta=delta, cv=cv, c=c, dout=dout, cout=cout)
    bytes_kernel = plan.bytes_alg()
    bytes_job = bytes_kernel * world if args.scaling == "weak" else (
        K * M_glob * s_in + M_glob * 4 if not scaffold else 2 * K * M_glob * 4 + M_glob * 4 + 2 * M_glob * 8)

    def step():
        plan.launch(stream)

    elapsed, ev_ms = _timed(ctx, step, args.steps, args.warmup)
    kern_ms = ev_ms / args.steps  # the step IS the one kernel, launched back to back
    # the kernel alone, launch by launch (HIP events on its stream): median / min for the spread
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(max(5, min(args.steps, 20)))]
    for a, b in evs:
        a.record(stream)
        plan.launch(stream)
        b.record(stream)
    torch.cuda.synchronize(device)
    each_ms = np.array([a.elapsed_time(b) for a, b in evs])
    elapsed, kern_ms_max = ctx.max_over_ranks([elapsed, kern_ms])
    ms_per_step = elapsed / args.steps * 1e3
    value = bytes_job / (elapsed / args.steps) / 1e9

    parity = spot_check(torch, world, rank, scaffold, K, M, layout, n_samples, kind, device, env)
    read_ceiling = read_probe(torch, ctx.lib, env["clients"] if not scaffold else env["delta"], stream, device,
                              ctx.native)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(wl, args.cpu_seconds, full=_cpu_full(args))
    sha = lib_sha256()
    traffic, tsrc = read_traffic(args, sha) if (world == 1 or args.scaling == "weak") else (None, None)
    achieved = bytes_kernel / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else 0.0
    if not scaffold:
        kname = f"fedavg_kernel<{'BF16' if kind == 'bf16' else 'F32'}>"
    elif ctx.lib.fedagg_scaffold_launches(max(1, K), 4, M, 1) == 2:  # the library's own launch plan
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
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "bf16-in/f32-acc" if kind == "bf16" else ("f32-in/f64-acc" if scaffold else "f32"),
        "data": "synthetic (N(0,1) client buckets generated on device, torch Philox seeds 20241016+k; "
                "n_samples = default_rng(7).integers(100, 10000, K))",
        "config": {
            # N > 1 weak: every rank reduces its own K x M (an N x M-param model, no bytes between
            # GPUs) -- per GPU the workload; BASELINE's C3 as written (M split over the GPUs, the
            # result gathered to rank 0) is the param_range_strong_gather leg of the same line
            "workload": wl["name"] + ("_per_gpu" if world > 1 and args.scaling == "weak" else ""),
            "strategy": wl["strategy"],
            "clients": K,
            "clients_per_gpu": K,
            "params_per_gpu": M,
            "global_params": M_glob if args.scaling == "strong" else M * world,
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
            "kernel_timing": "HIP events on the launch stream: timed region / steps",
            "read_stream_ceiling_GBps": round(read_ceiling, 1) if read_ceiling > 0 else None,
            "frac_of_read_ceiling": round(achieved / read_ceiling, 4) if read_ceiling > 0 else None,
        },
        "cpu_baseline": cpu,
        "parity": parity,
        "build": {"lib_sha256": sha},
        "device_quiet": getattr(ctx, "quiet", None),
    }
    if world > 1:
        line["process_group"] = {"backend": ctx.backend, "timeout_s": PG_TIMEOUT_S}
        # the job's fraction of N x 8 TB/s (the driver computes T(1)/T(N) itself)
        line["frac_of_n_x_hbm_peak"] = round(value / (world * HBM_PEAK_GBPS), 4)
    _label_shared_gpu(ctx, line, ("value", "frac_of_n_x_hbm_peak"))
    return line, {"kern_ms": kern_ms_max, "K": K, "M": M, "tiled": tiled}


def _label_shared_gpu(ctx, rec: dict, keys) -> None:
    """Ranks sharing one GPU (a rehearsal on a box with fewer GPUs than ranks) measure the
    protocol, not scaling: record the physical GPU count and null the aggregate-rate fields, so
    such a line can never read as an N-GPU scaling record."""
    phys = getattr(ctx, "physical_gpus", ctx.world)
    if phys >= ctx.world:
        return
    rec["physical_gpus"] = phys
    rec["shared_gpu"] = f"{ctx.world} ranks on {phys} GPU(s): a rehearsal of the N > 1 path, no scaling information"
    for k in keys:
        if k in rec:
            rec[k] = None


MULTI_DEVICE_DEADLINE_S = 180


def multi_device_leg(args, ctx):
    """The N > 1 line's ``multi_device`` field: the drop-in's own multi-GPU path, ONE process driving
    the N GPUs (MultiDeviceEngine: host buckets staged over each GPU's PCIe link, reduced, fetched
    into one host array -- the PCIe-inclusive rate of the aggregate task), run by rank 0 as a child
    process while the other ranks wait at the barrier (their buffers freed).  fp32 FedAvg workloads
    (C2, C3); an error or a timeout becomes an ``error`` field."""
    wl = ctx.wl
    res = None
    if ctx.rank == 0:
        if wl["strategy"] != "fedavg" or wl["kind"] != "f32":
            res = {"skipped": "the multi-device engine leg runs the fp32 FedAvg workloads (c2, c3)"}
        else:
            env = {k: v for k, v in os.environ.items()
                   if not k.startswith("TORCHELASTIC") and k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                                     "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT")}
            cmd = [sys.executable, str(Path(__file__).resolve()), "--engine", "multi-device", "--gpus", str(ctx.world),
                   "--workload", args.workload, "--steps", "5", "--warmup", "1"]
            deadline = leg_deadline(MULTI_DEVICE_DEADLINE_S, 15)
            t0 = time.perf_counter()
            if not deadline:
                res = {"skipped": f"line time budget ({LINE_BUDGET_S:.0f} s) spent: {line_time_left():.0f} s left"}
            else:
                p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                try:
                    so, se = p.communicate(timeout=deadline)
                    lines = [ln for ln in so.splitlines() if ln.startswith("{")]
                    if p.returncode != 0 or not lines:
                        res = {"error": f"leg exited with {p.returncode}: {se[-600:]}"}
                    else:
                        res = json.loads(lines[-1])
                except subprocess.TimeoutExpired:
                    p.kill()  # our own child, by PID
                    p.communicate()
                    res = {"error": f"did not finish within {deadline:.0f} s"}
            res["wall_s"] = round(time.perf_counter() - t0, 1)
    ctx.barrier()
    return res


# ======================================================================================
# client-shard (the north-star mode) -- its own line, or a field of the N > 1 line
# ======================================================================================
# (executor, scaling, line key, extra environment, extra arguments), in the order the N > 1 line
# runs them (client_shard_legs): the decisive comparison first -- the push executor,
# whose full output is compared with the native executor's on the same client blocks, and the
# native weak leg -- then C3 as written (M split over the GPUs, the result gathered to rank 0 over
# RCCL inside the step), then the rest
LEGS = (("push", "weak", "client_shard_push", {}, []),
        ("native", "weak", "client_shard", {}, ["--variant-rounds", "1.0;0.75,0.25"]),
        ("gather", "strong", "param_range_strong_gather", {}, []),
        ("torch", "weak", "client_shard_torch_pg", {}, []),
        ("native", "strong", "client_shard_strong", {}, []),
        ("native", "weak", "client_shard_copy_engine", {"NCCL_P2P_USE_CUDA_MEMCPY": "1"}, []))


def client_shard_legs(args, ctx, info, only_push=False):
    """The client-shard legs of an N > 1 line, each in a CHILD process per rank (a fresh
    interpreter with its own process group on a new port, started once this rank's parameter-range
    buffers are freed): ``client_shard`` with the native RCCL executor, ``client_shard_torch_pg``
    with the Python schedule over torch's RCCL process group.  A leg that fails, crashes or exceeds
    its deadline becomes an ``error`` field -- it can never cost the line.  Deadlines: rank 0's
    ``leg_deadline`` (CLIENT_SHARD_DEADLINE_S within the line budget, keeping room for the legs
    after it), broadcast so every rank agrees; within it, the set-up through the warm-up steps has
    its own LEG_CONNECT_S (run_leg_child), so a leg stuck in RCCL's connect costs that, not the
    leg's budget.  A leg that timed out does not cancel the next one (the two executors share
    RCCL's bootstrap but not its exchange code); the budget bounds both.  A failure of the host
    group itself ends the loop, keeping every leg gathered before it."""
    torch, dist = ctx.torch, ctx.dist
    torch.cuda.empty_cache()
    # weak (every rank holds the workload's K clients: north_star's scaling target) with both
    # executors, then strong (the workload's K clients split over the ranks: BASELINE.json's C3
    # as written, "64 clients ... sharded across 8 MI355X" -- the xGMI-bound regime)
    # ... and the native weak leg again with RCCL's copy-engine P2P path (NCCL_P2P_USE_CUDA_MEMCPY:
    # the xGMI bytes moved by SDMA engines instead of RCCL's CU kernels).  On one GPU, RCCL's P2P
    # kernels hide only ~0.3 of their time under an HBM-saturating chain kernel while SDMA copies
    # hide 0.87-1.0 (tools/executor_overlap_probe.py, profiles/r03m_executor_overlap_probe*.jsonl):
    # the two weak legs side by side show which engine the node's exchange should use.
    # (last, and with a shorter deadline: RCCL's copy-engine path has never run on this node)
    # The native weak leg also re-times the other round splits over its communicator
    # (rounds_variants): the model's choice of three rounds assumes full overlap.
    # the decisive comparison first: the push executor (its full output compared
    # with the native executor's on the same client blocks) and the native weak leg, then C3 as
    # written (M split over the GPUs, the result gathered to rank 0 over RCCL inside the step),
    # then the rest
    legs = LEGS
    if only_push:
        legs = tuple(leg for leg in legs if leg[0] == "push")
    md_reserve = MULTI_DEVICE_DEADLINE_S if args.multi_device_leg != "off" else 0
    out = {"legs_order": [leg[2] for leg in legs]}
    ports = [[_free_port() for _ in legs]] if ctx.rank == 0 else [None]
    if ctx.world > 1:
        dist.broadcast_object_list(ports, src=0)
    for i, ((executor, scaling, key, leg_env, leg_args), port) in enumerate(zip(legs, ports[0])):
        later = (len(legs) - 1 - i) * LEG_MIN_S + min(md_reserve, LEG_MIN_S) + 15
        cap = CLIENT_SHARD_DEADLINE_S if not (leg_env or executor in ("push", "gather")) else CLIENT_SHARD_DEADLINE_S / 2
        dl = [leg_deadline(cap, later)] if ctx.rank == 0 else [None]
        if ctx.world > 1:
            dist.broadcast_object_list(dl, src=0)
        deadline = dl[0]
        if not deadline:
            if ctx.rank == 0:
                out[key] = {"skipped": f"line time budget ({LINE_BUDGET_S:.0f} s): {line_time_left():.0f} s left",
                            "executor": executor}
            continue
        env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC")}
        env.update(RANK=str(ctx.rank), WORLD_SIZE=str(ctx.world), LOCAL_RANK=str(ctx.device.index),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # one node: RCCL's bootstrap over loopback (its P2P data path is xGMI either way), so an
        # interface the container cannot route never stalls ncclCommInitRank
        env.setdefault("NCCL_SOCKET_IFNAME", "lo")
        env.update(leg_env)
        cmd = [sys.executable, str(Path(__file__).resolve()), "--client-shard-child", "--executor", executor,
               "--scaling", scaling,
               "--gpus", str(ctx.world), "--workload", args.workload, "--combine", args.combine or "striped",
               "--layout", args.layout, "--steps", str(args.client_shard_steps), "--warmup", "3",
               "--client-shard-steps", str(args.client_shard_steps), "--t1-ms", str(info["kern_ms"]),
               "--chunk", str(args.chunk), "--rings", str(args.rings), "--no-cpu-baseline", *leg_args]
        if args.rounds:
            cmd += ["--rounds", args.rounds]
        elif scaling == "strong":  # exchange-bound: one round is the fastest (tools/lockstep_model.py)
            cmd += ["--rounds", "1.0"]
        if getattr(args, "rehearse_cpu", False):
            cmd += ["--rehearse-cpu", "--leg-key", key]
        t0 = time.perf_counter()
        try:
            so, se, rc, why, ready_s = run_leg_child(cmd, env, LEG_CONNECT_S, deadline)
            res = None
            if why:
                res = {"error": why}
            elif ctx.rank == 0:
                lines = [ln for ln in so.splitlines() if ln.startswith("{")]
                res = json.loads(lines[-1]) if lines else None
            if not why and rc != 0:
                res = {"error": f"leg exited with {rc}: {se[-600:]}"}
            elif not why and ctx.rank == 0 and res is None:
                res = {"error": f"no result line: {se[-600:]}"}
            if res is not None:
                res["wall_s"] = round(time.perf_counter() - t0, 1)
                res["executor"] = executor
                if leg_env:
                    res["env"] = dict(leg_env)
            # every rank's leg is over before the next one starts (errors and set-up times are per
            # rank: gather them)
            mine = ((res or {}).get("error"), ready_s)
            got = [mine] * ctx.world
            if ctx.world > 1:
                dist.all_gather_object(got, mine)
            errs = [g[0] for g in got]
            if ctx.rank == 0:
                bad = {r: e for r, e in enumerate(errs) if e}
                if bad and "error" not in res:
                    res["errors_on_other_ranks"] = bad
                # the leg's set-up through its warm-up steps (process start, process group, RCCL
                # connect, warm-up), slowest rank, beside the deadline it had (VERDICT r05 "Next 1")
                ready = [g[1] for g in got if g[1] is not None]
                res["connect_s"] = max(ready) if len(ready) == ctx.world else None
                res["connect_deadline_s"] = round(min(LEG_CONNECT_S, deadline), 1)
                res["deadline_s"] = round(deadline, 1)
                out[key] = res
        except Exception as e:  # noqa: BLE001 -- a leg never costs the legs gathered before it
            if ctx.rank == 0:
                out[key] = {"error": f"{type(e).__name__}: {e}"[:600], "executor": executor}
            break  # the host group itself failed: no later leg could meet its peers
    if ctx.rank == 0:  # every weak leg reduced the same K x M values: one expected output
        sums = {k: v.get("output_checksum") for k, v in out.items()
                if isinstance(v, dict) and v.get("scaling") == "weak" and v.get("checksum_comparable")
                and v.get("output_checksum") is not None}
        # agreement needs two legs at least: one leg agrees with nothing (null, not true)
        out["client_shard_output_checksums"] = {"legs": sorted(sums), "agree": len({tuple(c) for c in sums.values()}) == 1
                                                if len(sums) >= 2 else None}
    return out


def _elem_hash(torch, kk, e):
    """fp32 values in [-1, 1) hashed from (client index ``kk`` [Kb, 1], global element ``e`` [1, n])."""
    h = (e * 2654435761 + kk * 40503 + 12345) & 0xFFFFFFFF
    h = ((h ^ (h >> 15)) * 2246822519) & 0xFFFFFFFF
    h = ((h ^ (h >> 13)) * 3266489917) & 0xFFFFFFFF
    h = h ^ (h >> 16)
    return ((h & 0xFFFFFF).to(torch.float32) - 8388608.0) * (1.0 / 8388608.0)


def _synth_block_elems(torch, kind, k0, Kb, width, segs, device):
    """A client block's row buffer whose value at (client k, global element e) is a hash of (k, e)
    in [-1, 1): the same wherever a plan puts (k, e) -- so every weak client-shard leg (push,
    native, torch, copy-engine, any round split, rows or tiles) reduces the very same K x M
    problem and their full outputs must agree bit for bit (``output_checksum``)."""
    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f64": torch.float64}[kind]
    t = torch.zeros((max(1, Kb), max(1, width)), dtype=dt, device=device)
    if Kb == 0:
        return t[:0, :width]
    kk = torch.arange(k0, k0 + Kb, device=device, dtype=torch.int64)[:, None]
    step = 1 << 20
    for lo, hi, col in segs:
        for a in range(lo, hi, step):
            b = min(hi, a + step)
            e = torch.arange(a, b, device=device, dtype=torch.int64)[None, :]
            t[:Kb, col + a - lo: col + b - lo] = _elem_hash(torch, kk, e).to(dt)
    return t[:Kb, :width]


def _synth_tiled_elems(torch, kind, k0, Kb, width, segs, tv, ext, device):
    """The tile-interleaved form of :func:`_synth_block_elems` (sharding.TiledBlock, one bucket per
    run), filled run by run in tile chunks: the same (client, element) values, so a tiled leg's
    output is comparable with the row legs' by checksum."""
    from substrafl_amd.engine import _ELEMS_PER_VEC
    from substrafl_amd.sharding import TiledBlock

    blk = TiledBlock.empty(torch, kind, Kb, width, tv, ext, device)
    TL = int(tv) * _ELEMS_PER_VEC[kind]
    kk = torch.arange(k0, k0 + Kb, device=device, dtype=torch.int64)[:, None]
    chunk = max(1, (1 << 20) // TL)  # tiles per fill
    for c0, (t, n) in blk.buckets.items():
        tiles = -(-n // TL)
        tv3 = t.view(tiles, Kb, TL)
        for j0 in range(0, tiles, chunk):
            j1 = min(tiles, j0 + chunk)
            colpos = torch.arange(c0 + j0 * TL, c0 + j1 * TL, device=device, dtype=torch.int64)
            glob = torch.full_like(colpos, -1)
            for lo, hi, col in segs:
                m = (colpos >= col) & (colpos < col + hi - lo) & (colpos < c0 + n)
                glob[m] = lo + colpos[m] - col
            v = _elem_hash(torch, kk, glob[None, :].clamp(min=0))
            v[:, glob < 0] = 0.0  # the last tile's padding
            tv3[j0:j1].copy_(v.to(t.dtype).view(Kb, j1 - j0, TL).permute(1, 0, 2))
    return blk


def _output_checksum(torch, out, M):
    """Two sums of the output's bit patterns (plain, and position-weighted so a permutation shows)."""
    x = out[:M].contiguous().view(torch.int32).to(torch.int64)
    w = torch.arange(M, device=out.device, dtype=torch.int64) % 1021 + 1
    return [int(x.sum().item()), int((x * w).sum().item())]


def _synth_block(torch, kind, Kb, width, device, seed):
    """A client block's buffer: N(0,1) from torch's device Philox stream (bf16 via fp32)."""
    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f64": torch.float64}[kind]
    t = torch.empty((max(1, Kb), max(1, width)), dtype=dt, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    for k in range(Kb):
        if kind == "bf16":
            t[k].copy_(torch.randn(width, generator=g, device=device, dtype=torch.float32))
        else:
            t[k].normal_(generator=g)
    return t[:Kb, :width]


def measure_client_shard(args, ctx, combine, scaling, t1_ms=None, t1_source=None, tr=None, variants=True):
    """One rank's part of the client-sharded reduction (sharding.py; relay / striped: the
    lockstep schedule over ONE communicator, rccl / ordered: re-associating), device-resident,
    timed like the main line; returns the measurement as a dict (rank 0's is reported).
    ``--variant-rounds`` (striped): the same leg re-timed over the same communicator with each
    listed round split (``rounds_variants``; no spot check: the schedules' parity is the tests')."""
    torch, world, rank, device = ctx.torch, ctx.world, ctx.rank, ctx.device
    from substrafl_amd import lockstep
    from substrafl_amd.engine import (FedAvgPlan, ScaffoldPlan, TiledFedAvgPlan, fedavg_weights, scaffold_weights,
                                      tiled_recommended, tiled_tile)
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes
    from substrafl_amd.sharding import (SLOTS, DistTransport, FedAvgShard, GpuShardOps, LoopbackGroup, ScaffoldShard,
                                        TiledBlock, _block_layout, block_of, client_blocks, client_shard_fedavg,
                                        client_shard_scaffold, lockstep_fedavg, lockstep_scaffold, relay_plan,
                                        striped_plan)

    wl = ctx.wl
    K_per, M, kind = wl["K"], wl["M"], wl["kind"]
    scaffold = wl["strategy"] == "scaffold"
    K = K_per * world if scaling == "weak" else K_per
    n_samples = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    s_in = 2 if kind == "bf16" else 4
    shapes = synthetic_state_dict_shapes(M)
    layout = BucketLayout(list(range(len(shapes))), shapes, np.float32)
    pw = layout.pairwise_idx
    lockstep_mode = combine in ("relay", "striped")
    if tr is not None:
        pass
    elif world == 1:
        tr = LoopbackGroup(1).transport(0)
    elif args.executor in ("native", "push"):
        if not lockstep_mode:
            raise ValueError(f"the {args.executor} executor runs the lockstep schedules (relay, striped), not {combine}")
        if args.executor == "push":
            from substrafl_amd.push import PushTransport

            tr = PushTransport()
        else:
            from substrafl_amd.rccl import RcclTransport

            tr = RcclTransport()
    else:
        tr = DistTransport()
    ops = GpuShardOps()
    stream = ctx.stream
    mode = {"auto": "auto", "tiles": True, "rows": False}[args.layout] if args.executor != "push" else False
    w_all = fedavg_weights(n_samples, kind) if not scaffold else scaffold_weights(n_samples)
    gc = torch.Generator(device=device)
    gc.manual_seed(4242)
    c = torch.randn(layout.ld, dtype=torch.float32, device=device, generator=gc) if scaffold else None
    outs = {}
    if not scaffold:
        outs["out"] = torch.zeros(layout.ld, dtype=torch.float32, device=device)
    else:
        outs["dout"] = torch.zeros(layout.ld, dtype=torch.float64, device=device)
        outs["cout"] = torch.zeros(layout.ld, dtype=torch.float64, device=device)
    held = {}  # block -> (k0, data, segs) for the spot check
    tvs = set()
    if lockstep_mode:
        plan = striped_plan(M, world, rank, args.rings or None, _rounds(args)) if combine == "striped" else \
            relay_plan(M, world, rank, args.chunk)
        blocks = {}
        for b, segs in plan.blocks.items():
            k0, k1 = client_blocks(K, world)[b]
            seed = 20241016 + 104729 * b + 7919 * rank
            width = plan.block_len[b]
            if scaffold:
                d = _synth_block(torch, kind, k1 - k0, width, device, seed)
                v = _synth_block(torch, kind, k1 - k0, width, device, seed + 1)
                blocks[b] = ScaffoldShard(kind, d, v, None, w_all[k0:k1], k0, K, width, 1.0, np.zeros(0, np.uint64))
                held[b] = (k0, (d, v), segs)
                continue
            ext = TiledBlock.run_extents(plan, b)
            tv = _block_layout(torch, kind, k1 - k0, ext, mode)
            if tv:  # tiles: the same (client, element) values as the row legs, re-tiled per run
                rows = _synth_tiled_elems(torch, kind, k0, k1 - k0, width, segs, tv, ext, device)
                tvs.add(tv)
            else:  # rows: values addressed by (client, element), the same in every leg and round split
                rows = _synth_block_elems(torch, kind, k0, k1 - k0, width, segs, device)
                tvs.add(0)
            blocks[b] = FedAvgShard(kind, rows, w_all[k0:k1], k0, K, width, np.zeros(0, np.uint64))
            held[b] = (k0, rows, segs)
        slots = torch.empty(2 * SLOTS * max(1, plan.slot_elems), dtype=torch.float64 if scaffold else torch.float32,
                            device=device)
        ws = (torch.zeros(max(1, pw.size) * (2 * K + 1), dtype=torch.float64, device=device) if scaffold else
              torch.zeros((max(1, pw.size), K), dtype=torch.float32, device=device))

        def step():
            if scaffold:
                lockstep_scaffold(plan, blocks, outs["dout"], outs["cout"], tr, ops, pw, c, 1.0, ws=ws, slots=slots)
            else:
                lockstep_fedavg(plan, blocks, outs["out"], tr, ops, pw, ws=ws, slots=slots)

        acc = slots.view(-1)
        slot_n = max(1, plan.slot_elems)

        def compute_only():  # every run of this rank back to back, no exchange (the block kernel time)
            for runs in plan.runs:
                for r in runs:
                    sh = blocks[r.block]
                    if r.acc[0] == "out":  # the root's final runs accumulate in the output itself
                        a = (outs["dout"] if scaffold else outs["out"])[r.acc[2]: r.acc[2] + r.n]
                        a2 = outs["cout"][r.acc[2]: r.acc[2] + r.n] if scaffold else None
                    else:
                        a = acc[r.acc[1] * slot_n + r.acc[2]:][: r.n]
                        a2 = acc[(SLOTS + r.acc[1]) * slot_n + r.acc[2]:][: r.n] if scaffold else None
                    if scaffold:
                        ops.scaffold_run(kind, sh.delta[:, r.col: r.col + r.n], sh.cv[:, r.col: r.col + r.n], sh.w,
                                         r.seed, r.final, c[r.lo: r.lo + r.n], 1.0, a, a2)
                    else:
                        ops.fedavg_run(kind, sh.rows[:, r.col: r.col + r.n], sh.w, r.seed, a)

        run_bytes = sum((blocks[r.block].Kr * r.n * s_in * (2 if scaffold else 1)
                         + r.n * (8 if scaffold else 4) * (2 if scaffold else 1) * (1 if r.seed else 2))
                        for runs in plan.runs for r in runs)
        schedule = {"steps": plan.n_steps, "runs_per_rank": sum(len(x) for x in plan.runs),
                    "messages_per_rank": plan.stats.get("messages_of_this_rank"),
                    "elements_per_run": sorted({r.n for runs in plan.runs for r in runs})[-1:],
                    "issue": "one host thread, one communicator; exchange group t pairs only with group t of the peers"}
        if combine == "striped":
            schedule["rings"] = len(lockstep.ring_chains(world, args.rings or None))
            schedule["ring_hops"] = lockstep.ring_hops(world, args.rings or None)
            schedule["rounds"] = list(_rounds(args))
    else:
        k0, k1 = client_blocks(K, world)[block_of(rank, world)]
        Kr = k1 - k0
        seed = 20241016 + 104729 * block_of(rank, world)
        if scaffold:
            d = _synth_block(torch, kind, Kr, layout.ld, device, seed)
            v = _synth_block(torch, kind, Kr, layout.ld, device, seed + 1)
            sh = ScaffoldShard(kind, d, v, c, w_all[k0:k1], k0, K, M, 1.0, pw)
            held[block_of(rank, world)] = (k0, (d, v), [(0, M, 0)])
        else:
            rows = _synth_block(torch, kind, Kr, layout.ld, device, seed)
            sh = FedAvgShard(kind, rows, w_all[k0:k1], k0, K, M, pw)
            held[block_of(rank, world)] = (k0, rows, [(0, M, 0)])
        tvs.add(0)

        def step():
            if scaffold:
                client_shard_scaffold(sh, outs["dout"], outs["cout"], tr, ops, combine)
            else:
                client_shard_fedavg(sh, outs["out"], tr, ops, combine)

        def compute_only():
            if scaffold:
                ops.scaffold_chain(sh, 0, M, True, False, outs["dout"], outs["cout"])
            else:
                ops.fedavg_chain(kind, sh.rows, sh.w, 0, M, True, outs["out"])

        run_bytes = Kr * M * s_in * (2 if scaffold else 1) + M * (16 if scaffold else 4)
        schedule = {"issue": "dist.reduce per chunk (rccl) / dist.gather (ordered) on one communicator"}

    steps = max(1, min(args.steps, args.client_shard_steps))
    warm = max(1, min(args.warmup, 5))
    elapsed, _ev = _timed(ctx, step, steps, warm)
    # the block kernels alone, back to back (HIP events on their stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    compute_only()
    e0.record(stream)
    for _ in range(3):
        compute_only()
    e1.record(stream)
    torch.cuda.synchronize(device)
    block_ms = e0.elapsed_time(e1) / 3
    step()  # the outputs again (compute_only overwrote the root's final runs)
    torch.cuda.synchronize(device)
    parity = _client_shard_spot_check(ctx, K, M, layout, n_samples, kind, scaffold, held, outs, c, tvs) \
        if variants else None
    full_compare = None
    if variants and getattr(tr, "push", False) and world > 1 and lockstep_mode:
        # every element (numel == 1 ones included) against a second, independent transport
        full_compare = _push_vs_native(ctx, plan, blocks, outs, ops, pw, ws, slots, M, c if scaffold else None)
    # the whole output, summarised: every weak leg holds the same (client, element) values (rows),
    # so their checksums must be equal (client_shard_legs compares them across the legs)
    comparable = not scaffold and lockstep_mode  # rows and tiles hold the same (client, element) values
    checksum = _output_checksum(torch, outs["out"], M) if (not scaffold and rank == 0) else None
    if t1_ms is None:  # one GPU reducing the workload's own K x M: the weak-scaling reference
        t1_ms, t1_source = _single_gpu_ms(ctx, K_per, M, kind, scaffold, layout, n_samples), \
            "this rank, one GPU over the workload's K x M (same bench, same layout policy)"
    elapsed, block_ms, t1_ms = ctx.max_over_ranks([elapsed, block_ms, t1_ms])
    ms = elapsed / steps * 1e3
    bytes_job = (K * M * s_in + M * 4) if not scaffold else (2 * K * M * 4 + M * 4 + 2 * M * 8)
    gbps = bytes_job / (ms / 1e3) / 1e9
    layouts = sorted(tvs)
    res = {
        "combine": combine,
        "scaling": scaling,
        "clients": K,
        "clients_per_gpu": K // world if scaling == "weak" else -(-K // world),
        "params": M,
        "layout": "rows" if layouts == [0] else ", ".join(
            "rows" if t == 0 else f"tile-interleaved ({t} vectors per client tile)" for t in layouts),
        "steps": steps,
        "warmup": warm,
        "ms_per_step": round(ms, 5),
        "GBps": round(gbps, 2),
        "frac_of_n_x_hbm_peak": round(gbps / (world * HBM_PEAK_GBPS), 4),
        "block_kernel_ms": round(block_ms, 5),
        "block_kernel_GBps": round(run_bytes / (block_ms / 1e3) / 1e9, 1) if block_ms > 0 else None,
        "exchange_and_tail_ms": round(max(0.0, ms - block_ms), 5),
        "single_gpu_ms": round(t1_ms, 5),
        "single_gpu_source": t1_source,
        "bit_exact_by_construction": combine in ("relay", "striped"),
        "executor": ("push (IPC-mapped peer slots, substrafl_amd/push.py)" if getattr(tr, "push", False) else
                     "native RCCL (csrc/lockstep.hip)" if getattr(tr, "native", False) else
                     "Python schedule over torch.distributed" if world > 1 else "one rank (no exchange)"),
        "schedule": schedule,
        "hip_streams_per_rank": (f"{1 + len(tr._aux)} (compute + {len(tr._aux)} for a step's per-consumer launches)"
                                 if getattr(tr, "push", False) else
                                 "4 (compute + the communicator's + RCCL's device and host streams)"
                                 if getattr(tr, "native", False) and world > 1 else
                                 "2 (compute + the communicator's)") + " <= GPU_MAX_HW_QUEUES = 4",
        "parity": parity,
        "output_checksum": checksum,
        "checksum_comparable": comparable,
    }
    if getattr(tr, "push", False):
        res["late_landing_tags"] = int(sum(tr.late_tags()))  # every rank's count: one shared page
        res["wait_errors"] = tr.errors()
        if full_compare is not None or rank == 0:
            res["full_compare"] = full_compare
    elif getattr(tr, "comm_count", None) is not None:
        res["rccl_comm_count"] = tr.comm_count()
    if scaling == "weak":
        res["weak_efficiency"] = round(t1_ms / ms, 4) if ms > 0 else None
    else:  # the same K x M over the ranks: speedup over one GPU, and that over the rank count
        res["speedup"] = round(t1_ms / ms, 4) if ms > 0 else None
        res["strong_efficiency"] = round(t1_ms / (world * ms), 4) if ms > 0 else None
    _label_shared_gpu(ctx, res, ("GBps", "frac_of_n_x_hbm_peak", "weak_efficiency", "speedup", "strong_efficiency"))
    if variants and combine == "striped" and getattr(args, "variant_rounds", ""):
        # the other round splits over the same communicator, this leg's buffers freed first
        del step, compute_only, blocks, held, slots, ws, outs
        if hasattr(tr, "release_programs"):
            tr.release_programs()  # compiled programs hold their buffers (and, push, peer mappings)
        elif hasattr(tr, "_programs"):
            tr._programs.clear()
        torch.cuda.empty_cache()
        res["rounds_variants"] = []
        for spec in args.variant_rounds.split(";"):
            sub = argparse.Namespace(**{**vars(args), "rounds": spec})
            try:
                v = measure_client_shard(sub, ctx, combine, scaling, t1_ms, t1_source, tr=tr, variants=False)
                res["rounds_variants"].append({k: v.get(k) for k in (
                    "ms_per_step", "weak_efficiency", "speedup", "block_kernel_ms", "exchange_and_tail_ms")}
                    | {"rounds": v["schedule"].get("rounds"), "steps_of_schedule": v["schedule"].get("steps"),
                       # the whole output of this round split against the leg's own (same values)
                       "output_matches_leg": (v.get("output_checksum") == res["output_checksum"]
                                              if res["checksum_comparable"] and v.get("checksum_comparable")
                                              and rank == 0 else None)})
            except Exception as e:  # noqa: BLE001 -- a variant never costs the leg
                res["rounds_variants"].append({"rounds": spec, "error": f"{type(e).__name__}: {e}"[:300]})
            torch.cuda.empty_cache()
    return res


def _push_vs_native(ctx, plan, blocks, outs, ops, pw, ws, slots, M, c=None):
    """The push leg's whole output against the native RCCL executor's on the same plan and client
    blocks: two independent transports (stores into IPC-mapped peer memory against RCCL's P2P),
    one expected bit pattern -- both follow the reference's client order (fed_avg.py:221-222;
    Scaffold, ``c`` given: both sums, scaffold.py:262-263, 293).  Collective; returns the
    comparison on the root (every element, numel == 1 ones included)."""
    torch = ctx.torch
    from substrafl_amd.rccl import RcclTransport
    from substrafl_amd.sharding import lockstep_fedavg, lockstep_scaffold

    if torch.cuda.device_count() < ctx.world:
        return {"skipped": f"{ctx.world} ranks share {torch.cuda.device_count()} GPU(s): RCCL refuses duplicate GPUs"}
    names = ["dout", "cout"] if c is not None else ["out"]
    push_out = {k: outs[k].clone() for k in names}
    nat = RcclTransport()  # created after the push leg's timing: never live beside a push step
    try:
        count = nat.comm_count()
        for k in names:
            outs[k].fill_(float("nan"))
        if c is not None:
            lockstep_scaffold(plan, blocks, outs["dout"], outs["cout"], nat, ops, pw, c, 1.0, ws=ws, slots=slots)
        else:
            lockstep_fedavg(plan, blocks, outs["out"], nat, ops, pw, ws=ws, slots=slots)
        torch.cuda.synchronize(ctx.device)
        res = None
        if plan.rank == plan.root:
            bits = torch.int64 if c is not None else torch.int32
            mism = sum(int((push_out[k][:M].view(bits) != outs[k][:M].view(bits)).sum().item()) for k in names)
            res = {"against": "native RCCL executor (csrc/lockstep.hip), same plan and client blocks",
                   "elements": M * len(names), "mismatches": mism, "rccl_comm_count": count}
    finally:
        nat.close()
        for k in names:
            outs[k].copy_(push_out[k])
    return res


def measure_param_range_gather(args, ctx, t1_ms=None):
    """BASELINE.json's C3 as written on N GPUs ("64 clients x 125M ... sharded across 8 MI355X"),
    strong: rank r reduces elements [lo_r, hi_r) of all K clients with the single-GPU kernel
    (parameter-range sharding, bit-exact), and the timed step includes the RCCL gather of the N
    result slices into ONE full result on rank 0 (torch.distributed gather over the NCCL backend:
    (N - 1) / N of M * 4 bytes into rank 0 over its xGMI links).  Parity: every rank's sampled
    elements against the reference's sequential order, and rank 0's gathered slices against every
    rank's own by checksum."""
    torch, world, rank, device, dist = ctx.torch, ctx.world, ctx.rank, ctx.device, ctx.dist
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes
    from substrafl_amd.sharding import shard_bounds

    wl = ctx.wl
    if wl["strategy"] != "fedavg" or wl["kind"] != "f32":
        return {"skipped": "the gather leg runs the fp32 FedAvg workloads (c2, c3)"}
    K, M = wl["K"], wl["M"]
    layout = BucketLayout(list(range(len(synthetic_state_dict_shapes(M)))), synthetic_state_dict_shapes(M), np.float32)
    bounds = shard_bounds(M, world)
    lo, hi = bounds[rank]
    n = hi - lo
    chunk = bounds[0][1] - bounds[0][0]
    pw = layout.pairwise_idx.astype(np.int64)
    pw_local = (pw[(pw >= lo) & (pw < hi)] - lo).astype(np.uint64)
    n_samples = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    ld = max(64, -(-max(1, n) // 64) * 64)
    x = synth_clients(torch, K, ld, max(1, n), "f32", device, 20241016 + 1_000_003 * rank)
    send = torch.zeros(chunk, dtype=torch.float32, device=device)
    plan = FedAvgPlan("f32", x, fedavg_weights(n_samples, "f32"), n, send, pw_local)
    full = (torch.empty(world * chunk, dtype=torch.float32, device=device) if world > 1 else send) if rank == 0 else None
    glist = [full[r * chunk:(r + 1) * chunk] for r in range(world)] if rank == 0 else None
    stream = ctx.stream

    def gather():
        if world > 1:  # one rank: its slice is the whole result, already where it belongs
            dist.gather(send, gather_list=glist, dst=0)

    def step():
        plan.launch(stream)
        gather()

    steps = max(1, min(args.steps, args.client_shard_steps))
    warm = max(1, min(args.warmup, 5))
    elapsed, _ev = _timed(ctx, step, steps, warm)

    def timed_alone(fn, reps=10):
        torch.cuda.synchronize(device)
        ctx.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(device)
        return (time.perf_counter() - t0) / reps * 1e3

    kern_ms = timed_alone(lambda: plan.launch(stream))
    gather_ms = timed_alone(gather)
    # parity: sampled elements of this rank's slice against the sequential fp32 chain
    g = np.random.default_rng(123 + rank)
    idx = np.setdiff1d(np.unique(g.integers(0, max(1, n), 1024)), pw_local.astype(np.int64)) if n else np.zeros(0, np.int64)
    mism = 0
    if idx.size:
        tidx = torch.from_numpy(idx).to(device)
        xs = x[:, tidx].double().cpu().numpy()
        w32 = fedavg_weights(n_samples, "f32")
        acc = np.zeros(idx.size, np.float32)
        for k in range(K):
            acc = (acc + (xs[k].astype(np.float32) * w32[k]).astype(np.float32)).astype(np.float32)
        mism = int(np.sum(acc.view(np.uint32) != send[tidx].cpu().numpy().view(np.uint32)))
    # the gathered slices on rank 0 against each rank's own slice, by checksum of the bit patterns
    step()
    torch.cuda.synchronize(device)
    mine = int(send[:n].view(torch.int32).to(torch.int64).sum().item()) if n else 0
    sums = [(mine, mism)] * world
    if world > 1:
        dist.all_gather_object(sums, (mine, mism))
    elapsed, kern_ms, gather_ms = ctx.max_over_ranks([elapsed, kern_ms, gather_ms])
    got = [int(full[r * chunk: r * chunk + (b - a)].view(torch.int32).to(torch.int64).sum().item()) if b > a else 0
           for r, (a, b) in enumerate(bounds)] if rank == 0 else None
    pipe = None
    if args.gather_chunks > 0:  # collective: every rank runs it (an error is reported, never raised)
        try:
            pipe = _gather_pipelined(args, ctx, x, n_samples, pw_local, n, chunk, send, full, bounds, steps, warm)
        except Exception as e:  # noqa: BLE001 -- the variant never costs the leg
            pipe = {"error": f"{type(e).__name__}: {e}"[:400]}
    if rank != 0:
        return {}
    ms = elapsed / steps * 1e3
    bytes_job = K * M * 4 + M * 4
    res = {
        "workload": wl["name"] + " (BASELINE.json C3 as written: M split over the GPUs)",
        "scaling": "strong",
        "clients": K,
        "params": M,
        "params_per_gpu": chunk,
        "steps": steps,
        "warmup": warm,
        "ms_per_step": round(ms, 5),
        "GBps": round(bytes_job / (ms / 1e3) / 1e9, 2),
        "frac_of_n_x_hbm_peak": round(bytes_job / (ms / 1e3) / 1e9 / (world * HBM_PEAK_GBPS), 4),
        "kernel_ms": round(kern_ms, 5),
        "gather_ms": round(gather_ms, 5),
        "gather": "torch.distributed gather (NCCL backend = RCCL) of the N result slices into one buffer on rank 0",
        "gather_bytes_into_rank0": (world - 1) * chunk * 4,
        "parity": {"sampled_per_rank": 1024, "mismatches": int(sum(v[1] for v in sums)),
                   "gathered_slice_checksum_mismatches": int(sum(1 for r in range(world) if got[r] != sums[r][0]))},
    }
    if t1_ms:
        res["single_gpu_ms"] = round(t1_ms, 5)
        res["speedup"] = round(t1_ms / ms, 4) if ms > 0 else None
        res["strong_efficiency"] = round(t1_ms / (world * ms), 4) if ms > 0 else None
    if pipe is not None:
        res["pipelined"] = pipe
        if t1_ms and pipe.get("ms_per_step"):
            pipe["speedup"] = round(t1_ms / pipe["ms_per_step"], 4)
            pipe["strong_efficiency"] = round(t1_ms / (world * pipe["ms_per_step"]), 4)
        _label_shared_gpu(ctx, pipe, ("GBps", "speedup", "strong_efficiency"))
    _label_shared_gpu(ctx, res, ("GBps", "frac_of_n_x_hbm_peak", "speedup", "strong_efficiency"))
    return res


def _gather_cuts(chunk: int, n_chunks: int):
    """The pipelined gather's chunks of a rank's (padded) slice: ``n_chunks`` pieces of equal,
    SHARD_ALIGN-aligned length (the last one shorter), the same on every rank."""
    from substrafl_amd.lockstep import SHARD_ALIGN

    sub = max(SHARD_ALIGN, -(-(-(-chunk // max(1, int(n_chunks)))) // SHARD_ALIGN) * SHARD_ALIGN)
    return [(a, min(chunk, a + sub)) for a in range(0, chunk, sub)], sub


def _gather_pipelined(args, ctx, x, n_samples, pw_local, n, chunk, send, full, bounds, steps, warm):
    """The gather leg's pipelined variant: this rank's slice cut into ``--gather-chunks`` chunks;
    chunk c is reduced on the compute stream and gathered to rank 0 (RCCL, issued from a second
    stream after the chunk's event) while chunk c + 1 is reduced -- the kernel's HBM reads and the
    gather's xGMI traffic overlap instead of adding up.  The same elements and kernel arithmetic
    (parameter-range chunks of the single-GPU kernel, bit-exact); rank 0's gathered slices are
    checked against every rank's own by checksum.  Collective."""
    torch, world, rank, device, dist = ctx.torch, ctx.world, ctx.rank, ctx.device, ctx.dist
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    cuts, sub = _gather_cuts(chunk, args.gather_chunks)
    w = fedavg_weights(n_samples, "f32")
    plans = []
    for a, b in cuts:
        m = max(0, min(b, n) - a)
        if m:
            pw = pw_local.astype(np.int64)
            pwc = (pw[(pw >= a) & (pw < a + m)] - a).astype(np.uint64)
            ptrs = [x[k].data_ptr() + a * 4 for k in range(x.shape[0])]
            plans.append(FedAvgPlan("f32", ptrs, w, m, send[a:b], pwc))
        else:
            plans.append(None)
    glists = [[full[r * chunk + a: r * chunk + b] for r in range(world)] if rank == 0 else None for a, b in cuts]
    stream, comm = ctx.stream, torch.cuda.Stream(device=device)
    evs = [torch.cuda.Event() for _ in cuts]

    def step():
        works = []
        for c, (a, b) in enumerate(cuts):
            if plans[c] is not None:
                plans[c].launch(stream)
            if world > 1:
                evs[c].record(stream)
                with torch.cuda.stream(comm):
                    comm.wait_event(evs[c])
                    works.append(dist.gather(send[a:b], gather_list=glists[c], dst=0, async_op=True))
        for wk in works:
            if wk is not None:
                wk.wait()

    elapsed, _ev = _timed(ctx, step, steps, warm)
    send.zero_()
    if full is not None:
        full.fill_(float("nan"))
    step()
    torch.cuda.synchronize(device)
    mine = int(send[:n].view(torch.int32).to(torch.int64).sum().item()) if n else 0
    sums = [mine] * world
    if world > 1:
        dist.all_gather_object(sums, mine)
    (elapsed,) = ctx.max_over_ranks([elapsed])
    if rank != 0:
        return {}
    got = [int(full[r * chunk: r * chunk + (b - a)].view(torch.int32).to(torch.int64).sum().item()) if b > a else 0
           for r, (a, b) in enumerate(bounds)]
    return {"chunks": len(cuts), "elements_per_chunk": sub, "ms_per_step": round(elapsed / steps * 1e3, 5),
            "gathered_slice_checksum_mismatches": int(sum(1 for r in range(world) if got[r] != sums[r])),
            "issue": "chunk kernel on the compute stream; its gather (async, NCCL backend) from a second stream "
                     "after the chunk's event"}


def p2p_probe(torch, dist, rank, world, device, barrier, max_over_ranks, ring_mib=256, peers_mib=64, iters=5):
    """Point-to-point rates of this node's GPU links over the process group's RCCL (gloo on the
    CPU rehearsal): ``ring``: every rank sends ``ring_mib`` to rank r + 1 while receiving from
    r - 1 (one link per direction, all links of the ring busy at once -- the relay's pattern);
    ``all_peers``: every rank sends ``peers_mib`` to each of its G - 1 peers and receives as much
    from each, in one batch (every link of the mesh busy -- the striped schedule's pattern).
    GB/s per rank and direction, over the slowest rank."""
    dt = torch.float32
    out = {"iters": iters}

    def timed(fn):
        fn()  # connects the peers and warms the path
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        return max_over_ranks([(time.perf_counter() - t0) / iters])[0]

    def run(ops):
        for w in dist.batch_isend_irecv(ops) or []:
            w.wait()

    n = ring_mib << 18
    send, recv = torch.ones(n, dtype=dt, device=device), torch.empty(n, dtype=dt, device=device)
    ring = [dist.P2POp(dist.isend, send, (rank + 1) % world), dist.P2POp(dist.irecv, recv, (rank - 1) % world)]
    sec = timed(lambda: run(ring))
    out["ring"] = {"MiB": ring_mib, "ms": round(sec * 1e3, 3), "GBps_per_direction": round(n * 4 / sec / 1e9, 2)}
    del send, recv
    m = peers_mib << 18
    peers = [p for p in range(world) if p != rank]
    sends = torch.ones((len(peers), m), dtype=dt, device=device)
    recvs = torch.empty((len(peers), m), dtype=dt, device=device)
    ops = [dist.P2POp(dist.isend, sends[i], p) for i, p in enumerate(peers)] + \
          [dist.P2POp(dist.irecv, recvs[i], p) for i, p in enumerate(peers)]
    sec = timed(lambda: run(ops))
    out["all_peers"] = {"MiB_per_peer": peers_mib, "peers": len(peers), "ms": round(sec * 1e3, 3),
                        "GBps_per_rank_egress": round(len(peers) * m * 4 / sec / 1e9, 2),
                        "GBps_per_link_direction": round(m * 4 / sec / 1e9, 2)}
    return out


def _rounds(args):
    from substrafl_amd import lockstep

    if not args.rounds:  # the schedule's default for the executor (lockstep.py)
        return lockstep.default_rounds(args.gpus, args.executor == "native")  # push: one round (no gather tail)
    return tuple(float(x) for x in args.rounds.split(","))


def _single_gpu_ms(ctx, K, M, kind, scaffold, layout, n_samples):
    """Kernel time of one GPU reducing K clients x M (the layout the library recommends)."""
    torch, device, stream = ctx.torch, ctx.device, ctx.stream
    from substrafl_amd.engine import (FedAvgPlan, ScaffoldPlan, TiledFedAvgPlan, fedavg_weights, scaffold_weights,
                                      tiled_recommended, tiled_tile)

    if scaffold:
        d = torch.empty((K, layout.ld), dtype=torch.float32, device=device).normal_()
        v = torch.empty_like(d).normal_()
        c = torch.randn(layout.ld, dtype=torch.float32, device=device)
        do = torch.empty(layout.ld, dtype=torch.float64, device=device)
        co = torch.empty_like(do)
        plan = ScaffoldPlan(kind, d, v, c, scaffold_weights(n_samples[:K]), M, 1.0, do, co, layout.pairwise_idx)
    else:
        out = torch.empty(layout.ld, dtype=torch.float32, device=device)
        w = fedavg_weights(n_samples[:K], kind)
        if tiled_recommended(kind, K, M):
            tv = tiled_tile(kind, K, M)
            buf = synth_tiled(torch, K, M, kind, device, 1, tv)
            plan = TiledFedAvgPlan(kind, buf, K, w, M, out, layout.pairwise_idx, tv=tv)
        else:
            buf = synth_clients(torch, K, layout.ld, M, kind, device, 1)
            plan = FedAvgPlan(kind, buf, w, M, out, layout.pairwise_idx)
    for _ in range(3):
        plan.launch(stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(10):
        plan.launch(stream)
    e1.record(stream)
    torch.cuda.synchronize(device)
    ms = e0.elapsed_time(e1) / 10
    del plan
    torch.cuda.empty_cache()
    return ms


def _held_values(torch, kind, data, cols, Kb):
    """[Kb, len(cols)] fp64 values of a block buffer (rows tensor or TiledBlock) at columns."""
    from substrafl_amd.engine import tiled_index
    from substrafl_amd.sharding import TiledBlock

    if not isinstance(data, TiledBlock):
        return data[:, torch.from_numpy(cols).to(data.device)].to(torch.float64)
    out = torch.empty((Kb, len(cols)), dtype=torch.float64, device=next(iter(data.buckets.values()))[0].device)
    for j, col in enumerate(cols):
        t, e = data.locate(int(col))
        idx = tiled_index(kind, Kb, np.arange(Kb), e, data.tv)
        out[:, j] = t[torch.from_numpy(idx).to(t.device)].to(torch.float64)
    return out


def _client_shard_spot_check(ctx, K, M, layout, n_samples, kind, scaffold, held, outs, c, tvs):
    """Sampled elements against the reference's sequential order: every rank writes the values it
    holds into a zeroed [K, S] fp64 matrix (each (client, element) is held by exactly one rank),
    the matrices are summed onto the root over RCCL, which recomputes the chain on the host."""
    torch, world, rank, device = ctx.torch, ctx.world, ctx.rank, ctx.device
    from substrafl_amd.engine import fedavg_weights, scaffold_weights

    g = np.random.default_rng(123)
    idx = np.setdiff1d(np.unique(g.integers(0, M, 2048)), layout.pairwise_idx.astype(np.int64))
    nf = 2 if scaffold else 1
    dense = torch.zeros((nf, K, idx.size), dtype=torch.float64, device=device)
    for b, (k0, data, segs) in held.items():
        parts = data if scaffold else (data,)
        Kb = parts[0].shape[0]
        if Kb == 0:
            continue
        for lo, hi, col in segs:
            sel = np.nonzero((idx >= lo) & (idx < hi))[0]
            if not sel.size:
                continue
            cols = (idx[sel] - lo + col).astype(np.int64)
            for f, part in enumerate(parts):
                dense[f, k0: k0 + Kb, torch.from_numpy(sel).to(device)] = _held_values(torch, kind, part, cols, Kb)
    dense = dense.cpu()
    if world > 1:  # over the host group (gloo): every leg has it
        ctx.dist.reduce(dense, dst=0)
    if rank != 0:
        return None
    xs = dense.numpy()
    tidx = torch.from_numpy(idx).to(device)
    if not scaffold:
        got = outs["out"][tidx].cpu().numpy()
        w32 = fedavg_weights(n_samples, "f32")
        acc = np.zeros(idx.size, np.float32)
        for k in range(K):
            acc = (acc + (xs[0, k].astype(np.float32) * w32[k]).astype(np.float32)).astype(np.float32)
        bad = acc.view(np.uint32) != got.view(np.uint32)
        return {"sampled": int(idx.size), "mismatches": int(np.sum(bad))}
    w64 = scaffold_weights(n_samples)
    ad, ac = np.zeros(idx.size), np.zeros(idx.size)
    for k in range(K):
        ad = ad + xs[0, k] * w64[k]
        ac = ac + xs[1, k] * w64[k]
    ad = 1.0 * ad
    ac = ac + c[tidx].double().cpu().numpy()
    gd, gcv = outs["dout"][tidx].cpu().numpy(), outs["cout"][tidx].cpu().numpy()
    return {"sampled": int(idx.size), "mismatches": int(np.sum(ad.view(np.uint64) != gd.view(np.uint64))
                                                        + np.sum(ac.view(np.uint64) != gcv.view(np.uint64)))}


def client_shard_line(args, ctx, cs):
    """``--mode client-shard``: the client-shard measurement as the line itself."""
    wl = ctx.wl
    line = {
        "metric": METRIC,
        "value": cs["GBps"],
        "unit": "GB/s",
        "n_gpus": ctx.world,
        "steps": cs["steps"],
        "warmup": cs["warmup"],
        "ms_per_step": cs["ms_per_step"],
        "higher_is_better": True,
        "scaling": cs["scaling"],
        "vs_baseline": None,
        "dtype": "bf16-in/f32-acc" if wl["kind"] == "bf16" else (
            "f32-in/f64-acc" if wl["strategy"] == "scaffold" else "f32"),
        "data": "synthetic (N(0,1) client blocks generated on device, torch Philox; "
                "n_samples = default_rng(7).integers(100, 10000, K))",
        "config": {"workload": wl["name"], "strategy": wl["strategy"], "clients": cs["clients"],
                   "clients_per_gpu": cs["clients_per_gpu"], "global_params": cs["params"],
                   "parallelism": f"client-shard x{ctx.world} ({cs['combine']})" if ctx.world > 1 else "single-gpu",
                   "layout": cs["layout"]},
        "roofline": {"bound": "hbm", "achieved": cs["block_kernel_GBps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round((cs["block_kernel_GBps"] or 0) / HBM_PEAK_GBPS, 4), "traffic": None,
                     "kernel": "fedavg_kernel (chain runs of the schedule)" if wl["strategy"] == "fedavg" else
                               "scaffold chain runs", "kernel_ms": cs["block_kernel_ms"],
                     "kernel_timing": "HIP events: this rank's block kernels alone, back to back, max over ranks"},
        "cpu_baseline": None,
        "parity": cs["parity"],
        "client_shard": cs,
        "build": {"lib_sha256": lib_sha256()},
    }
    if ctx.world > 1:
        line["process_group"] = {"backend": ctx.backend, "timeout_s": PG_TIMEOUT_S}
    return line


def spot_check(torch, world, rank, scaffold, K, M, layout, n_samples, kind, device, env):
    """Sampled output elements against the reference's sequential order (fp32 FedAvg chain /
    fp64 Scaffold with c last and lr after the sum), on each rank's own reduction.  numel == 1
    elements are excluded here (pairwise order: tests/ check them against the oracle)."""
    from substrafl_amd.engine import fedavg_weights, scaffold_weights

    g = np.random.default_rng(123)
    idx = np.setdiff1d(np.unique(g.integers(0, M, 4096)), layout.pairwise_idx.astype(np.int64))
    tidx = torch.from_numpy(idx).to(device)

    def cols(x):  # [K, S] sampled columns of the client buckets
        if env.get("tiled"):  # tile-interleaved buffer: gather each client's sampled elements
            from substrafl_amd.engine import tiled_index

            pos = tiled_index(kind, K, np.arange(K)[:, None], idx[None, :], env["tv"])
            return x[torch.from_numpy(pos.reshape(-1)).to(device)].view(K, -1).to(torch.float64).cpu().numpy()
        return x[:, tidx].to(torch.float64).cpu().numpy()

    if not scaffold:
        xs = cols(env["clients"])
        got = env["out"][tidx].cpu().numpy()
        w32 = fedavg_weights(n_samples, "f32")
        acc = np.zeros(idx.size, np.float32)
        for k in range(xs.shape[0]):
            acc = (acc + (xs[k].astype(np.float32) * w32[k]).astype(np.float32)).astype(np.float32)
        bad = acc.view(np.uint32) != got.view(np.uint32)
        res = {"sampled": int(idx.size), "mismatches": int(np.sum(bad))}
        if bad.any():
            ia, ib = acc.view(np.int32).astype(np.int64), got.view(np.int32).astype(np.int64)
            res["max_ulp"] = int(np.max(np.abs(ia - ib)))
        return res
    xd, xc = cols(env["delta"]), cols(env["cv"])
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
    eng = MultiDeviceEngine(devices, pack_threads=args.md_pack_threads or None)
    eng.kernel_events = True
    for _ in range(max(1, args.warmup)):
        eng.fedavg(pus, n_samples)
    walls, shards = [], []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        res = eng.fedavg(pus, n_samples)
        walls.append(time.perf_counter() - t0)
        shards.append(eng.last_timing["shards"])
    wall = float(np.median(walls))
    py_bits = np.concatenate([np.asarray(a).reshape(-1) for a in res]).view(np.uint32).copy()
    del res
    # the same plan through the one-call C entry (fedagg_multi_fedavg_f32, csrc/multi.hip): the
    # orchestration in C++ instead of Python threads, same devices, same host buckets
    from substrafl_amd.multi_device import NativeMultiFedAvg

    nat = NativeMultiFedAvg(devices, pack_threads=args.md_pack_threads or 0)
    for _ in range(max(1, args.warmup)):
        nat.fedavg(pus, n_samples)
    nwalls = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        nres = nat.fedavg(pus, n_samples)
        nwalls.append(time.perf_counter() - t0)
    nwall = float(np.median(nwalls))
    native_entry = {"ms_per_call_median": round(nwall * 1e3, 3),
                    "value": round((K * M * 4 + M * 4) / nwall / 1e9, 2), "unit": "GB/s",
                    "mismatches_vs_python_engine": int(np.sum(np.concatenate(
                        [np.asarray(a).reshape(-1) for a in nres]).view(np.uint32) != py_bits)),
                    "shards": nat.shard_info(), "entry": "fedagg_multi_fedavg_f32 (one C call per aggregation)"}
    del nres
    nat.close()
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
        # host ingress per shard: pack threads (CPUs allowed // GPUs), their NUMA node (the GPU's,
        # from sysfs), the CPUs they are bound to and the node the pinned ring landed on
        "placement": eng.placement_report(),
        "native_c_entry": native_entry,
        "cpus_allowed": len(os.sched_getaffinity(0)),
        "note": "end-to-end (pinned-ring pack + H2D + kernel + D2H); not the device-resident metric",
    }), flush=True)


# ======================================================================================
# --rehearse-cpu (tests): the launcher / rank / timing plumbing without a GPU
# ======================================================================================
class _RehearsalOps:
    """NumPy chain arithmetic for --rehearse-cpu (the schedule's plumbing over gloo, no GPU)."""

    def fedavg_run(self, kind, rows, w, seed, acc):
        a = np.zeros(acc.shape[0], np.float32) if seed else acc.numpy().copy()
        x = rows.numpy()
        for k in range(x.shape[0]):
            a = (a + (x[k] * np.float32(w[k])).astype(np.float32)).astype(np.float32)
        acc.copy_(__import__("torch").from_numpy(a))

    def fedavg_products_at(self, kind, rows, w, kbase, K, idx, ws):
        x = rows.numpy()
        for p, i in enumerate(np.asarray(idx, np.int64)):
            for k in range(x.shape[0]):
                ws[p, kbase + k] = float(np.float32(x[k, i] * np.float32(w[k])))

    def fedavg_finish(self, kind, ws, K, pairwise_idx, out):
        for p, i in enumerate(np.asarray(pairwise_idx, np.int64)):
            out[int(i)] = float(np.float32(ws[p, :K].numpy().astype(np.float32).sum()))


def rehearse(args, world, rank):
    """--rehearse-cpu (tests): the launcher, the process group with its timeout, the barrier /
    max-over-ranks timing and, for N > 1, the client-shard leg's lockstep schedule over gloo on
    a tiny synthetic problem -- the same line fields as a GPU run, nothing measured."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo", **pg_kwargs())
    if args.client_shard_child:  # one leg child of a --rehearse-legs line
        return _rehearse_leg_child(args, world, rank)
    x = np.ones(1 << 16, np.float32)
    for _ in range(args.warmup):
        x = x * np.float32(1.0)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x = x * np.float32(1.0)
    elapsed = time.perf_counter() - t0
    cs = gather_leg = None
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        if args.rehearse_legs:  # the leg mechanism itself: child processes, deadlines, failures
            import types

            ctx = _Ctx(torch=torch, dist=dist, world=world, rank=rank, device=types.SimpleNamespace(index=rank))
            legs = client_shard_legs(args, ctx, {"kern_ms": 1.0})
        elif args.client_shard != "off":
            cs = _rehearse_client_shard(args, world, rank)
            probe = p2p_probe(torch, dist, rank, world, torch.device("cpu"), dist.barrier,
                              lambda v: [float(x) for x in _all_max(torch, dist, v)], ring_mib=1, peers_mib=1, iters=2)
            if cs is not None:
                cs["xgmi_p2p"] = probe
            gather_leg = _rehearse_gather(world, rank)
    if rank == 0:
        line = {"metric": METRIC + " [CPU rehearsal of the launcher: not a measurement]",
                "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 6),
                "rehearsal": True, "ranks_seen": world}
        wl = WORKLOADS[args.workload]
        line["config"] = {"workload": wl["name"] + ("_per_gpu" if world > 1 and args.scaling == "weak" else ""),
                          "parallelism": f"param-range x{world}" if world > 1 else "single-gpu"}
        if world > 1 and args.rehearse_legs:
            line["process_group"] = {"backend": dist.get_backend(), "timeout_s": PG_TIMEOUT_S}
            line.update(legs)
            line["line_wall_s"] = round(time.monotonic() - _T_START, 1)
        elif world > 1:
            line["process_group"] = {"backend": dist.get_backend(), "timeout_s": PG_TIMEOUT_S}
            line["client_shard"] = cs
            line["legs_order"] = [leg[2] for leg in LEGS]
            # one leg agrees with nothing: null (client_shard_legs' rule)
            line["client_shard_output_checksums"] = {"legs": ["client_shard"], "agree": None} if cs else None
            line["param_range_strong_gather"] = gather_leg
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _rehearse_leg_child(args, world, rank):
    """A leg child under --rehearse-legs: the gloo group is up; the warm-up is one barrier, then
    LEG_READY, then the leg's rehearsal (the gather leg's or the client-shard schedule's).
    ``BENCH_REHEARSE_HANG=<leg key>:connect|timed`` (tests) makes that leg hang before or after
    it reports ready -- a leg stuck in RCCL's connect, or in its timed steps."""
    import torch.distributed as dist

    hang = os.environ.get("BENCH_REHEARSE_HANG", "")
    if hang == f"{args.leg_key}:connect":
        time.sleep(3600)
    dist.barrier()
    print(LEG_READY, flush=True)
    if hang == f"{args.leg_key}:timed":
        time.sleep(3600)
    res = _rehearse_gather(world, rank) if args.executor == "gather" else _rehearse_client_shard(args, world, rank)
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()


def _all_max(torch, dist, vals):
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def _rehearse_client_shard(args, world, rank):
    """The striped schedule over gloo (one communicator, one issuing thread) on 2 x 3 x 4 x 512
    elements per rank; rank 0 checks its result against a host recomputation."""
    import torch

    from substrafl_amd.sharding import (DistTransport, FedAvgShard, client_blocks, lockstep_fedavg, relay_plan,
                                        striped_plan)

    combine = args.combine if args.combine in ("relay", "striped") else "striped"
    K, M = 3 * world, 2 * world * 4 * 512 * 3 + 77
    rng = np.random.default_rng(11)
    data = rng.standard_normal((K, M)).astype(np.float32)
    w = (np.arange(1, K + 1) / np.sum(np.arange(1, K + 1))).astype(np.float32)
    plan = striped_plan(M, world, rank) if combine == "striped" else relay_plan(M, world, rank, 4096)
    blocks = {}
    for b, segs in plan.blocks.items():
        k0, k1 = client_blocks(K, world)[b]
        t = torch.zeros((k1 - k0, plan.block_len[b]), dtype=torch.float32)
        for lo, hi, col in segs:
            t[:, col: col + hi - lo] = torch.from_numpy(data[k0:k1, lo:hi])
        blocks[b] = FedAvgShard("f32", t, w[k0:k1], k0, K, plan.block_len[b], np.zeros(0, np.uint64))
    out = torch.zeros(M, dtype=torch.float32)
    tr = DistTransport()
    t0 = time.perf_counter()
    root = lockstep_fedavg(plan, blocks, out, tr, _RehearsalOps(), np.zeros(0, np.int64))
    ms = (time.perf_counter() - t0) * 1e3
    # the full comparison the push leg makes against the native executor, rehearsed as the other
    # lockstep schedule over the same blocks (one expected bit pattern)
    other = "relay" if combine == "striped" else "striped"
    plan2 = relay_plan(M, world, rank, 4096) if other == "relay" else striped_plan(M, world, rank)
    blocks2 = {}
    for b, segs in plan2.blocks.items():
        k0, k1 = client_blocks(K, world)[b]
        t = torch.zeros((k1 - k0, plan2.block_len[b]), dtype=torch.float32)
        for lo, hi, col in segs:
            t[:, col: col + hi - lo] = torch.from_numpy(data[k0:k1, lo:hi])
        blocks2[b] = FedAvgShard("f32", t, w[k0:k1], k0, K, plan2.block_len[b], np.zeros(0, np.uint64))
    out2 = torch.zeros(M, dtype=torch.float32)
    lockstep_fedavg(plan2, blocks2, out2, tr, _RehearsalOps(), np.zeros(0, np.int64))
    if not root:
        return None
    acc = np.zeros(M, np.float32)
    for k in range(K):
        acc = (acc + (data[k] * w[k]).astype(np.float32)).astype(np.float32)
    mism = int(np.sum(acc.view(np.uint32) != out.numpy().view(np.uint32)))
    full = {"against": f"the {other} schedule over the same client blocks (gloo rehearsal; on GPUs: the native "
                       "RCCL executor)", "elements": M,
            "mismatches": int(np.sum(out.numpy().view(np.uint32) != out2.numpy().view(np.uint32)))}
    keys = ("combine", "scaling", "clients", "clients_per_gpu", "params", "layout", "steps", "warmup", "ms_per_step",
            "GBps", "frac_of_n_x_hbm_peak", "block_kernel_ms", "block_kernel_GBps", "exchange_and_tail_ms",
            "single_gpu_ms", "single_gpu_source", "weak_efficiency", "bit_exact_by_construction", "schedule",
            "hip_streams_per_rank", "parity")
    res = {k: None for k in keys}
    res.update(combine=combine, scaling="weak", clients=K, clients_per_gpu=K // world, params=M, layout="rows",
               steps=1, warmup=0, ms_per_step=round(ms, 3), bit_exact_by_construction=True,
               schedule={"steps": plan.n_steps, "issue": "one host thread, one communicator (gloo rehearsal)"},
               parity={"sampled": M, "mismatches": mism}, rehearsal=True, full_compare=full,
               late_landing_tags=None, rccl_comm_count=world, checksum_comparable=True,
               output_checksum=_output_checksum(torch, out, M))
    return res


def _rehearse_gather(world, rank):
    """The param_range_strong_gather leg over gloo on a tiny problem: every rank reduces its
    parameter range (NumPy, the reference's order), the slices are gathered into one buffer on
    rank 0, checked by checksum and against a host recomputation of the whole result."""
    import torch
    import torch.distributed as dist

    from substrafl_amd.sharding import shard_bounds

    K, M = 5, 3 * 4096 + 77
    rng = np.random.default_rng(5)
    data = rng.standard_normal((K, M)).astype(np.float32)
    w = (np.arange(1, K + 1) / np.sum(np.arange(1, K + 1))).astype(np.float32)
    bounds = shard_bounds(M, world)
    lo, hi = bounds[rank]
    chunk = bounds[0][1] - bounds[0][0]
    acc = np.zeros(hi - lo, np.float32)
    for k in range(K):
        acc = (acc + (data[k, lo:hi] * w[k]).astype(np.float32)).astype(np.float32)
    send = torch.zeros(chunk, dtype=torch.float32)
    send[: hi - lo] = torch.from_numpy(acc)
    full = torch.zeros(world * chunk, dtype=torch.float32) if rank == 0 else None
    dist.gather(send, gather_list=[full[r * chunk:(r + 1) * chunk] for r in range(world)] if rank == 0 else None,
                dst=0)
    mine = int(send[: hi - lo].view(torch.int32).to(torch.int64).sum().item())
    sums = [None] * world
    dist.all_gather_object(sums, mine)
    # the pipelined variant's chunked gathers into views of the same buffer
    full2 = torch.full((world * chunk,), float("nan"), dtype=torch.float32) if rank == 0 else None
    cuts, _sub = _gather_cuts(chunk, 4)
    for a, b in cuts:
        dist.gather(send[a:b], gather_list=[full2[r * chunk + a: r * chunk + b] for r in range(world)]
                    if rank == 0 else None, dst=0)
    if rank != 0:
        return None
    ref = np.zeros(M, np.float32)
    for k in range(K):
        ref = (ref + (data[k] * w[k]).astype(np.float32)).astype(np.float32)
    got = [int(full[r * chunk: r * chunk + (b - a)].view(torch.int32).to(torch.int64).sum().item())
           for r, (a, b) in enumerate(bounds)]
    keys = ("workload", "scaling", "clients", "params", "params_per_gpu", "steps", "warmup", "ms_per_step", "GBps",
            "frac_of_n_x_hbm_peak", "kernel_ms", "gather_ms", "gather", "gather_bytes_into_rank0", "parity",
            "single_gpu_ms", "speedup", "strong_efficiency")
    res = {k: None for k in keys}
    res.update(scaling="strong", clients=K, params=M, params_per_gpu=chunk, rehearsal=True,
               gather="torch.distributed gather (gloo rehearsal; on GPUs: NCCL backend = RCCL)",
               gather_bytes_into_rank0=(world - 1) * chunk * 4,
               parity={"mismatches": int(np.sum(full[:M].numpy().view(np.uint32) != ref.view(np.uint32))),
                       "gathered_slice_checksum_mismatches": int(sum(1 for r in range(world) if got[r] != sums[r]))})
    res["pipelined"] = {"chunks": len(cuts), "rehearsal": True,
                        "mismatches_vs_whole_gather": int(torch.sum(full2.view(torch.int32) != full.view(torch.int32)))}
    return res


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
    out = {
        "value": round(nbytes / best / 1e9, 3),
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{'FULL SIZE: ' if full else ''}{K} clients x {M_s} fp32 params ({len(shapes)} layers), "
                  f"best of {len(times)} runs "
                  f"({best * 1e3:.1f} ms); oracle/aggregation.py reference call structure; "
                  f"host has {os.cpu_count()} cpus, affinity {aff}, NumPy ufuncs single-threaded",
    }
    if wl["strategy"] == "fedavg":
        out["threaded_variant"] = _cpu_threaded(fedavg_reference_structure, pus, n_samples, nbytes,
                                                min(CPU_THREADS, aff or 1))
    return out


CPU_THREADS = 16  # the host share of one GPU on the test boxes


def _cpu_threaded(reduce_fn, pus, n_samples, nbytes, threads):
    """SURVEY.md §8(d)'s optional multi-core CPU figure, NOT the reference: the same per-element
    arithmetic (``reduce_fn``: cpu_baseline's oracle call structure) over element chunks of the layers, the chunks spread
    over ``threads`` threads (NumPy releases the GIL inside its ufuncs).  Chunks keep >= 2 elements,
    and numel == 1 layers stay whole, so no chunk changes NumPy's summation order."""
    from concurrent.futures import ThreadPoolExecutor

    total = sum(a.size for a in pus[0])
    target = max(2, total // (4 * threads))
    chunks = []
    for li, a in enumerate(pus[0]):
        n = a.size
        if n == 1:
            chunks.append((li, 0, 1))
            continue
        cuts = list(range(0, n, target)) + [n]
        if len(cuts) > 2 and cuts[-1] - cuts[-2] < 2:
            cuts.pop(-2)
        chunks += [(li, lo, hi) for lo, hi in zip(cuts, cuts[1:])]
    chunks.sort(key=lambda c: c[2] - c[1], reverse=True)
    load, parts = [0] * threads, [[] for _ in range(threads)]
    for c in chunks:  # largest first onto the least loaded thread
        t = load.index(min(load))
        parts[t].append(c)
        load[t] += c[2] - c[1]
    views = [[[pu[li].reshape(-1)[lo:hi] for li, lo, hi in part] for pu in pus] for part in parts if part]

    def run():
        with ThreadPoolExecutor(len(views)) as ex:
            list(ex.map(lambda v: reduce_fn(v, n_samples), views))

    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        run()
        times.append(time.perf_counter() - t0)
    best = min(times)
    return {"value": round(nbytes / best / 1e9, 3), "unit": "GB/s", "cores": len(views),
            "kind": "port, chunked over threads -- not the reference",
            "sample": f"the same sample, {len(chunks)} element chunks over {len(views)} threads, best of 3 "
                      f"({best * 1e3:.1f} ms)"}


if __name__ == "__main__":
    main()
