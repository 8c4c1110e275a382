#!/usr/bin/env python3
"""C5's launch-duration step (VERDICT r05 "Next 2"): in one process, time every C5 launch
(fedavg_tiled_bf16, 128 x 350M, 91.0 GB per launch) with HIP events on its stream, while a thread
samples the GPU's power-management state (amdsmi gpu_metrics: gfx / soc / memory clocks, socket
power, hotspot / HBM temperature, throttle status) every ~2 ms on the same host clock.  Bursts:

  1. ``first``:   120 launches right after the buckets are synthesised (what bench.py does);
  2. ``idle``:    the same buffer after 3 s with the GPU idle -- a power-management ramp recurs
                  after idle, a one-time allocation / first-use effect does not;
  3. ``fresh``:   a SECOND, newly allocated 91 GB buffer (new pages, new page-table entries) --
                  an allocation-side effect recurs here;
  4. ``old``:     the first buffer again, 40 launches (is it still at its steady time?).

Per burst: every launch's duration and start (host clock), the step (the split of the launch
sequence that best separates two levels), the mean before / after it, and the clocks, power and
temperatures sampled during each launch.  One JSON object to --out.
"""

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

BYTES = 128 * 350_000_000 * 2 + 350_000_000 * 4
_T0 = time.time()  # this process's start (wall clock, comparable across processes)


class Sampler(threading.Thread):
    """amdsmi gpu_metrics of the GPU at ``bdf`` every ``period`` s: (host time, fields)."""

    FIELDS = ("current_gfxclks", "current_socclks", "current_uclk", "current_socket_power", "average_socket_power",
              "temperature_hotspot", "temperature_mem", "throttle_status", "indep_throttle_status",
              "ppt_residency_acc", "socket_thm_residency_acc", "hbm_thm_residency_acc", "gfxclk_lock_status",
              "average_umc_activity", "average_gfx_activity", "firmware_timestamp", "average_gfxclk_frequency",
              "average_socclk_frequency", "average_uclk_frequency", "prochot_residency_acc", "vr_thm_residency_acc",
              "mem_activity_acc", "gfx_activity_acc", "accumulation_counter", "voltage_soc", "voltage_gfx",
              "voltage_mem", "energy_accumulator", "pcie_bandwidth_inst")

    def __init__(self, bdf, period=0.002, enabled=True):
        super().__init__(daemon=True)
        self.period, self.samples, self.error, self.stop_ev = period, [], None, threading.Event()
        self.handle = None
        if not enabled:
            self.error = "disabled (--no-sampler)"
            return
        try:
            import amdsmi

            self.smi = amdsmi
            amdsmi.amdsmi_init()
            handles = amdsmi.amdsmi_get_processor_handles()
            bdfs = [amdsmi.amdsmi_get_gpu_device_bdf(h).lower() for h in handles]
            want = [i for i, b in enumerate(bdfs) if bdf and b.endswith(bdf.lower()[-7:])]
            self.handle = handles[want[0]] if want else (handles[0] if len(handles) == 1 else None)
            self.bdfs = bdfs
            if self.handle is None:
                self.error = f"no amdsmi handle for {bdf} among {bdfs}"
        except Exception as e:  # noqa: BLE001 -- the launch timings stand without the sampler
            self.error = f"{type(e).__name__}: {e}"[:300]

    def read(self):
        m = self.smi.amdsmi_get_gpu_metrics_info(self.handle)
        out = {}
        for f in self.FIELDS:
            v = m.get(f)
            if isinstance(v, list):
                v = [x for x in v if isinstance(x, (int, float))]
                v = (float(np.mean(v)) if v else None)
            out[f] = v if isinstance(v, (int, float)) else None
        return out

    def run(self):
        if self.handle is None:
            return
        try:
            while not self.stop_ev.is_set():
                t = time.perf_counter()
                self.samples.append((t, self.read()))
                time.sleep(max(0.0, self.period - (time.perf_counter() - t)))
        except Exception as e:  # noqa: BLE001
            self.error = f"{type(e).__name__}: {e}"[:300]


TRACE_FIELDS = ("current_socclks", "current_gfxclks", "current_uclk", "average_umc_activity", "average_gfx_activity",
                "current_socket_power", "pcie_bandwidth_inst")


def step_split(d):
    """The index s (2 <= s <= n-2) splitting durations d into two levels with the least
    within-level squared error; returns (s, mean before, mean after)."""
    d = np.asarray(d, np.float64)
    n = len(d)
    if n < 6:
        return None, None, None
    best = None
    for s in range(2, n - 1):
        a, b = d[:s], d[s:]
        err = ((a - a.mean()) ** 2).sum() + ((b - b.mean()) ** 2).sum()
        if best is None or err < best[0]:
            best = (err, s)
    s = best[1]
    return s, float(d[:s].mean()), float(d[s:].mean())


def burst(torch, plan, stream, n, sampler, label, sync=True):
    if sync:  # (False: the launches queue behind whatever the stream still has to run)
        torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    t_ref = time.perf_counter()
    for a, b in evs:
        a.record(stream)
        plan.launch(stream)
        b.record(stream)
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    dur = [a.elapsed_time(b) for a, b in evs]
    # host-clock starts anchored at the burst's END (the synchronize returns right after the last
    # launch): with sync=False the first launch waits behind the synthesis, so t_ref (enqueue time)
    # is not when it ran
    last = evs[-1][1]
    start = [t_end - a.elapsed_time(last) / 1e3 for a, _ in evs]
    t_ref = start[0] if sync is False else t_ref
    s, before, after = step_split(dur)
    samples = list(sampler.samples) if sampler.handle is not None else []
    per_launch = []
    for t0, ms in zip(start, dur):
        inside = [m for (t, m) in samples if t0 <= t <= t0 + ms / 1e3]
        rec = {"start_s": round(t0 - t_ref, 5), "ms": round(ms, 4), "samples": len(inside)}
        for f in ("current_gfxclks", "current_socclks", "current_uclk", "current_socket_power", "temperature_hotspot",
                  "temperature_mem", "throttle_status"):
            v = [m[f] for m in inside if m.get(f) is not None]
            rec[f] = round(float(np.mean(v)), 1) if v else None
        per_launch.append(rec)
    res = {"label": label, "launches": n, "ms_mean": round(float(np.mean(dur)), 4),
           "ms_median": round(float(np.median(dur)), 4), "ms_min": round(float(np.min(dur)), 4),
           "ms_max": round(float(np.max(dur)), 4),
           "step_index": s, "ms_mean_before_step": round(before, 4) if before else None,
           "ms_mean_after_step": round(after, 4) if after else None,
           "step_at_s": round(start[s] - t_ref, 4) if s else None,
           "frac_before": round(BYTES / (before / 1e3) / 8e12, 4) if before else None,
           "frac_after": round(BYTES / (after / 1e3) / 8e12, 4) if after else None,
           "per_launch": per_launch,
           # the raw samples of the burst (time from its first launch, every field), for a step
           "samples": [[round(t - t_ref, 5), m] for (t, m) in samples
                       if start and start[0] - 0.05 <= t <= start[-1] + dur[-1] / 1e3 + 0.05]}
    if s:  # the sampled state on either side of the step
        for side, rng in (("before", per_launch[:s]), ("after", per_launch[s:])):
            for f in ("current_gfxclks", "current_socclks", "current_uclk", "current_socket_power",
                      "temperature_hotspot", "temperature_mem"):
                v = [r[f] for r in rng if r[f] is not None]
                res[f"{f}_{side}"] = round(float(np.mean(v)), 1) if v else None
            ts = sorted({r["throttle_status"] for r in rng if r["throttle_status"] is not None})
            res[f"throttle_status_{side}"] = ts
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--first", type=int, default=120)
    ap.add_argument("--idle-s", type=float, default=3.0)
    ap.add_argument("--second", type=int, default=60)
    ap.add_argument("--fresh", type=int, default=60)
    ap.add_argument("--old", type=int, default=40)
    ap.add_argument("--no-sampler", action="store_true", help="no amdsmi polling (does the polling itself matter?)")
    ap.add_argument("--no-sync-after-synth", action="store_true",
                    help="enqueue the first launches right behind the synthesis, as bench.py does")
    ap.add_argument("--sleep-after-synth", type=float, default=0.0, help="idle seconds between synthesis and launches")
    ap.add_argument("--sleep-before-synth", type=float, default=0.0,
                    help="idle seconds between HIP start-up and the 91 GB allocation (does the step move with it?)")
    args = ap.parse_args()

    import torch

    import bench
    from substrafl_amd.engine import TiledFedAvgPlan, fedavg_weights, tiled_tile
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes
    from substrafl_amd.runtime import device_pci_bus_id

    K, M, kind = 128, 350_000_000, "bf16"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    marks = {}  # wall seconds since process start of each phase
    torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    marks["hip_ready"] = round(time.time() - _T0, 4)
    sampler = Sampler(device_pci_bus_id(0), enabled=not args.no_sampler)
    sampler.start()
    marks["sampler_started"] = round(time.time() - _T0, 4)
    if args.sleep_before_synth:
        time.sleep(args.sleep_before_synth)
    out = {"workload": "c5 fedavg_bf16_128x350M tiled", "bytes_alg_per_launch": BYTES, "process_start_wall": _T0,
           "sampler": {"error": sampler.error, "period_s": sampler.period,
                       "bdfs": getattr(sampler, "bdfs", None)}, "bursts": []}
    shapes = synthetic_state_dict_shapes(M)
    pw = BucketLayout(list(range(len(shapes))), shapes, np.float32).pairwise_idx
    n_samples = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    w = fedavg_weights(n_samples, kind)
    tv = tiled_tile(kind, K, M)
    t0 = time.perf_counter()
    marks["alloc_start"] = round(time.time() - _T0, 4)
    buf_a = bench.synth_tiled(torch, K, M, kind, dev, 20241016, tv)
    ld = BucketLayout(list(range(len(shapes))), shapes, np.float32).ld
    out_a = torch.empty(ld, dtype=torch.float32, device=dev)
    marks["synth_enqueued"] = round(time.time() - _T0, 4)
    if not args.no_sync_after_synth:  # bench.py enqueues its first launches behind the synthesis
        torch.cuda.synchronize()
    out["synth_s"] = round(time.perf_counter() - t0, 2)
    out["sync_after_synth"] = not args.no_sync_after_synth
    if args.sleep_after_synth:
        time.sleep(args.sleep_after_synth)
    out["sleep_after_synth_s"] = args.sleep_after_synth
    plan_a = TiledFedAvgPlan(kind, buf_a, K, w, M, out_a, pw, tv=tv)
    print(f"synth {out['synth_s']} s; sampler {sampler.error or 'ok'}", flush=True)
    out["process_start_to_first_launch_s"] = round(time.time() - _T0, 2)
    marks["first_launch_enqueued"] = round(time.time() - _T0, 4)
    out["marks"] = marks
    out["sleep_before_synth_s"] = args.sleep_before_synth
    out["bursts"].append(burst(torch, plan_a, stream, args.first, sampler, "first: right after synthesis",
                               sync=not args.no_sync_after_synth))
    print(json.dumps({k: v for k, v in out["bursts"][-1].items() if k != "per_launch"}), flush=True)
    if args.second:
        time.sleep(args.idle_s)
        out["bursts"].append(burst(torch, plan_a, stream, args.second, sampler,
                                   f"idle: same buffer after {args.idle_s} s idle"))
        print(json.dumps({k: v for k, v in out["bursts"][-1].items() if k != "per_launch"}), flush=True)
    if args.fresh:
        t0 = time.perf_counter()
        buf_b = bench.synth_tiled(torch, K, M, kind, dev, 20241016, tv)  # a second, newly allocated buffer
        out_b = torch.empty(ld, dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        out["synth_fresh_s"] = round(time.perf_counter() - t0, 2)
        plan_b = TiledFedAvgPlan(kind, buf_b, K, w, M, out_b, pw, tv=tv)
        out["bursts"].append(burst(torch, plan_b, stream, args.fresh, sampler, "fresh: a newly allocated 91 GB buffer"))
        print(json.dumps({k: v for k, v in out["bursts"][-1].items() if k != "per_launch"}), flush=True)
        out["outputs_equal"] = bool(torch.equal(out_a[:M].view(torch.int32), out_b[:M].view(torch.int32)))
    if args.old:
        out["bursts"].append(burst(torch, plan_a, stream, args.old, sampler, "old: the first buffer again"))
        print(json.dumps({k: v for k, v in out["bursts"][-1].items() if k != "per_launch"}), flush=True)
    sampler.stop_ev.set()
    sampler.join(timeout=2)
    out["sampler"]["samples"] = len(sampler.samples)
    # the whole process's trace of the firmware-averaged clocks and activity (seconds since process
    # start), to place the SOC clock's fall against the marks above
    t_off = time.time() - time.perf_counter() - _T0
    out["trace"] = [[round(t + t_off, 4)] + [m.get(f) for f in TRACE_FIELDS] for t, m in sampler.samples]
    out["trace_fields"] = ["t_s"] + list(TRACE_FIELDS)
    out["sampler"]["error"] = sampler.error
    if sampler.samples:
        dt = np.diff([t for t, _ in sampler.samples])
        out["sampler"]["median_interval_ms"] = round(float(np.median(dt)) * 1e3, 3) if len(dt) else None
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(out))
    print("done", flush=True)


if __name__ == "__main__":
    os.environ.setdefault("PYTHONUNBUFFERED", "1")
    main()
