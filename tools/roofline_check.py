#!/usr/bin/env python3
"""Put a bench line's roofline next to the rocprofv3 summary it must agree with.

tools/profile_round.sh runs, per workload, the plain bench line and then the SAME command under
``rocprofv3 --kernel-trace --stats``; that second line's HIP-event kernel time comes from the very
process rocprof traced.  This writes one JSON per workload with the three views of the dominant
kernel -- plain run (HIP events), profiled run (HIP events) and rocprof (average / min / max over
every launch of the process, warm-up and single launches included) -- and the roofline fraction
each gives, so the line's ``roofline.frac`` can be reproduced from ``profiles/``.

    python3 tools/roofline_check.py --bench B.json --profiled P.json --stats S.csv --kernel fedavg_kernel
"""

from __future__ import annotations

import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench", required=True, help="the plain bench line (JSON)")
    ap.add_argument("--profiled", required=True, help="the bench line printed under rocprofv3")
    ap.add_argument("--stats", required=True, help="rocprofv3 *_kernel_stats.csv of that run")
    ap.add_argument("--kernel", required=True, help="kernel name prefix (after 'void (anonymous namespace)::')")
    ap.add_argument("--group", type=int, default=1, help="launches per step (Scaffold one-bucket pair: 2)")
    ap.add_argument("--trace", default="", help="rocprofv3 *_kernel_trace.csv of that run: per-launch durations")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    def line(path):
        with open(path) as f:
            return json.loads([ln for ln in f if ln.startswith("{")][-1])

    plain, prof = line(args.bench), line(args.profiled)
    peak = plain["roofline"]["peak"]
    nbytes = plain["config"]["bytes_alg_per_launch_rank0"]
    rows = []
    with open(args.stats) as f:
        for r in csv.DictReader(f):
            name = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            if name.startswith(args.kernel):
                rows.append(r)
    calls = sum(int(r["Calls"]) for r in rows)
    total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    avg_ms = total_ns / max(1, calls) / 1e6 * args.group
    mn = min((float(r["MinNs"]) for r in rows), default=0.0) / 1e6 * args.group
    mx = max((float(r["MaxNs"]) for r in rows), default=0.0) / 1e6 * args.group

    def frac(ms):
        return round(nbytes / (ms / 1e3) / 1e9 / peak, 4) if ms else None

    def view(ln):
        rf = ln["roofline"]
        return {"kernel_ms": rf["kernel_ms"], "kernel_ms_median": rf.get("kernel_ms_median"),
                "kernel_ms_min": rf.get("kernel_ms_min"), "frac": rf["frac"], "ms_per_step": ln["ms_per_step"],
                "lib_sha256": ln.get("build", {}).get("lib_sha256")}

    out = {
        "workload": plain["config"]["workload"],
        "bytes_alg_per_step": nbytes,
        "peak_GBps": peak,
        "plain_bench_hip_events": view(plain),
        "profiled_bench_hip_events": view(prof),
        "rocprof": {"kernel": args.kernel, "launches_per_step": args.group, "calls": calls,
                    "avg_ms_per_step": round(avg_ms, 5), "min_ms": round(mn, 5), "max_ms": round(mx, 5),
                    "frac_avg": frac(avg_ms), "frac_min": frac(mn)},
        "profiled_events_vs_rocprof_avg": round(prof["roofline"]["kernel_ms"] / avg_ms - 1, 4) if avg_ms else None,
        "plain_vs_profiled": round(plain["roofline"]["kernel_ms"] / prof["roofline"]["kernel_ms"] - 1, 4),
    }
    if args.trace:
        out["per_launch"] = per_launch(args.trace, args.kernel, args.group, frac)
    text = json.dumps(out, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    print(text)


def per_launch(path, kernel, group, frac):
    """The kernel's launches in the traced process, in order (VERDICT r05 "Next 2"): the first
    launch apart (the first touch of a fresh allocation and the clock ramp), the steady state
    (median of the second half), and the split of the launches after the first into two levels that
    leaves the least squared error (a step, if the process has one) with the mean on either side."""
    d = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            if name.startswith(kernel):
                d.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    d = [ms for _, ms in sorted(d)]
    if group > 1:  # launches of one step summed
        d = [sum(d[i: i + group]) for i in range(0, len(d) - group + 1, group)]
    if len(d) < 6:
        return {"launches": len(d)}
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    steady = med(d[len(d) // 2:])
    best = None
    rest = d[1:]  # the first launch is reported apart: the step is looked for after it
    for s in range(2, len(rest) - 1):
        a, b = rest[:s], rest[s:]
        ma, mb = sum(a) / len(a), sum(b) / len(b)
        err = sum((x - ma) ** 2 for x in a) + sum((x - mb) ** 2 for x in b)
        if best is None or err < best[0]:
            best = (err, s, ma, mb)
    _, s, ma, mb = best
    return {"launches": len(d), "first_ms": round(d[0], 5), "frac_first": frac(d[0]),
            "steady_ms": round(steady, 5), "frac_steady": frac(steady),
            "mean_after_first_ms": round(sum(d[1:]) / (len(d) - 1), 5),
            "step": {"at_launch": s + 1, "mean_before_ms": round(ma, 5), "mean_after_ms": round(mb, 5),
                     "relative": round(ma / mb - 1, 4)}}


if __name__ == "__main__":
    main()
