#!/usr/bin/env python3
"""Per-launch HBM bytes of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Corrections per MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7: both counters are in
KiB; on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide coalesced streaming read
(128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane
streaming stores.  Usage:
  pmc_traffic.py --fetch <dir>/..._counter_collection.csv --write <...csv> --kernel fedavg_kernel
                 --bytes-alg 900000000 --out profiles/traffic_c2.json
"""

import argparse
import csv
import json
from pathlib import Path


def per_dispatch(path, counter, kernel, group=1):
    """Counter total per dispatch of ``kernel`` (substring of the name); with ``group`` > 1,
    totals of consecutive groups of that many dispatches (one call = several launches, e.g.
    Scaffold's two one-bucket launches)."""
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if kernel not in name:
                continue
            if row.get("Counter_Name") != counter:
                continue
            d = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    seq = [vals[d] for d in sorted(vals)]
    if group > 1:
        if len(seq) % group:
            raise SystemExit(f"{len(seq)} dispatches of {kernel} do not split into groups of {group}")
        seq = [sum(seq[i:i + group]) for i in range(0, len(seq), group)]
    return seq


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="fedavg_kernel")
    ap.add_argument("--bytes-alg", type=float, required=True)
    ap.add_argument("--group", type=int, default=1, help="launches per call (summed per call)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--lib", default="", help="libfedagg.so the passes ran (its sha256 goes into the record)")
    ap.add_argument("--collected", default="", help="free text: box / command / date of the passes")
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel, a.group)
    write = per_dispatch(a.write, "WRITE_SIZE", a.kernel, a.group)
    if not fetch or not write:
        raise SystemExit(f"no rows for {a.kernel}: fetch={len(fetch)} write={len(write)}")
    f_kib = sorted(fetch)[len(fetch) // 2]
    w_kib = sorted(write)[len(write) // 2]
    read_b = 2.0 * f_kib * 1024  # gfx950: FETCH_SIZE = half the bytes of a wide streaming read
    write_b = w_kib * 1024
    res = {
        "kernel": a.kernel,
        "launches_per_call": a.group,
        "dispatches": {"fetch": len(fetch), "write": len(write)},
        "FETCH_SIZE_KiB_median": f_kib,
        "WRITE_SIZE_KiB_median": w_kib,
        "hbm_read_bytes_per_launch": read_b,
        "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "bytes_alg_per_launch": a.bytes_alg,
        "traffic_over_alg": (read_b + write_b) / a.bytes_alg,
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream tally), KiB x1024",
    }
    if a.lib:
        import hashlib

        res["lib_sha256"] = hashlib.sha256(Path(a.lib).read_bytes()).hexdigest()[:16]
    if a.collected:
        res["collected"] = a.collected
    Path(a.out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
