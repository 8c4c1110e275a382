#!/usr/bin/env python3
"""Summarise tools/turnaround_counters.sh's PMC passes per product kernel (VERDICT r04 "Next 5").

Per kernel (one template instance; C4's Scaffold call is two one-bucket launches, reported
separately), medians over its dispatches of:
  * read / write memory-side requests (TCC_EA0_RDREQ / WRREQ) and the write share of them;
  * average memory-side read and write latency in cycles: LEVEL / REQ (the counter description's
    own formula: the integral of requests in flight over cycles, divided by the requests);
  * DRAM credit stalls of reads and writes, the EA write-request stall and the too-many-writes
    stall, each as a fraction of channel-cycles (the _sum counters add 8 XCCs x 16 channels;
    GRBM_GUI_ACTIVE adds the 8 XCCs' busy cycles);
  * the same for bench.py's read-only probe kernels (read_probe*), the control: a pure read
    stream at the box's read ceiling.
Usage: turnaround_counters.py --tag TAG --dir gpurun_out c2 c4 c3
"""

import argparse
import csv
import json
import statistics
from collections import defaultdict
from pathlib import Path

PRODUCT = ("fedavg_kernel", "scaffold_bucket_kernel", "scaffold_kernel", "read_probe")  # + the read-only control
XCC, CHANNELS = 8, 16  # GRBM_GUI_ACTIVE sums the 8 XCCs' busy cycles; the TCC _sum counters 8 x 16 channels


def load(path):
    """{kernel name: {dispatch: {counter: value}}} of the product kernels."""
    out = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if not any(p in name for p in PRODUCT):
                continue
            d = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
            out[name][d][row["Counter_Name"]] += float(row["Counter_Value"])
    return out


def med(vals):
    return statistics.median(vals) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--dir", required=True)
    ap.add_argument("workloads", nargs="+")
    a = ap.parse_args()
    res = {"counters": "rocprofv3 --pmc, two passes per workload (tools/turnaround_counters.sh)",
           "latency_formula": "TCC_EA0_{RD,WR}REQ_LEVEL / TCC_EA0_{RD,WR}REQ (cycles)", "kernels": {}}
    for wl in a.workloads:
        A = load(Path(a.dir) / f"{a.tag}_{wl}_pmcA.csv")
        B = load(Path(a.dir) / f"{a.tag}_{wl}_pmcB.csv")
        for name in sorted(set(A) | set(B)):
            da, db = A.get(name, {}), B.get(name, {})
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split(">(")[0].split("(")[0] + ">"

            def col(d, c):
                return [v[c] for v in d.values() if c in v]

            rd, wr = med(col(da, "TCC_EA0_RDREQ_sum")), med(col(da, "TCC_EA0_WRREQ_sum"))
            rl, wl_ = med(col(da, "TCC_EA0_RDREQ_LEVEL_sum")), med(col(da, "TCC_EA0_WRREQ_LEVEL_sum"))
            cyc_a, cyc_b = med(col(da, "GRBM_GUI_ACTIVE")), med(col(db, "GRBM_GUI_ACTIVE"))
            rec = {"workload": wl, "dispatches": len(da), "rdreq": rd, "wrreq": wr,
                   "write_share_of_requests": round(wr / (rd + wr), 4) if rd and wr else None,
                   "read_latency_cycles": round(rl / rd, 1) if rl and rd else None,
                   "write_latency_cycles": round(wl_ / wr, 1) if wl_ and wr else None,
                   "xcc_cycles": round(cyc_a / XCC) if cyc_a else None}
            for c, key in (("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "rd_dram_credit_stall_frac"),
                           ("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", "wr_dram_credit_stall_frac"),
                           ("TCC_EA0_WRREQ_STALL_sum", "ea_wrreq_stall_frac"),
                           ("TCC_TOO_MANY_EA_WRREQS_STALL_sum", "too_many_wrreqs_stall_frac")):
                v = med(col(db, c))
                # a fraction of channel-cycles: the sum over 128 channels / (8 x per-XCC cycles x 16)
                rec[key] = round(v / (cyc_b * CHANNELS), 5) if v is not None and cyc_b else None
            res["kernels"][f"{wl}: {short}"] = rec
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
