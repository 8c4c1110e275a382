"""Reduce a rocprofv3 kernel_trace.csv to the product kernel's launches (launch, kernel, start_ns,
end_ns, duration_ms), the form profiles/ keeps.
  python tools/reduce_trace.py IN.csv OUT.csv KERNEL_SUBSTRING"""

import csv
import sys


def main(src, dst, sub):
    rows = [r for r in csv.DictReader(open(src)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["launch", "kernel", "start_ns", "end_ns", "duration_ms"])
        for i, r in enumerate(rows):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            w.writerow([i, r["Kernel_Name"][:60], s, e, round((e - s) / 1e6, 5)])
    print(f"{dst}: {len(rows)} launches")


if __name__ == "__main__":
    main(*sys.argv[1:4])
