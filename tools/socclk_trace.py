"""Sample the GPU's firmware metrics (amdsmi gpu_metrics) every 2 ms from a process that does
no HIP work itself, for --seconds, and write [wall time, fields...] rows as JSON.  Run beside a
sequence of GPU processes (tools/alloc_exit.py) to see what each process's start, allocation
and exit do to the SOC clock -- the clock whose fall coincides with C5's launch-duration step
("C5 per launch")."""

import argparse
import json
import time

FIELDS = ("current_socclks", "current_gfxclks", "current_uclk", "average_umc_activity", "average_gfx_activity",
          "current_socket_power", "pcie_bandwidth_inst")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--period", type=float, default=0.002)
    args = ap.parse_args()
    import amdsmi

    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    rows, t_end = [], time.time() + args.seconds
    print("sampling", flush=True)
    while time.time() < t_end:
        t = time.time()
        m = amdsmi.amdsmi_get_gpu_metrics_info(h)
        row = [round(t, 4)]
        for f in FIELDS:
            v = m.get(f)
            if isinstance(v, list):
                v = [x for x in v if isinstance(x, (int, float))]
                v = sum(v) / len(v) if v else None
            row.append(v if isinstance(v, (int, float)) else None)
        rows.append(row)
        time.sleep(max(0.0, args.period - (time.time() - t)))
    amdsmi.amdsmi_shut_down()
    with open(args.out, "w") as f:
        json.dump({"fields": ["wall_s"] + list(FIELDS), "rows": rows}, f)
    print("done", len(rows), flush=True)


if __name__ == "__main__":
    main()
