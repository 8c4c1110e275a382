"""Summarise round 6's VRAM-clear evidence ("C5 per launch") from the raw session
outputs into one JSON: scripts/r06_c5_sampled.sh (r06q), r06_c5_socclk.sh (r06r),
r06_socclk_seq.sh (r06s) and r06_quiet.sh (r06t).
  python tools/vram_clear_summary.py gpurun_out profiles/r06_vram_clear.json"""

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from c5_step_probe import step_split  # noqa: E402

HIGH = 300.0  # firmware-averaged SOC clock while the clear runs: 300-330 MHz; idle / own work 39-100


def probe_step(d):
    """C5 probe process: its launch-duration step (the first launch, the after-idle one, left out),
    the time of the step and of the SOC clock's fall since the process started."""
    b = d["bursts"][0]
    fl = d["process_start_to_first_launch_s"]
    pl = b["per_launch"][1:]
    s, a, c = step_split([r["ms"] for r in pl])
    rec = {"first_launch_s": fl, "ms_before": round(a, 3), "ms_after": round(c, 3),
           "step_pct": round((a - c) / a * 100, 2), "step_at_s": round(fl + pl[s]["start_s"], 3)}
    trace = d.get("trace") or []
    if trace:  # [t since process start, socclk, ...]
        rec["socclk_at_first_sample"] = trace[0][1]
        fall = [trace[i][0] for i in range(1, len(trace)) if trace[i - 1][1] >= HIGH > trace[i][1]]
        rec["socclk_fall_s"] = round(fall[0], 3) if fall else None
    elif b.get("samples"):  # r06q: the burst's samples only (seconds from the first launch)
        sm = b["samples"]
        rec["socclk_at_first_sample"] = sm[0][1]["current_socclks"]
        fall = [sm[i][0] for i in range(1, len(sm))
                if sm[i - 1][1]["current_socclks"] >= HIGH > sm[i][1]["current_socclks"]]
        rec["socclk_fall_s"] = round(fl + fall[0], 3) if fall else None
    return rec


def main(src, out):
    src = Path(src)
    res = {"what": "the driver's clear of a previous process's freed VRAM (SOC clock high) and C5's launch-duration step"}
    res["r06q_sampled_back_to_back"] = {p.stem: probe_step(json.loads(p.read_text()))
                                        for p in sorted(src.glob("r06q_p*.json"))}
    res["r06r_idle_before_alloc"] = {p.stem: dict(probe_step(json.loads(p.read_text())),
                                                  marks=json.loads(p.read_text())["marks"])
                                     for p in sorted(src.glob("r06r_*.json"))}
    # r06s: the standalone sampler's trace across predecessors of 91 / 45 / 8 / 0 / 91 GiB
    tr = json.loads((src / "r06s_trace.json").read_text())
    rows = tr["rows"]
    preds = [json.loads(ln) for ln in (src / "r06s_pred.jsonl").read_text().splitlines() if ln.strip()]
    exits = [p["exited"] for p in preds if "exited" in p]
    gibs = [p["gib"] for p in preds if "gib" in p] + ["c5 probe (92 GB)", "c5 probe (92 GB)"]
    windows = []
    for i, (g, ex) in enumerate(zip(gibs, exits)):
        nxt = exits[i + 1] if i + 1 < len(exits) else float("inf")
        after = [r for r in rows if ex - 1.0 <= r[0] <= min(ex + 4.0, nxt)]
        hi = [r[0] for r in after if r[1] is not None and r[1] >= HIGH]
        windows.append({"predecessor": g, "exit_wall": round(ex, 3),
                        "high_from_s": round(hi[0] - ex, 3) if hi else None,
                        "high_until_s": round(hi[-1] - ex, 3) if hi else None,
                        "high_s": round(hi[-1] - hi[0], 3) if hi else 0.0,
                        "clear_GBps": round(g * 1.073741824 / (hi[-1] - hi[0]), 1)
                        if hi and isinstance(g, float) and g > 0 and hi[-1] > hi[0] else None})
    res["r06s_predecessor_windows"] = windows
    res["r06s_probes"] = {p.stem: probe_step(json.loads(p.read_text())) for p in sorted(src.glob("r06s_c*.json"))}
    # the SOC clock at its change points (the firmware updates it every ~20 ms)
    pts, prev = [], None
    for r in rows:
        if r[1] != prev:
            pts.append([round(r[0] - rows[0][0], 3), r[1], r[4]])
            prev = r[1]
    res["r06s_socclk_change_points"] = {"fields": ["t_s", "current_socclks", "average_umc_activity"], "rows": pts}
    lines = {}
    for p in sorted(src.glob("r06t_*.json")):
        d = json.loads(p.read_text().strip().splitlines()[-1])
        r = d["roofline"]
        lines[p.stem] = {"workload": d["config"]["workload"], "ms_per_step": d["ms_per_step"],
                         "kernel_ms_mean_timed": r["kernel_ms"], "kernel_ms_median_after": r["kernel_ms_median"],
                         "frac": r["frac"], "device_quiet": d.get("device_quiet")}
    res["r06t_bench_after_a_91GB_process"] = lines
    Path(out).write_text(json.dumps(res, indent=1))
    print(json.dumps({k: v for k, v in res.items() if k != "r06s_socclk_change_points"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
