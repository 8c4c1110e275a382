"""The PMC post-processing behind `roofline.traffic` (tools/pmc_traffic.py): per-dispatch totals,
launch grouping (Scaffold's one-bucket launch pair counts as one call), the gfx950 FETCH_SIZE
correction and the build tag.  CPU only, synthetic counter files."""

import csv
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

import pmc_traffic  # noqa: E402

FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]


def _write(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(FIELDS, r)))


def test_per_dispatch_sums_rows_and_filters_by_name(tmp_path):
    p = tmp_path / "c.csv"
    _write(p, [(3, "void fedavg_kernel<F32>", "FETCH_SIZE", 10.0), (3, "void fedavg_kernel<F32>", "FETCH_SIZE", 5.0),
               (1, "void fedavg_kernel<F32>", "FETCH_SIZE", 7.0), (2, "other", "FETCH_SIZE", 99.0),
               (1, "void fedavg_kernel<F32>", "WRITE_SIZE", 1.0)])
    assert pmc_traffic.per_dispatch(p, "FETCH_SIZE", "fedavg_kernel") == [7.0, 15.0]  # dispatch order


def test_per_dispatch_groups_launch_pairs(tmp_path):
    p = tmp_path / "c.csv"
    names = ["void scaffold_bucket_kernel<float, 64, true, 1, 8, 4, 0, false>",
             "void scaffold_bucket_kernel<float, 64, true, 1, 8, 4, 1, false>"]
    rows = [(d, names[d % 2], "WRITE_SIZE", float(100 + d)) for d in range(6)]
    _write(p, rows)
    assert pmc_traffic.per_dispatch(p, "WRITE_SIZE", "scaffold", group=2) == [201.0, 205.0, 209.0]
    _write(p, rows[:5])
    with pytest.raises(SystemExit):
        pmc_traffic.per_dispatch(p, "WRITE_SIZE", "scaffold", group=2)


def test_cli_applies_the_fetch_correction_and_records_the_build(tmp_path):
    fetch, write, lib, out = (tmp_path / n for n in ("f.csv", "w.csv", "lib.so", "t.json"))
    _write(fetch, [(d, "k", "FETCH_SIZE", 1000.0) for d in range(4)])
    _write(write, [(d, "k", "WRITE_SIZE", 250.0) for d in range(4)])
    lib.write_bytes(b"not a library")
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_traffic.py"), "--fetch", str(fetch), "--write",
                        str(write), "--kernel", "k", "--group", "2", "--bytes-alg", str(5000 * 1024),
                        "--lib", str(lib), "--out", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    res = json.loads(out.read_text())
    assert res["launches_per_call"] == 2
    assert res["hbm_read_bytes_per_launch"] == 2 * 2000.0 * 1024  # FETCH_SIZE x2, KiB, per call
    assert res["hbm_write_bytes_per_launch"] == 500.0 * 1024
    assert res["traffic_over_alg"] == pytest.approx(4500 / 5000)
    assert len(res["lib_sha256"]) == 16


def test_roofline_check_reports_first_launch_and_steady_state_apart(tmp_path):
    """VERDICT r05 "Next 2": from the traced process's per-launch durations, roofline_check puts the
    first launch (a fresh allocation's first touch, the clock ramp) and the steady state apart, and
    finds a step in the launch sequence if there is one."""
    import csv

    sys.path.insert(0, str(ROOT / "tools"))
    import roofline_check as rc

    p = tmp_path / "trace.csv"
    durs = [16.0] + [13.0] * 26 + [12.7] * 33  # first launch, then a 2.4 % step at launch 27
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        t = 1_000_000
        for ms in durs:
            w.writerow(["void (anonymous namespace)::fedavg_kernel<x>", t, t + int(ms * 1e6)])
            w.writerow(["read_probe_kernel", t + int(ms * 1e6), t + int(ms * 1e6) + 10])
            t += int(ms * 1e6) + 1000
    frac = lambda ms: round(91e9 / (ms / 1e3) / 1e9 / 8000, 4)  # noqa: E731
    res = rc.per_launch(str(p), "fedavg_kernel", 1, frac)
    assert res["launches"] == 60 and res["first_ms"] == 16.0 and res["steady_ms"] == 12.7
    assert res["step"]["at_launch"] == 27 and abs(res["step"]["relative"] - 0.0236) < 0.002
    assert res["frac_steady"] == frac(12.7)
