"""tools/n_gt_1_report.py: reads N > 1 bench lines wherever a record nests them and flags what
DESIGN.md §9.4 says must hold on the first multi-GPU run."""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

import n_gt_1_report as rep  # noqa: E402


def _line(n, **legs):
    return {"metric": "m", "n_gpus": n, "value": 1.0, "unit": "GB/s", "ms_per_step": 4.0 * (1 if n == 1 else 1.05),
            "scaling": "weak", "parity": {"mismatches": 0}, "legs_order": list(legs), **legs}


def test_clean_record_has_no_flags(tmp_path):
    rec = {"runs": [{"stdout": json.dumps(_line(1))}, {"line": _line(8, client_shard_push={
        "ms_per_step": 4.3, "weak_efficiency": 0.93, "parity": {"mismatches": 0}, "wait_errors": {},
        "late_landing_tags": 0, "full_compare": {"mismatches": 0, "elements": 10}},
        client_shard={"ms_per_step": 4.4, "parity": {"mismatches": 0}, "rccl_comm_count": 8})}]}
    p = tmp_path / "scale.json"
    p.write_text(json.dumps(rec))
    lines = list(rep._load(p))
    assert sorted(ln["n_gpus"] for ln in lines) == [1, 8]
    assert rep.report(lines) == []


def test_bad_legs_are_flagged():
    lines = [_line(8, client_shard_push={"parity": {"mismatches": 0}, "wait_errors": {3: "counter of rank 1"},
                                         "full_compare": {"mismatches": 5, "elements": 10}},
                   client_shard={"parity": {"mismatches": 2}, "rccl_comm_count": 7},
                   client_shard_torch_pg={"error": "leg exited with 1"})]
    lines[0]["client_shard_output_checksums"] = {"legs": ["a", "b"], "agree": False}
    flags = "\n".join(rep.report(lines))
    for needle in ("full comparison differs", "wait errors", "spot check mismatches", "ncclCommCount 7 != 8",
                   "client_shard_torch_pg: error", "outputs differ"):
        assert needle in flags, (needle, flags)


def test_timing_inside_the_drivers_clear_is_flagged(capsys):
    """bench.wait_device_quiet gave up (the driver still clearing freed VRAM when the timed region
    started): the line and the leg are flagged; a wait that ended is only printed."""
    ok = _line(2, client_shard={"ms_per_step": 4.4, "parity": {"mismatches": 0}, "rccl_comm_count": 2,
                                "device_quiet": {"waited_s": 0.8, "gave_up": False}})
    ok["device_quiet"] = {"waited_s": 1.3, "gave_up": False, "soc_clock_mhz_at_check": 328.5,
                          "soc_clock_mhz_at_start": 180.0}
    assert rep.report([ok]) == []
    assert "waited 1.3 s for the driver's clear" in capsys.readouterr().out
    bad = _line(8, client_shard={"ms_per_step": 4.4, "parity": {"mismatches": 0}, "rccl_comm_count": 8,
                                 "device_quiet": {"waited_s": 12.0, "gave_up": True}})
    bad["device_quiet"] = {"waited_s": 12.0, "gave_up": True}
    flags = "\n".join(rep.report([bad]))
    assert "N=8: timed while the driver was still clearing" in flags
    assert "N=8 client_shard: timed while the driver was still clearing" in flags
