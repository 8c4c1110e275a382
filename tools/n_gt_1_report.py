"""Read the N > 1 bench lines (a driver SCALE / MULTICHIP record, or bench.py's own output) and print
what DESIGN.md §9.4 says to read from the first multi-GPU run, flagging what is wrong:

* per N: the parameter-range value (GB/s, fraction of N x 8 TB/s) and the efficiency T(1)/T(N)
  when the N = 1 line is there;
* per client-shard leg: errors / skips, bit-exactness of the spot check, the push leg's full
  comparison with the native executor (must be 0 mismatches), its wait errors and late landing
  tags, ncclCommCount (must equal N), weak / strong efficiency, block kernel vs exchange time;
* whether the weak legs' output checksums agree (one expected output);
* the strong "C3 as written" gather leg and the xGMI probe of the torch leg.

  python tools/n_gt_1_report.py SCALE_r05.json [more files]     (exit 1 if anything is flagged)
"""

from __future__ import annotations

import json
import sys
from pathlib import Path


def _lines(obj):
    """Every bench line (a dict with "metric" and "n_gpus") anywhere inside ``obj``."""
    if isinstance(obj, dict):
        if "metric" in obj and "n_gpus" in obj:
            yield obj
        for v in obj.values():
            yield from _lines(v)
    elif isinstance(obj, list):
        for v in obj:
            yield from _lines(v)
    elif isinstance(obj, str) and obj.lstrip().startswith("{"):
        for ln in obj.splitlines():
            try:
                yield from _lines(json.loads(ln))
            except ValueError:
                pass


def _load(path: Path):
    text = path.read_text()
    try:
        yield from _lines(json.loads(text))
    except ValueError:  # JSON lines
        for ln in text.splitlines():
            if ln.strip().startswith("{"):
                try:
                    yield from _lines(json.loads(ln))
                except ValueError:
                    pass


def report(lines) -> list:
    flags = []
    by_n = {}
    for ln in lines:
        by_n.setdefault(int(ln["n_gpus"]), ln)
    t1 = by_n.get(1, {}).get("ms_per_step")
    for n in sorted(by_n):
        ln = by_n[n]
        eff = round(t1 / ln["ms_per_step"], 4) if t1 and ln.get("ms_per_step") and ln.get("scaling") == "weak" else None
        print(f"N={n}: value {ln.get('value')} {ln.get('unit')}  ms/step {ln.get('ms_per_step')}  "
              f"frac_of_n_x_peak {ln.get('frac_of_n_x_hbm_peak', ln.get('roofline', {}).get('frac'))}  "
              f"T(1)/T(N) {eff}  parity {ln.get('parity')}")
        if (ln.get("parity") or {}).get("mismatches"):
            flags.append(f"N={n}: parameter-range spot check mismatches")
        quiet = ln.get("device_quiet") or {}
        if quiet.get("waited_s") is not None:  # bench.wait_device_quiet: the driver's clear of freed VRAM
            print(f"  waited {quiet['waited_s']} s for the driver's clear (SOC clock {quiet.get('soc_clock_mhz_at_check')}"
                  f" -> {quiet.get('soc_clock_mhz_at_start')} MHz)")
        if quiet.get("gave_up"):
            flags.append(f"N={n}: timed while the driver was still clearing freed memory (gave up after "
                         f"{quiet.get('waited_s')} s)")
        for key in ln.get("legs_order", []):
            leg = ln.get(key) or {}
            if "error" in leg or "skipped" in leg:
                print(f"  {key}: {'ERROR ' + str(leg['error'])[:300] if 'error' in leg else 'skipped: ' + str(leg['skipped'])}")
                if "error" in leg:
                    flags.append(f"N={n} {key}: error")
                continue
            parts = [f"ms/step {leg.get('ms_per_step')}", f"weak_eff {leg.get('weak_efficiency')}",
                     f"speedup {leg.get('speedup')}", f"block {leg.get('block_kernel_ms')} ms",
                     f"exchange+tail {leg.get('exchange_and_tail_ms')} ms"]
            if (leg.get("parity") or {}).get("mismatches"):
                flags.append(f"N={n} {key}: spot check mismatches {leg['parity']}")
            if (leg.get("device_quiet") or {}).get("gave_up"):
                flags.append(f"N={n} {key}: timed while the driver was still clearing freed memory")
            if leg.get("connect_s") is not None:
                parts.append(f"set-up {leg['connect_s']} s of {leg.get('connect_deadline_s')} s")
                if leg.get("connect_deadline_s") and leg["connect_s"] > 0.8 * leg["connect_deadline_s"]:
                    flags.append(f"N={n} {key}: set-up took {leg['connect_s']} s, over 80 % of its "
                                 f"{leg['connect_deadline_s']} s deadline")
            fc = leg.get("full_compare")
            if isinstance(fc, dict) and "mismatches" in fc:
                parts.append(f"full_compare {fc['mismatches']}/{fc.get('elements')}")
                if fc["mismatches"]:
                    flags.append(f"N={n} {key}: push vs native full comparison differs in {fc['mismatches']} elements")
            if "wait_errors" in leg:
                parts.append(f"late_tags {leg.get('late_landing_tags')}")
                if leg["wait_errors"]:
                    flags.append(f"N={n} {key}: wait errors {leg['wait_errors']}")
            if "rccl_comm_count" in leg:
                parts.append(f"ncclCommCount {leg['rccl_comm_count']}")
                if leg["rccl_comm_count"] != n:
                    flags.append(f"N={n} {key}: ncclCommCount {leg['rccl_comm_count']} != {n}")
            if key == "param_range_strong_gather":
                parts.append(f"gather {leg.get('gather_ms')} ms")
                pipe = leg.get("pipelined") or {}
                parts.append(f"pipelined {pipe.get('ms_per_step')} ms/step speedup {pipe.get('speedup')}"
                             if "error" not in pipe else f"pipelined ERROR {str(pipe['error'])[:120]}")
                if pipe.get("gathered_slice_checksum_mismatches"):
                    flags.append(f"N={n} {key}: pipelined gather slices differ")
            if isinstance(leg.get("xgmi_p2p"), dict):
                parts.append(f"xgmi {json.dumps(leg['xgmi_p2p'])[:200]}")
            print(f"  {key}: " + ", ".join(parts))
        sums = ln.get("client_shard_output_checksums")
        if isinstance(sums, dict):
            print(f"  weak legs' output checksums: {sums}")
            if sums.get("agree") is False:
                flags.append(f"N={n}: the weak legs' outputs differ")
        md = ln.get("multi_device")
        if isinstance(md, dict):
            print(f"  multi_device: {'ERROR ' + str(md['error'])[:200] if 'error' in md else md.get('value')}")
    return flags


def main(argv):
    if not argv:
        print(__doc__)
        return 2
    lines = [ln for p in argv for ln in _load(Path(p))]
    if not lines:
        print("no bench lines found")
        return 2
    flags = report(lines)
    print("FLAGS:" if flags else "no flags")
    for f in flags:
        print("  " + f)
    return 1 if flags else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
