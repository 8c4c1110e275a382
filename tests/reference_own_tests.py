"""CONTAINER-ONLY checker (runs /root/reference's own test files in place; never on the GPU box):
the reference's OWN unit tests of the strategies and torch algorithms, run twice on the same
files --

  * baseline: the unmodified classes (with the import stubs for the absent substra packages,
    refplugin/fedagg_refstubs.py);
  * swapped: ``substrafl.strategies.{FedAvg, Scaffold, FedPCA, NewtonRaphson}`` replaced by
    ``accelerate(...)`` and ``substrafl.algorithms.pytorch.{TorchFedAvgAlgo, TorchScaffoldAlgo}``
    by ``accelerate_algo(...)`` before the test modules import them (refplugin/fedagg_swap.py;
    the aggregation engine is the oracle-backed double, there is no GPU here) --

and compares the outcome of every test id: a test the reference passes must pass with the
accelerated classes.  (The baseline failures are the graph-building tests that need a real
``substra`` SDK -- SURVEY.md §4.)  Nothing is written under /root/reference (no bytecode, no cache,
the junit reports go to a temporary directory).  Prints one JSON line.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import xml.etree.ElementTree as ET
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent
REF = Path("/root/reference")
FILES = ["tests/strategies/test_fed_avg.py", "tests/strategies/test_scaffold.py",
         "tests/strategies/test_newton_raphson.py", "tests/strategies/test_fed_pca.py",
         "tests/algorithms/pytorch/test_fed_avg.py", "tests/algorithms/pytorch/test_scaffold.py",
         "tests/algorithms/pytorch/test_weight_manager.py"]


def run(plugin: str, tmp: Path):
    junit = tmp / f"{plugin}.xml"
    report = tmp / f"{plugin}.json"
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", FEDAGG_SWAP_REPORT=str(report),
               PYTHONPATH=os.pathsep.join([str(HERE / "refplugin"), str(ROOT), str(REF)]))
    cmd = [sys.executable, "-m", "pytest", "-p", plugin, "-p", "no:cacheprovider", "--rootdir", str(REF),
           *[str(REF / f) for f in FILES], "-m", "not substra and not slow and not gpu", "--mode=subprocess",
           "-q", f"--junitxml={junit}", "-p", "no:randomly"]
    r = subprocess.run(cmd, cwd=tmp, env=env, capture_output=True, text=True, timeout=1200)
    outcomes = {}
    for case in ET.parse(junit).getroot().iter("testcase"):
        tid = f"{case.get('classname')}::{case.get('name')}"
        if case.find("failure") is not None or case.find("error") is not None:
            outcomes[tid] = "failed"
        elif case.find("skipped") is not None:
            outcomes[tid] = "skipped"
        else:
            outcomes[tid] = outcomes.get(tid, "passed")
    extra = json.loads(report.read_text()) if report.exists() else {}
    return outcomes, extra, r.returncode


def main():
    if not REF.exists():
        raise SystemExit("reference_own_tests.py needs /root/reference (build container only)")
    with tempfile.TemporaryDirectory() as d:
        tmp = Path(d)
        base, _, _ = run("fedagg_refstubs", tmp)
        swap, extra, _ = run("fedagg_swap", tmp)
    passed = sorted(t for t, o in base.items() if o == "passed")
    lost = sorted(t for t in passed if swap.get(t) != "passed")
    print(json.dumps({"tests": len(base), "passed_reference": len(passed),
                      "passed_accelerated": sum(1 for o in swap.values() if o == "passed"),
                      "passed_by_reference_but_not_accelerated": lost,
                      "failed_reference": sorted(t for t, o in base.items() if o == "failed"),
                      "engine_calls": extra.get("engine_calls"), "swapped": extra.get("swapped")}))


if __name__ == "__main__":
    main()
