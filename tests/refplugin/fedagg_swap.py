"""pytest plugin (CONTAINER-ONLY checker, ``-p fedagg_swap``; tests/reference_own_tests.py): runs
the reference's OWN test suite with its strategy and torch algorithm classes swapped for the
accelerated ones -- ``substrafl.strategies.{FedAvg, Scaffold, FedPCA, NewtonRaphson}`` ->
``accelerate(...)`` and ``substrafl.algorithms.pytorch.{TorchFedAvgAlgo, TorchScaffoldAlgo}`` ->
``accelerate_algo(...)`` -- before any test module imports them.  No GPU here: the engine behind
the accelerated aggregation bodies is the oracle-backed double (refplugin/oracle_engine.py); the
client algorithms take their torch loops on the CPU.  The engine's call counts are written to
$FEDAGG_SWAP_REPORT at the end of the session."""

import json
import os

import fedagg_refstubs  # noqa: F401  (stubs for substra / substratools / docker first)
from oracle_engine import OracleEngine

import substrafl.algorithms.pytorch as P  # noqa: E402
import substrafl.strategies as S  # noqa: E402
import substrafl_amd.integration as integ  # noqa: E402
import substrafl_amd.strategies.fed_avg as mirror  # noqa: E402

ENGINE = OracleEngine()
integ.engine_for = mirror.engine_for = lambda device=None: ENGINE
SWAPPED = {}
for name in ("FedAvg", "Scaffold", "FedPCA", "NewtonRaphson"):
    setattr(S, name, integ.accelerate(getattr(S, name)))
    SWAPPED[name] = getattr(S, name).__qualname__
for name in ("TorchFedAvgAlgo", "TorchScaffoldAlgo"):
    setattr(P, name, integ.accelerate_algo(getattr(P, name)))
    SWAPPED[name] = getattr(P, name).__qualname__


def pytest_sessionfinish(session, exitstatus):
    path = os.environ.get("FEDAGG_SWAP_REPORT")
    if path:
        with open(path, "w") as f:
            json.dump({"engine_calls": ENGINE.calls, "swapped": SWAPPED}, f)
