"""Test double of :class:`substrafl_amd.engine.AggregationEngine` for the GPU-less build container
(TEST INFRASTRUCTURE ONLY): the engine's entry points computed by the oracle's restatements
(oracle/aggregation.py, pinned bit-exact by the golden vectors the reference produced), each call
counted.  Used where the reference's own drivers or tests exercise ``accelerate``'d classes here
(tests/reference_drop_in.py, tests/reference_own_tests.py); the GPU side of the same calls is the
golden replay through the real engine (tests/test_accelerate_standin.py, test_newton_raphson.py)."""

import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from oracle import fedavg_explicit, scaffold_explicit  # noqa: E402


class OracleEngine:
    def __init__(self):
        self.calls = {"fedavg": 0, "scaffold": 0, "sequential": 0}

    def fedavg(self, parameters_updates, n_samples, wire=False):
        assert not wire, "reference schemas take plain NumPy arrays"
        self.calls["fedavg"] += 1
        dts = {a.dtype for pu in parameters_updates for a in pu}
        if dts <= {np.dtype(np.float32), np.dtype(np.float64)} and len(dts) == 1:
            return fedavg_explicit(parameters_updates, n_samples)
        # other dtypes (the reference's integer unit-test inputs): NumPy's own promotion, as the
        # engine reproduces on the device (fed_avg.py:217-222)
        n_all = sum(n_samples)
        return [np.sum([pu[i] * (n / n_all) for pu, n in zip(parameters_updates, n_samples)], axis=0)
                for i in range(len(parameters_updates[0]))]

    def scaffold(self, parameters_updates, control_variate_updates, server_control_variates, n_samples,
                 aggregation_lr, wire=False):
        assert not wire
        self.calls["scaffold"] += 1
        c0 = server_control_variates[0]
        mism = 0
        for ci in server_control_variates[1:]:
            for a, b in zip(c0, ci):
                a, b = np.asarray(a), np.asarray(b)
                mism += int(np.sum(~((a == b) | (np.isnan(a) & np.isnan(b)))))
        new_c, avg = scaffold_explicit(parameters_updates, control_variate_updates, c0, n_samples, aggregation_lr)
        return mism, new_c, avg

    def sequential_sum(self, rows, n_samples, wire=False):
        """NewtonRaphson's chain (newton_raphson.py:195-211), per layer."""
        assert not wire
        self.calls["sequential"] += 1
        n_all = sum(n_samples)
        out = []
        for li in range(len(rows[0])):
            total = None
            for k, row in enumerate(rows):
                p = row[li] * (n_samples[k] / n_all)
                if total is None:
                    total = p
                else:
                    total += p
            out.append(total)
        return out
