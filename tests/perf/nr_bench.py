"""NewtonRaphson's aggregation (newton_raphson.py:195-216) on the engine against the reference's
NumPy sequence (the oracle's restatement of the same calls), host inputs in both cases:
K clients' P x P float64 Hessians + P float32 gradients.  Reports the weighted sums (engine:
staging + kernels + fetch, i.e. PCIe-inclusive) and the dense solve, which both paths run with
NumPy on the host.  One JSON line per (K, P); sums checked bit for bit.

    python3 tests/perf/nr_bench.py --configs 8x2048,8x4096,16x4096
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="8x2048,8x4096,16x4096")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from oracle import newton_raphson_sums
    from standin_substrafl.strategies.schemas import NewtonRaphsonSharedState
    from substrafl_amd.integration import newton_raphson_sums as engine_sums

    for cfg in args.configs.split(","):
        K, P = (int(v) for v in cfg.split("x"))
        rng = np.random.default_rng(K + P)
        grads = [[rng.standard_normal(P).astype(np.float32)] for _ in range(K)]
        hess = [rng.standard_normal((P, P)) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 1000, K)]
        states = [NewtonRaphsonSharedState(gradients=g, hessian=h, n_samples=n) for g, h, n in zip(grads, hess, ns)]
        engine_sums(states)  # warm: session, ring, buffers
        t_eng, t_ref = [], []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            H, G = engine_sums(states)
            t_eng.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            Hr, Gr = newton_raphson_sums(grads, hess, ns)
            t_ref.append(time.perf_counter() - t0)
        same = np.array_equal(H.view(np.uint64), Hr.view(np.uint64)) and np.array_equal(G.view(np.uint32),
                                                                                        Gr.view(np.uint32))
        t0 = time.perf_counter()
        np.linalg.solve(Hr + np.eye(P) * P, Gr)
        t_solve = time.perf_counter() - t0
        nbytes = K * P * P * 8 + K * P * 4
        print(json.dumps({"clients": K, "params": P, "input_bytes": nbytes, "sums_engine_s": round(min(t_eng), 4),
                          "sums_reference_numpy_s": round(min(t_ref), 4),
                          "speedup": round(min(t_ref) / min(t_eng), 2),
                          "engine_GBps_pcie_inclusive": round(nbytes / min(t_eng) / 1e9, 1),
                          "solve_s_host_both_paths": round(t_solve, 4), "sums_bit_identical": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
