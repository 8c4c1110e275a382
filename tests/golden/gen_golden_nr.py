"""Golden vectors of ``NewtonRaphson.compute_averaged_states`` produced by the REFERENCE itself
(substrafl/strategies/newton_raphson.py:151-216), called with ``_skip=True`` as the aggregate task
does.  CONTAINER-ONLY (imports /root/reference, refuses to run without it), like gen_golden.py;
writes ``golden_newton_raphson.npz`` + ``golden_newton_raphson_meta.json`` next to it.

Cases: the reference's own unit-test inputs (tests/strategies/test_newton_raphson.py:15-32,
integer gradients and Hessians), random fp64 Hessians (symmetric, diagonally dominant) with fp32
gradient layers including numel == 1 ones, client counts 1-17, a zero-sample client, and
``-0.0`` off-diagonal Hessian entries shared by every client (the reference's explicit ``+=``
chain keeps them ``-0.0``; NumPy's ``np.sum`` would give ``+0.0``).  Run:
    python tests/golden/gen_golden_nr.py
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True
HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
from gen_golden import REF, _install_stubs  # noqa: E402


def _import():
    if not REF.exists():
        raise SystemExit("gen_golden_nr.py needs /root/reference (build container only)")
    _install_stubs()
    sys.path.insert(0, str(REF))
    from substrafl.algorithms.algo import Algo
    from substrafl.remote.decorators import remote_data
    from substrafl.strategies import NewtonRaphson
    from substrafl.strategies.schemas import NewtonRaphsonSharedState, StrategyName

    class DummyAlgo(Algo):  # tests/conftest.py:395-421
        strategies = property(lambda self: list(StrategyName))
        model = property(lambda self: "model")

        @remote_data
        def train(self, data_from_opener, shared_state):
            return None

        def predict(self, data_from_opener, shared_state):
            return None

        def load_local_state(self, path):
            return self

        def save_local_state(self, path):
            pass

    return NewtonRaphson, NewtonRaphsonSharedState, DummyAlgo


def _hessian(rng, P, neg_zero_mask=None):
    a = rng.standard_normal((P, P))
    h = (a + a.T) * 0.5 + np.eye(P) * (P + 1.0)
    if neg_zero_mask is not None:
        h[neg_zero_mask] = -0.0
    return h


def main():
    NewtonRaphson, State, DummyAlgo = _import()
    arrays, cases = {}, []

    def record(key, grads, hess, ns, damping):
        strategy = NewtonRaphson(algo=DummyAlgo(), damping_factor=damping)
        states = [State(gradients=g, hessian=h, n_samples=n) for g, h, n in zip(grads, hess, ns)]
        out = strategy.compute_averaged_states(shared_states=states, _skip=True).parameters_update
        L = len(grads[0])
        for k in range(len(grads)):
            arrays[f"{key}/k{k}/h"] = hess[k]
            for li in range(L):
                arrays[f"{key}/k{k}/g{li}"] = grads[k][li]
        arrays[f"{key}/n_samples"] = np.array(ns, dtype=np.int64)
        for li, o in enumerate(out):
            arrays[f"{key}/out{li}"] = o
        cases.append({"key": key, "K": len(grads), "layers": L, "outputs": len(out), "damping_factor": damping})

    # the reference's unit-test inputs (integer arrays: int64 x Python float -> float64)
    record("unit0", [[np.array([[2]]), np.array([2])], [np.array([[1]]), np.array([1])]],
           [np.array([[1, 0], [0, 1]]), np.array([[1, 0], [0, 1]])], [1, 1], 1)
    record("unit1", [[np.array([[6, 4]]), np.array([3])], [np.array([[3, 1]]), np.array([3])]],
           [np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1]]), np.array([[4, 0, 0], [0, 4, 0], [0, 0, 4]])], [1, 2], 0.8)

    rng = np.random.default_rng(20241016)
    for K, P, damping in ((1, 5, 1.0), (2, 3, 0.5), (3, 33, 1.0), (8, 17, 0.8), (9, 40, 1.0), (17, 12, 0.25)):
        shapes = [(P - 1,), (1,)] if P > 2 else [(P,)]
        grads = [[(rng.standard_normal(s) * 10.0 ** rng.integers(-2, 2)).astype(np.float32) for s in shapes]
                 for _ in range(K)]
        hess = [_hessian(rng, P) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 5000, K)]
        record(f"rand_K{K}_P{P}", grads, hess, ns, damping)

    # -0.0 off-diagonal entries in every client's Hessian, a zero-sample client, -0.0 gradients
    P, K = 9, 5
    mask = np.zeros((P, P), bool)
    mask[0, 3] = mask[3, 0] = mask[2, 7] = mask[7, 2] = True
    grads = [[np.where(rng.random(P) < 0.3, np.float32(-0.0), rng.standard_normal(P).astype(np.float32))]
             for _ in range(K)]
    for g in grads:
        g[0][4] = np.float32(-0.0)  # one gradient column -0.0 in every client
    hess = [_hessian(rng, P, mask) for _ in range(K)]
    record("negzero", grads, hess, [7, 0, 3, 11, 2], 1.0)

    np.savez_compressed(HERE / "golden_newton_raphson.npz", **arrays)
    (HERE / "golden_newton_raphson_meta.json").write_text(json.dumps(
        {"generator": "tests/golden/gen_golden_nr.py", "reference": "substrafl v1.0.0 NewtonRaphson.compute_averaged_states",
         "numpy": np.__version__, "cases": cases}, indent=1))
    print(f"{len(cases)} cases, {len(arrays)} arrays")


if __name__ == "__main__":
    main()
