"""The CPU oracle against the golden vectors captured from the reference (tests/golden/gen_golden.py)
and against NumPy itself.  CPU only."""

import numpy as np
import pytest

from oracle import (
    fedavg_explicit,
    fedavg_reference_structure,
    numpy_pairwise_sum,
    scaffold_explicit,
    scaffold_reference_structure,
)


def _bits(a):
    a = np.asarray(a)
    return a.view({4: np.uint32, 8: np.uint64, 2: np.uint16}[a.dtype.itemsize])


def _fedavg_case(arrays, case):
    key, K, L = case["key"], case["K"], case["layers"]
    ns = [int(v) for v in arrays[f"{key}/n_samples"]]
    xs = [arrays[f"{key}/x{li}"] for li in range(L)]
    pus = [[xs[li][k] for li in range(L)] for k in range(K)]
    outs = [arrays[f"{key}/out{li}"] for li in range(L)]
    return pus, ns, outs


def test_golden_fedavg_bit_exact(golden):
    arrays, meta = golden
    cases = [c for c in meta["cases"] if c["strategy"] == "fedavg"]
    assert len(cases) >= 40
    for case in cases:
        pus, ns, outs = _fedavg_case(arrays, case)
        for fn in (fedavg_reference_structure, fedavg_explicit):
            got = fn(pus, ns)
            for g, r in zip(got, outs):
                assert g.dtype == r.dtype and g.shape == r.shape, case
                assert np.array_equal(_bits(g), _bits(r)), (case, fn.__name__)


def test_golden_scaffold_bit_exact(golden):
    arrays, meta = golden
    for case in [c for c in meta["cases"] if c["strategy"] == "scaffold"]:
        key, K, L = case["key"], case["K"], case["layers"]
        ns = [int(v) for v in arrays[f"{key}/n_samples"]]
        lr = int(case["lr"]) if case["lr_is_int"] else float(case["lr"])
        pu = [[arrays[f"{key}/pu{li}"][k] for li in range(L)] for k in range(K)]
        cv = [[arrays[f"{key}/cv{li}"][k] for li in range(L)] for k in range(K)]
        c = [arrays[f"{key}/c{li}"] for li in range(L)]
        for fn in (scaffold_reference_structure, scaffold_explicit):
            new_c, avg = fn(pu, cv, c, ns, lr)
            for li in range(L):
                for g, r in ((new_c[li], arrays[f"{key}/newc{li}"]), (avg[li], arrays[f"{key}/avg{li}"])):
                    assert g.dtype == np.float64 == r.dtype
                    assert np.array_equal(_bits(g), _bits(r)), (case, li, fn.__name__)


def test_golden_reference_unit_known_answers(golden):
    """tests/strategies/test_fed_avg.py:17-54 known answers, as produced by the reference."""
    arrays, _ = golden
    np.testing.assert_array_equal(arrays["g5/unit_fedavg_0"], np.ones((5, 10)))
    np.testing.assert_array_equal(arrays["g5/unit_fedavg_1"], np.ones((5, 10)))
    np.testing.assert_array_equal(arrays["g5/unit_fedavg_2"], 1.5 * np.ones((5, 10)))
    assert np.allclose(arrays["g5/unit_fedavg_int64_0"], [[12, 15.25], [14, 16]])
    assert np.allclose(arrays["g5/unit_fedavg_int64_1"], [[18, 20], [22, 24]])
    # the oracle reproduces them bit for bit
    ns = [1, 3]
    pus = [
        [np.asarray([[0, 1], [2, 4]]), np.asarray([[6, 8], [10, 12]])],
        [np.asarray([[16, 20], [18, 20]]), np.asarray([[22, 24], [26, 28]])],
    ]
    got = fedavg_reference_structure(pus, ns)
    assert np.array_equal(got[0], arrays["g5/unit_fedavg_int64_0"]) and got[0].dtype == np.float64


def test_golden_error_conventions(golden):
    _, meta = golden
    assert meta["errors"] == {
        "fedavg_empty": "EmptySharedStatesError",
        "fedavg_zero_samples": "ZeroDivisionError",
        "fedavg_layer_count": "AssertionError",
        "fedavg_shape_mismatch": "ValueError",
        "fedavg_0d": "ValidationError",
        "fedavg_float_n_samples": "ValidationError",
        "scaffold_empty": "AssertionError",
        "scaffold_c_mismatch": "AssertionError",
        "scaffold_negative_lr": "ValueError",
    }


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_pairwise_matches_numpy(dtype):
    rng = np.random.default_rng(5)
    for K in list(range(1, 140)) + [255, 256, 257, 300, 1000, 1031]:
        v = (rng.standard_normal(K) * 10.0 ** rng.integers(-3, 3, K)).astype(dtype)
        ref = np.sum(v.reshape(K, 1), axis=0)[0]
        got = dtype(0.0) + numpy_pairwise_sum(v)
        assert _bits(np.array(got, dtype)) == _bits(np.array(ref, dtype)), K


def test_explicit_equals_structure_random():
    rng = np.random.default_rng(11)
    shapes = [(3, 5), (1,), (1, 1), (7,), (2, 1, 3)]
    for trial in range(60):
        K = int(rng.integers(1, 200))
        heavy = trial % 2
        pus = []
        for k in range(K):
            layers = []
            for s in shapes:
                x = rng.standard_normal(s).astype(np.float32)
                if heavy:
                    x = (x + np.float32(1e4 * (-1) ** k)).astype(np.float32)
                layers.append(x)
            pus.append(layers)
        ns = [int(v) for v in rng.integers(0, 5000, K)]
        ns[-1] += 1
        for a, b in zip(fedavg_reference_structure(pus, ns), fedavg_explicit(pus, ns)):
            assert np.array_equal(_bits(a), _bits(b))


def test_signed_zero_seed():
    """NumPy seeds add.reduce with +0.0: an all -0.0 column sums to +0.0 (both orders)."""
    for shp in [(1,), (3, 2)]:
        pus = [[np.full(shp, -0.0, np.float32)] for _ in range(3)]
        out = fedavg_reference_structure(pus, [0, 0, 4])[0]
        assert not np.signbit(out).any()
        assert np.array_equal(_bits(out), _bits(fedavg_explicit(pus, [0, 0, 4])[0]))


def test_golden_fedpca_is_fedavg_arithmetic(golden):
    """FedPCA's plain average is FedAvg's arithmetic, bit for bit."""
    arrays, meta = golden
    for case in [c for c in meta["cases"] if c["strategy"] == "fedpca"]:
        key, K, L = case["key"], case["K"], case["layers"]
        ns = [int(v) for v in arrays[f"{key}/n_samples"]]
        pus = [[arrays[f"{key}/x{li}"][k] for li in range(L)] for k in range(K)]
        for g, r in zip(fedavg_reference_structure(pus, ns), [arrays[f"{key}/avg{li}"] for li in range(L)]):
            assert np.array_equal(_bits(g), _bits(r))


def test_golden_newton_raphson_bit_exact():
    """The oracle's restatement of NewtonRaphson.compute_averaged_states (newton_raphson.py:
    195-216) reproduces the reference's outputs (golden_newton_raphson.npz, gen_golden_nr.py) bit
    for bit, including the -0.0 case."""
    import json
    from pathlib import Path

    from oracle import newton_raphson_reference_structure

    d = Path(__file__).resolve().parent / "golden"
    arrays = np.load(d / "golden_newton_raphson.npz", allow_pickle=False)
    meta = json.loads((d / "golden_newton_raphson_meta.json").read_text())
    assert len(meta["cases"]) >= 9
    for c in meta["cases"]:
        key, K, L = c["key"], c["K"], c["layers"]
        grads = [[arrays[f"{key}/k{k}/g{li}"] for li in range(L)] for k in range(K)]
        hess = [arrays[f"{key}/k{k}/h"] for k in range(K)]
        ns = [int(v) for v in arrays[f"{key}/n_samples"]]
        got = newton_raphson_reference_structure(grads, hess, ns, c["damping_factor"])
        ref = [arrays[f"{key}/out{li}"] for li in range(c["outputs"])]
        assert len(got) == len(ref)
        for g, r in zip(got, ref):
            assert g.dtype == r.dtype and g.shape == r.shape
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64)), key
