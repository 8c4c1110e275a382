"""Parity of the HIP path (through libfedagg.so's C ABI) with the oracle and the reference's
golden vectors.  Bar: bit-exact (the reference arithmetic is deterministic IEEE fp32/fp64)."""

import ctypes
import pickle
import subprocess
import sys
from pathlib import Path

import numpy as np
import pydantic
import pytest

from oracle import fedavg_reference_structure, numpy_pairwise_sum, scaffold_reference_structure

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


from conftest import PRODUCT_KNOBS, experiment_knobs  # noqa: E402


def _tuning_only(*knob_dicts):
    """Skip unless every knob is one the loaded library has: experiment knobs select variants the
    product library does not instantiate (a FEDAGG_TUNING build does: ``build(tuning=True)``,
    ``FEDAGG_LIB=substrafl_amd/libfedagg_tuning.so``).  Such tests are deselected at collection
    unless that build is requested (conftest.py), so this only guards a mismatched FEDAGG_LIB."""
    from substrafl_amd import _native

    if experiment_knobs(*knob_dicts) and not _native.tuning_build():
        pytest.skip("experiment variant: needs the FEDAGG_TUNING build of libfedagg")


def _product(d):
    """``d`` without the experiment knobs when the product library is loaded."""
    from substrafl_amd import _native

    return dict(d) if _native.tuning_build() else {k: v for k, v in d.items() if k in PRODUCT_KNOBS}


def _bits(a):
    a = np.asarray(a)
    return a.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize])


def _assert_same(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert isinstance(g, np.ndarray)
        assert g.dtype == r.dtype and g.shape == r.shape, (g.dtype, r.dtype, g.shape, r.shape)
        assert np.array_equal(_bits(g), _bits(r))


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from substrafl_amd import _native

    _native.load()
    return torch


# ------------------------------------------------------------------------------------------
# golden vectors (captured from the reference itself)
# ------------------------------------------------------------------------------------------
def test_golden_fedavg(golden, torch_gpu, dummy_algo_class):
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    arrays, meta = golden
    strategy = FedAvg(algo=dummy_algo_class())
    n = 0
    for case in [c for c in meta["cases"] if c["strategy"] == "fedavg"]:
        key, K, L = case["key"], case["K"], case["layers"]
        ns = [int(v) for v in arrays[f"{key}/n_samples"]]
        states = [FedAvgSharedState(n_samples=ns[k], parameters_update=[arrays[f"{key}/x{li}"][k] for li in range(L)])
                  for k in range(K)]
        got = strategy.avg_shared_states(shared_states=states, _skip=True).avg_parameters_update
        _assert_same(got, [arrays[f"{key}/out{li}"] for li in range(L)])
        n += 1
    assert n >= 40


def test_golden_scaffold(golden, torch_gpu, dummy_algo_class):
    from substrafl_amd.schemas import ScaffoldSharedState
    from substrafl_amd.strategies import Scaffold

    arrays, meta = golden
    for case in [c for c in meta["cases"] if c["strategy"] == "scaffold"]:
        key, K, L = case["key"], case["K"], case["layers"]
        lr = int(case["lr"]) if case["lr_is_int"] else float(case["lr"])
        ns = [int(v) for v in arrays[f"{key}/n_samples"]]
        c = [arrays[f"{key}/c{li}"] for li in range(L)]
        states = [
            ScaffoldSharedState(
                parameters_update=[arrays[f"{key}/pu{li}"][k] for li in range(L)],
                control_variate_update=[arrays[f"{key}/cv{li}"][k] for li in range(L)],
                n_samples=ns[k],
                server_control_variate=c,
            )
            for k in range(K)
        ]
        res = Scaffold(algo=dummy_algo_class(), aggregation_lr=lr).avg_shared_states(shared_states=states, _skip=True)
        _assert_same(res.avg_parameters_update, [arrays[f"{key}/avg{li}"] for li in range(L)])
        _assert_same(res.server_control_variate, [arrays[f"{key}/newc{li}"] for li in range(L)])


@pytest.mark.parametrize("n_samples, factor", [([1, 0, 0], 1.0), ([1, 1, 1], 1.0), ([1, 0, 1], 1.5)])
def test_reference_unit_fedavg(torch_gpu, dummy_algo_class, n_samples, factor, golden):
    """tests/strategies/test_fed_avg.py:17-38 (float64 inputs, exact equality)."""
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    states = [
        FedAvgSharedState(parameters_update=[np.ones((5, 10))], n_samples=n_samples[0]),
        FedAvgSharedState(parameters_update=[np.zeros((5, 10))], n_samples=n_samples[1]),
        FedAvgSharedState(parameters_update=[2 * np.ones((5, 10))], n_samples=n_samples[2]),
    ]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(states, _skip=True).avg_parameters_update
    assert (factor * np.ones((5, 10)) == got).all() and got[0].dtype == np.float64


@pytest.mark.parametrize("n_samples, factor", [([1, 0, 0], 1.0), ([1, 1, 1], 1.0), ([1, 0, 1], 1.5)])
def test_reference_unit_fedpca(torch_gpu, dummy_algo_class, n_samples, factor):
    """tests/strategies/test_fed_pca.py:12-33 on the GPU path (float64, exact equality)."""
    from substrafl_amd.schemas import FedPCASharedState
    from substrafl_amd.strategies import FedPCA

    states = [
        FedPCASharedState(parameters_update=[np.ones((5, 10))], n_samples=n_samples[0]),
        FedPCASharedState(parameters_update=[np.zeros((5, 10))], n_samples=n_samples[1]),
        FedPCASharedState(parameters_update=[2 * np.ones((5, 10))], n_samples=n_samples[2]),
    ]
    got = FedPCA(algo=dummy_algo_class()).avg_shared_states(states, _skip=True).avg_parameters_update
    assert (factor * np.ones((5, 10)) == got).all()


@pytest.mark.parametrize("shared, expected", [
    ([(np.array([[0.5, 0, 0], [1, 0, 1.5], [2, 2.5, 3]]), 2), (np.array([[1, 0, 0], [2, 0, 3], [4, 5, 6]]), 1)],
     np.array([[1, 0, 0], [0, 0, 1], [0, 1, 0]])),
    ([(np.array([[1, 1, 1, 1], [-1, 4, 4, -1], [4, -2, 2, 0]]), 1)],
     np.array([[0.5, 0.5, 0.5, 0.5], [-0.5, 0.5, 0.5, -0.5], [0.5, -0.5, 0.5, -0.5]])),
])
def test_reference_unit_fedpca_qr(torch_gpu, dummy_algo_class, shared, expected):
    """tests/strategies/test_fed_pca.py:36-65: each returned row spans the expected direction
    (rtol 1e-5, tests/conftest.py:345-352)."""
    from substrafl_amd.schemas import FedPCASharedState
    from substrafl_amd.strategies import FedPCA

    states = [FedPCASharedState(parameters_update=[x], n_samples=n) for x, n in shared]
    got = FedPCA(algo=dummy_algo_class()).avg_shared_states_with_qr(states, _skip=True).avg_parameters_update[0]
    assert all(np.allclose(np.dot(expected[i], row) * row, expected[i], rtol=1e-5) for i, row in enumerate(got))


def test_reference_unit_int64_layers(torch_gpu, dummy_algo_class, golden):
    """tests/strategies/test_fed_avg.py:41-54: int64 layers promote to float64."""
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    arrays, _ = golden
    states = [
        FedAvgSharedState(parameters_update=[np.asarray([[0, 1], [2, 4]]), np.asarray([[6, 8], [10, 12]])], n_samples=1),
        FedAvgSharedState(parameters_update=[np.asarray([[16, 20], [18, 20]]), np.asarray([[22, 24], [26, 28]])],
                          n_samples=3),
    ]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(states, _skip=True).avg_parameters_update
    _assert_same(got, [arrays["g5/unit_fedavg_int64_0"], arrays["g5/unit_fedavg_int64_1"]])


@pytest.mark.parametrize(
    "aggregation_lr, expected",
    [(0, [np.zeros(5), np.zeros(5)]), (1, [0.75 * np.ones(5), 1.75 * np.ones(5)]), (2, [1.5 * np.ones(5), 3.5 * np.ones(5)])],
)
def test_reference_unit_scaffold_lr(torch_gpu, dummy_algo_class, aggregation_lr, expected):
    """tests/strategies/test_scaffold.py:149-176."""
    from substrafl_amd.schemas import ScaffoldSharedState
    from substrafl_amd.strategies import Scaffold

    states = [
        ScaffoldSharedState(parameters_update=[0 * np.ones(5), np.ones(5)], control_variate_update=[np.ones(5), np.ones(5)],
                            n_samples=1, server_control_variate=[np.ones(5), np.ones(5)]),
        ScaffoldSharedState(parameters_update=[np.ones(5), 2 * np.ones(5)], control_variate_update=[np.ones(5), np.ones(5)],
                            n_samples=3, server_control_variate=[np.ones(5), np.ones(5)]),
    ]
    res = Scaffold(algo=dummy_algo_class(), aggregation_lr=aggregation_lr).avg_shared_states(shared_states=states,
                                                                                           _skip=True)
    for g, e in zip(res.avg_parameters_update, expected):
        assert np.allclose(g, e)
    for g in res.server_control_variate:
        assert np.allclose(g, 2 * np.ones(5))


# ------------------------------------------------------------------------------------------
# randomized parity against the oracle: client-count edges, chunking, dtypes
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("K", [1, 2, 7, 8, 9, 127, 128, 129, 300])
def test_fedavg_random_vs_oracle(torch_gpu, dummy_algo_class, K):
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    rng = np.random.default_rng(K)
    shapes = [(33, 17), (1,), (5,), (1, 1), (2, 1, 3), (1031,)]
    pus = [[(rng.standard_normal(s) * 10.0 ** rng.integers(-3, 3)).astype(np.float32) for s in shapes] for _ in range(K)]
    if K % 2:
        pus = [[(a + np.float32(1e4 * (-1) ** k)).astype(np.float32) for a in p] for k, p in enumerate(pus)]
    ns = [int(v) for v in rng.integers(0, 5000, K)]
    ns[0] += 1
    states = [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, pus)]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(states, _skip=True).avg_parameters_update
    _assert_same(got, fedavg_reference_structure(pus, ns))


@pytest.mark.parametrize("dtype", [np.float64, np.float16, np.int32])
def test_fedavg_other_dtypes(torch_gpu, dummy_algo_class, dtype):
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    rng = np.random.default_rng(3)
    shapes = [(40, 3), (1,), (17,)]
    K = 11
    pus = [[(rng.standard_normal(s) * 20).astype(dtype) for s in shapes] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    states = [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, pus)]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(states, _skip=True).avg_parameters_update
    _assert_same(got, fedavg_reference_structure(pus, ns))


def test_fedavg_mixed_dtypes_in_one_layer(torch_gpu, dummy_algo_class):
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    rng = np.random.default_rng(4)
    K = 5
    pus = [[rng.standard_normal((9, 7)).astype(np.float32 if k % 2 else np.float64),
            rng.standard_normal(4).astype(np.float32)] for k in range(K)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    states = [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, pus)]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(states, _skip=True).avg_parameters_update
    _assert_same(got, fedavg_reference_structure(pus, ns))


def test_fedavg_0d_layer_fails_validation_like_reference(torch_gpu, dummy_algo_class):
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    states = [FedAvgSharedState(parameters_update=[np.ones((), np.float32)], n_samples=1)] * 2
    with pytest.raises(pydantic.ValidationError):
        FedAvg(algo=dummy_algo_class()).avg_shared_states(states, _skip=True)


@pytest.mark.parametrize("K, lr", [(1, 1), (3, 0.7), (64, 2), (65, 0), (130, 1.3)])
def test_scaffold_random_vs_oracle(torch_gpu, dummy_algo_class, K, lr):
    from substrafl_amd.schemas import ScaffoldSharedState
    from substrafl_amd.strategies import Scaffold

    rng = np.random.default_rng(100 + K)
    shapes = [(13, 7), (1,), (1, 1), (130,)]
    mk = lambda: [(rng.standard_normal(s) * 10.0 ** rng.integers(-3, 3)).astype(np.float32) for s in shapes]  # noqa
    pus, cvs, c = [mk() for _ in range(K)], [mk() for _ in range(K)], mk()
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    states = [ScaffoldSharedState(parameters_update=pus[k], control_variate_update=cvs[k], n_samples=ns[k],
                                  server_control_variate=c) for k in range(K)]
    res = Scaffold(algo=dummy_algo_class(), aggregation_lr=lr).avg_shared_states(shared_states=states, _skip=True)
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, lr)
    _assert_same(res.server_control_variate, rc)
    _assert_same(res.avg_parameters_update, ra)


def test_scaffold_fp64_inputs_and_c_check(torch_gpu, dummy_algo_class):
    from substrafl_amd.schemas import ScaffoldSharedState
    from substrafl_amd.strategies import Scaffold

    rng = np.random.default_rng(9)
    K = 4
    shapes = [(6, 2), (1,)]
    pus = [[rng.standard_normal(s) for s in shapes] for _ in range(K)]
    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c = [np.array([[np.nan, 0.0]] * 6), np.array([-0.0])]
    ns = [3, 1, 4, 1]
    states = [ScaffoldSharedState(parameters_update=pus[k], control_variate_update=cvs[k], n_samples=ns[k],
                                  server_control_variate=[a.copy() for a in c]) for k in range(K)]
    states[2].server_control_variate[1] = np.array([0.0])  # +0 == -0 and NaN == NaN for assert_array_equal
    res = Scaffold(algo=dummy_algo_class(), aggregation_lr=1).avg_shared_states(shared_states=states, _skip=True)
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 1)
    _assert_same(res.server_control_variate, rc)
    _assert_same(res.avg_parameters_update, ra)
    states[3].server_control_variate[0] = np.ones((6, 2))
    with pytest.raises(AssertionError):
        Scaffold(algo=dummy_algo_class()).avg_shared_states(shared_states=states, _skip=True)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("c_check", ["host", "device"])
def test_scaffold_shared_c_objects_staged_once(torch_gpu, dtype, c_check):
    """All clients holding the very same c arrays (simulation mode) stage one copy and skip the
    check; equal-valued copies (separately unpickled, the task-process case) are checked on the
    host while ONE copy is staged (default) or, with the knob, staged K times and checked on the
    device -- the same mismatch count either way."""
    from substrafl_amd.engine import AggregationEngine

    rng = np.random.default_rng(21)
    K = 5
    shapes = [(300, 7), (1,), (4096,)]
    mk = lambda: [rng.standard_normal(s).astype(dtype) for s in shapes]  # noqa: E731
    pus, cvs, c = [mk() for _ in range(K)], [mk() for _ in range(K)], mk()
    c[0][3, 3] = np.nan
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.9)
    eng = AggregationEngine(0, c_check=c_check)
    for rows, check in (([c] * K, "identity"), ([list(c) for _ in range(K)], "identity"),
                        ([[a.copy() for a in c] for _ in range(K)], c_check)):
        mism, new_c, avg = eng.scaffold(pus, cvs, rows, ns, 0.9)
        assert mism == 0 and eng.last_timing["c_check"] == check
        _assert_same(new_c, rc)
        _assert_same(avg, ra)
    rows = [list(c) for _ in range(K)]
    rows[K - 1][2] = c[2].copy()
    rows[K - 1][2][-1] += 1
    rows[1] = [a.copy() for a in c]
    rows[1][0][0, 0] = -rows[1][0][0, 0] if rows[1][0][0, 0] != 0 else 1.0
    rows[1][0][3, 3] = -np.nan  # NaN == NaN for assert_array_equal
    mism, _, _ = eng.scaffold(pus, cvs, rows, ns, 0.9)
    assert mism == 2 and eng.last_timing["c_check"] == c_check


def test_scaffold_host_c_check_signed_zero_and_flat_rows(torch_gpu):
    """+0 == -0 and NaN == NaN on the host check too; flat wire-format c rows (one buffer per
    client) are checked as one segment."""
    from substrafl_amd.engine import AggregationEngine
    from substrafl_amd.wire import BucketArray, pack

    rng = np.random.default_rng(3)
    K = 4
    shapes = [(2000,), (1,), (33, 3)]
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    c[0][:10] = 0.0
    c[2][0, 0] = np.nan
    ns = [4, 1, 7, 2]
    rows = []
    for k in range(K):
        ck = [a.copy() for a in c]
        if k % 2:
            ck[0][:10] = -0.0
        rows.append(pack(ck) if k == 2 else ck)
    eng = AggregationEngine(0)
    mism, new_c, avg = eng.scaffold(pus, cvs, rows, ns, 1.1)
    assert mism == 0 and eng.last_timing["c_check"] == "host"
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 1.1)
    _assert_same_nan_aware(new_c, rc)
    _assert_same(avg, ra)
    assert isinstance(rows[2][0], BucketArray)


# ------------------------------------------------------------------------------------------
# device-resident plans through the C ABI (bf16, unaligned rows, full size)
# ------------------------------------------------------------------------------------------
def test_bf16_plan_equals_reference_on_upcast(torch_gpu):
    torch = torch_gpu
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    K, M = 37, 10_007
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn((K, M + 9), generator=g, device="cuda").to(torch.bfloat16)
    ns = list(range(1, K + 1))
    out = torch.empty(M + 9, dtype=torch.float32, device="cuda")
    FedAvgPlan("bf16", x, fedavg_weights(ns, "bf16"), M, out, [5, M - 1]).launch()
    torch.cuda.synchronize()
    up = x.float().cpu().numpy()[:, :M]
    ref = fedavg_reference_structure([[up[k].copy()] for k in range(K)], ns)[0]
    got = out.cpu().numpy()[:M]
    mask = np.ones(M, bool)
    mask[[5, M - 1]] = False
    assert np.array_equal(_bits(got[mask]), _bits(ref[mask]))
    w = fedavg_weights(ns, "f32")
    for p in (5, M - 1):
        prods = (up[:, p] * w).astype(np.float32)
        assert _bits(np.float32(0.0) + numpy_pairwise_sum(prods)) == _bits(got[p])


def test_unaligned_rows_take_scalar_path(torch_gpu):
    torch = torch_gpu
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    K, M = 5, 4099
    base = torch.randn(K * (M + 1) + 1, device="cuda")
    rows = [base.data_ptr() + 4 * (1 + k * (M + 1)) for k in range(K)]  # 4-B aligned only
    out = torch.empty(M, device="cuda")
    ns = [5, 4, 3, 2, 1]
    FedAvgPlan("f32", rows, fedavg_weights(ns, "f32"), M, out).launch()
    torch.cuda.synchronize()
    h = base.cpu().numpy()
    pus = [[h[1 + k * (M + 1): 1 + k * (M + 1) + M].copy()] for k in range(K)]
    assert np.array_equal(_bits(out.cpu().numpy()), _bits(fedavg_reference_structure(pus, ns)[0]))


@pytest.mark.parametrize("K, M, kind", [(8, 25_000_000, "f32"), (64, 4_000_000, "f32"), (200, 1_000_000, "f32"),
                                        (8, 9_000_011, "bf16"), (128, 2_000_000, "bf16")])
def test_full_size_vs_torch_sequential(torch_gpu, K, M, kind):
    """At BASELINE sizes: bit-exact against a torch fp32 eager sequential reference on the device
    (every torch op is one separately rounded IEEE op: same order as the reference)."""
    torch = torch_gpu
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes

    shapes = synthetic_state_dict_shapes(M)
    lay = BucketLayout(range(len(shapes)), shapes, np.float32)
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn((K, lay.ld), generator=g, device="cuda")
    if kind == "bf16":
        x = x.to(torch.bfloat16)
    ns = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    w = fedavg_weights(ns, "f32")
    out = torch.empty(lay.ld, device="cuda")
    FedAvgPlan(kind, x, w, M, out, lay.pairwise_idx).launch()
    x = x.float()
    acc = torch.zeros(M, device="cuda")
    for k in range(K):
        acc = acc + x[k, :M] * torch.tensor(w[k], device="cuda")
    torch.cuda.synchronize()
    mask = torch.ones(M, dtype=torch.bool, device="cuda")
    mask[torch.from_numpy(lay.pairwise_idx.astype(np.int64)).cuda()] = False
    assert torch.equal(out[:M][mask].view(torch.int32), acc[mask].view(torch.int32))
    for p in lay.pairwise_idx.astype(np.int64):
        prods = (x[:, p].cpu().numpy() * w).astype(np.float32)
        assert _bits(np.float32(0.0) + numpy_pairwise_sum(prods)) == _bits(out[p].cpu().numpy())


@pytest.mark.parametrize("K, M, kind", [(64, 125_000_000, "f32"), (128, 350_000_000, "bf16")])
def test_baseline_config_sizes_vs_torch_sequential(torch_gpu, K, M, kind):
    """BASELINE.json configs C3 (64 x 125M fp32, 32.5 GB) and C5 (128 x 350M bf16, 91 GB) on one
    GPU: bit-exact against torch eager ops applied client by client in list order (one rounded
    IEEE op each), built row by row so no fp32 copy of the whole bucket is made."""
    torch = torch_gpu
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes

    shapes = synthetic_state_dict_shapes(M)
    lay = BucketLayout(range(len(shapes)), shapes, np.float32)
    dt = torch.bfloat16 if kind == "bf16" else torch.float32
    x = torch.empty((K, lay.ld), device="cuda", dtype=dt)
    g = torch.Generator(device="cuda").manual_seed(11)
    for k in range(K):
        x[k].copy_(torch.randn(lay.ld, generator=g, device="cuda"))
    ns = [int(v) for v in np.random.default_rng(11).integers(100, 10000, K)]
    w = fedavg_weights(ns, "f32")
    out = torch.empty(lay.ld, device="cuda")
    FedAvgPlan(kind, x, w, M, out, lay.pairwise_idx).launch()
    acc = torch.zeros(M, device="cuda")
    for k in range(K):
        acc = acc + x[k, :M].float() * torch.tensor(w[k], device="cuda")
    torch.cuda.synchronize()
    mask = torch.ones(M, dtype=torch.bool, device="cuda")
    mask[torch.from_numpy(lay.pairwise_idx.astype(np.int64)).cuda()] = False
    same = torch.equal(out[:M][mask].view(torch.int32), acc[mask].view(torch.int32))
    for p in lay.pairwise_idx.astype(np.int64):
        prods = (x[:, p].float().cpu().numpy() * w).astype(np.float32)
        same = same and _bits(np.float32(0.0) + numpy_pairwise_sum(prods)) == _bits(out[p].cpu().numpy())
    del x, acc, mask, out
    torch.cuda.empty_cache()
    assert same


@pytest.mark.parametrize("K, M, kind", [(64, 125_000_000, "f32"), (128, 350_000_000, "bf16")])
def test_baseline_config_sizes_tiled_as_timed(torch_gpu, K, M, kind):
    """The headline kernels exactly as bench.py times them: C3 (64 x 125M fp32) and C5 (128 x 350M
    bf16) on tile-interleaved buckets (TiledFedAvgPlan with the library's tile -- 8192 / 4096
    vectors -- and the fused numel == 1 patch), checked on EVERY element: bit-exact against torch
    eager ops applied client by client in list order, the numel == 1 elements against NumPy's
    pairwise sum (fed_avg.py:217-222)."""
    torch = torch_gpu
    from substrafl_amd.engine import TiledFedAvgPlan, fedavg_weights, tiled_client_view, tiled_elems, tiled_tile
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes

    shapes = synthetic_state_dict_shapes(M)
    lay = BucketLayout(range(len(shapes)), shapes, np.float32)
    tv = tiled_tile(kind, K, M)
    assert tv == (8192 if kind == "f32" else 4096)  # the recommended layout of the headline line
    dt = torch.bfloat16 if kind == "bf16" else torch.float32
    buf = torch.zeros(tiled_elems(kind, K, M, tv), device="cuda", dtype=dt)
    g = torch.Generator(device="cuda").manual_seed(13)
    for k in range(K):
        view = tiled_client_view(buf, kind, K, k, tv)
        row = torch.zeros(view.numel(), device="cuda")
        row[:M].normal_(generator=g)
        view.copy_(row.view(view.shape))
        del row
    ns = [int(v) for v in np.random.default_rng(17).integers(100, 10000, K)]
    w = fedavg_weights(ns, kind)
    out = torch.empty(lay.ld, device="cuda")
    TiledFedAvgPlan(kind, buf, K, w, M, out, lay.pairwise_idx, tv=tv).launch()
    acc = torch.zeros(M, device="cuda")
    pw = lay.pairwise_idx.astype(np.int64)
    prods = np.zeros((pw.size, K), np.float32)
    for k in range(K):
        xk = tiled_client_view(buf, kind, K, k, tv).reshape(-1)[:M].float()
        acc = acc + xk * torch.tensor(w[k], device="cuda")
        prods[:, k] = (xk[torch.from_numpy(pw).cuda()].cpu().numpy() * w[k]).astype(np.float32)
        del xk
    torch.cuda.synchronize()
    mask = torch.ones(M, dtype=torch.bool, device="cuda")
    mask[torch.from_numpy(pw).cuda()] = False
    same = torch.equal(out[:M][mask].view(torch.int32), acc[mask].view(torch.int32))
    for i, p in enumerate(pw):
        same = same and _bits(np.float32(0.0) + numpy_pairwise_sum(prods[i])) == _bits(out[p].cpu().numpy())
    del buf, acc, mask, out
    torch.cuda.empty_cache()
    assert same


@pytest.mark.parametrize("K, M", [(16, 25_000_000), (16, 5_000_011), (3, 2_000_000)])
def test_scaffold_full_size_vs_torch_fp64(torch_gpu, K, M):
    """Scaffold at size: bit-exact against torch fp64 eager ops (w*x, +, c last, lr*) on the device."""
    torch = torch_gpu
    from substrafl_amd.engine import ScaffoldPlan, scaffold_weights

    ld = (M + 63) // 64 * 64
    d = torch.randn((K, ld), device="cuda")
    cv = torch.randn((K, ld), device="cuda")
    c = torch.randn(ld, device="cuda")
    ns = [int(v) for v in np.random.default_rng(3).integers(100, 10000, K)]
    w = scaffold_weights(ns)
    do = torch.empty(ld, dtype=torch.float64, device="cuda")
    co = torch.empty(ld, dtype=torch.float64, device="cuda")
    ScaffoldPlan("f32", d, cv, c, w, M, 0.7, do, co).launch()
    ad = torch.zeros(M, dtype=torch.float64, device="cuda")
    ac = torch.zeros(M, dtype=torch.float64, device="cuda")
    for k in range(K):
        wk = torch.tensor(w[k], dtype=torch.float64, device="cuda")
        ad = ad + wk * d[k, :M].double()
        ac = ac + wk * cv[k, :M].double()
    ac = ac + c[:M].double()
    ad = torch.tensor(0.7, dtype=torch.float64, device="cuda") * ad
    torch.cuda.synchronize()
    assert torch.equal(do[:M].view(torch.int64), ad.view(torch.int64))
    assert torch.equal(co[:M].view(torch.int64), ac.view(torch.int64))


@pytest.mark.parametrize("M", [100_000, 100_003, 4096 * 4 * 256 + 37])
@pytest.mark.parametrize("kind", ["f32", "f64"])
@pytest.mark.parametrize("vec", [1, 0])
def test_equal_count_variants(torch_gpu, M, kind, vec):
    """scaffold.py:193-196 assert_array_equal semantics (+0 == -0, NaN == NaN) on the vectorised
    and the scalar check, aligned and unaligned rows, tails, and a differing reference copy."""
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import equal_count

    dt = torch.float32 if kind == "f32" else torch.float64
    K = 13
    c = torch.randn(M, device="cuda", dtype=dt)
    c[11] = 0.0
    c[5] = float("nan")
    copies = c.repeat(K, 1)
    copies[4, 11] = -0.0  # equal
    copies[3, 17] = 1e9  # 1
    copies[12, M - 1] = float("nan")  # 1 (NaN vs number)
    copies[9, M - 2] = -copies[9, M - 2]  # 1 (tail element)
    copies[0, 100] = 7.0  # reference copy differs: every other copy mismatches there (K - 1)
    copies[6, :5] = 1e30  # 5
    expected = 1 + 1 + 1 + (K - 1) + 5
    _native.tune(eq_vec=vec)
    try:
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        equal_count(kind, copies, M, cnt)
        torch.cuda.synchronize()
    finally:
        _native.tune(eq_vec=1)
    assert int(cnt.item()) == expected


def test_equal_count_kernel(torch_gpu):
    torch = torch_gpu
    from substrafl_amd.engine import equal_count

    K, M = 9, 100_003
    c = torch.randn(M, device="cuda")
    copies = c.repeat(K, 1)
    copies[3, 17] = 1e9
    copies[7, M - 1] = float("nan")
    copies[:, 5] = float("nan")  # NaN == NaN
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    equal_count("f32", copies, M, cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == 2


# ------------------------------------------------------------------------------------------
# subprocess-mode emulation: the aggregate task in its own process (generic_function contract)
# ------------------------------------------------------------------------------------------
def test_generic_function_in_child_process(torch_gpu, tmp_path, dummy_algo_class):
    from substrafl_amd.remote import PickleSerializer
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    rng = np.random.default_rng(21)
    shapes = [(128, 64), (64,), (1,)]
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(3)]
    ns = [100, 250, 7]
    paths = []
    for k in range(3):
        p = tmp_path / f"shared_{k}"
        PickleSerializer.save(FedAvgSharedState(n_samples=ns[k], parameters_update=pus[k]), p)
        paths.append(str(p))
    import cloudpickle

    cloudpickle.register_pickle_by_value(sys.modules[__name__])  # the child cannot import this test module
    FedAvg(algo=_PicklableAlgo()).avg_shared_states(shared_states=paths).remote_struct.save(tmp_path)
    out = tmp_path / "out_shared"
    script = (
        "import sys; sys.path.insert(0, %r)\n"
        "from substrafl_amd.remote import RemoteStruct\n"
        "rs = RemoteStruct.load(__import__('pathlib').Path(%r))\n"
        "rs.get_remote_instance().generic_function({'shared': %r}, {'shared': %r}, {})\n"
    ) % (str(ROOT), str(tmp_path), paths, str(out))
    subprocess.run([sys.executable, "-c", script], check=True, timeout=300)
    with open(out, "rb") as f:  # our own output file
        res = pickle.load(f)
    _assert_same(res.avg_parameters_update, fedavg_reference_structure(pus, ns))


class _PicklableAlgo:
    def __init__(self, *args, **kwargs):
        self.args, self.kwargs = args, kwargs

    strategies = ["Federated Averaging", "Scaffold"]


@pytest.mark.parametrize("fuse", [1, 0])
def test_many_numel1_layers_fused_and_separate(torch_gpu, dummy_algo_class, fuse):
    """P > FEDAGG_FUSED_PAIRWISE numel==1 tensors, and the fused path switched off."""
    from substrafl_amd import _native
    from substrafl_amd.schemas import FedAvgSharedState, ScaffoldSharedState
    from substrafl_amd.strategies import FedAvg, Scaffold

    rng = np.random.default_rng(31)
    shapes = [(1,)] * 9 + [(3, 4)] + [(1, 1)] * 12 + [(5,)]
    K = 12
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    _native.tune(fuse_pairwise=fuse)
    try:
        got = FedAvg(algo=dummy_algo_class()).avg_shared_states(
            [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, pus)], _skip=True)
        _assert_same(got.avg_parameters_update, fedavg_reference_structure(pus, ns))
        res = Scaffold(algo=dummy_algo_class(), aggregation_lr=0.3).avg_shared_states(
            [ScaffoldSharedState(parameters_update=pus[k], control_variate_update=cvs[k], n_samples=ns[k],
                                 server_control_variate=c) for k in range(K)], _skip=True)
        rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.3)
        _assert_same(res.server_control_variate, rc)
        _assert_same(res.avg_parameters_update, ra)
    finally:
        _native.tune(fuse_pairwise=1)


@pytest.mark.parametrize("knobs", [dict(vpt=2), dict(nt_load=0), dict(nt_store=1), dict(grid_cap=7),
                                   dict(unroll=4), dict(unroll=16), dict(pipe=1), dict(vpt=2, tile=1),
                                   dict(vpt=4, tile=1, grid_cap=5), dict(vpt=8, unroll=2, tile=1),
                                   dict(vpt=8, unroll=4, tile=1, grid_cap=3), dict(vpt=1, tile=0),
                                   dict(vpt=16, unroll=2, tile=1), dict(vpt=16, unroll=1, tile=1, grid_cap=3),
                                   dict(xcd=1), dict(vpt=16, unroll=2, tile=1, xcd=1),
                                   dict(vpt=4, unroll=4, tile=1, pipe=1), dict(vpt=8, tile=1, pipe=1, grid_cap=3),
                                   dict(tpb=3), dict(tpb=7, grid_cap=5), dict(vpt=16, unroll=2, tile=1, tpb=2)])
def test_launch_variants_bit_identical(torch_gpu, knobs):
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    K, M = 19, 1_000_003
    x = torch.randn((K, M + 5), device="cuda")
    ns = list(range(3, 3 + K))
    outs = []
    default = dict(vpt=0, nt_load=1, nt_store=1, grid_cap=0, unroll=8, pipe=0, tile=1, xcd=0, tpb=1, fa_occ=0, buf=0,
                   fa_blk=0)
    _tuning_only(knobs)
    default = _product(default)
    for kn in (default, knobs):
        _native.tune(**kn)
        out = torch.empty(M + 5, device="cuda")
        FedAvgPlan("f32", x, fedavg_weights(ns, "f32"), M, out, [0, 17, M - 1]).launch()
        torch.cuda.synchronize()
        outs.append(out[:M].clone())
    _native.tune(**default)
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))


@pytest.mark.parametrize("kind", ["f32", "bf16"])
@pytest.mark.parametrize("knobs", [dict(vpt=8, unroll=4, fa_occ=3), dict(vpt=8, unroll=4, fa_occ=4, grid_cap=3),
                                   dict(vpt=16, unroll=2, fa_occ=2), dict(vpt=16, unroll=1, fa_occ=3),
                                   dict(vpt=0, fa_occ=2), dict(vpt=0, buf=1), dict(vpt=8, unroll=4, buf=1),
                                   dict(vpt=8, unroll=4, fa_occ=3, buf=1, grid_cap=5), dict(vpt=16, unroll=2, buf=1),
                                   dict(vpt=16, unroll=2, fa_occ=2, buf=1), dict(vpt=16, unroll=1, buf=1),
                                   dict(vpt=16, unroll=1, fa_occ=2, buf=1, grid_cap=3),
                                   dict(vpt=16, unroll=2, fa_blk=512), dict(vpt=8, unroll=2, fa_blk=512),
                                   dict(vpt=0, fa_blk=256), dict(vpt=0, fa_blk=512), dict(vpt=8, unroll=2, fa_blk=1024),
                                   dict(vpt=4, unroll=4, fa_blk=1024, grid_cap=3),
                                   dict(vpt=0, st_sc1=1), dict(vpt=0, st_sc1=0), dict(vpt=8, unroll=4, st_sc1=1, grid_cap=3),
                                   dict(vpt=16, unroll=2, fa_occ=2, st_sc1=1), dict(vpt=16, unroll=2, buf=1, st_sc1=1),
                                   dict(vpt=16, unroll=2, fa_blk=512, st_sc1=1), dict(vpt=4, unroll=4, st_sc1=1),
                                   dict(vpt=8, unroll=4, fa_blk=512, grid_cap=3), dict(vpt=4, unroll=4, fa_blk=512)])
def test_occupancy_capped_variants_bit_identical(torch_gpu, kind, knobs):
    """Register-capped (amdgpu_waves_per_eu) builds of the 8/16-KiB shapes: same bits as the
    default launch, for fp32 and bf16 inputs, with numel==1 patches and a ragged tail."""
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    K, M = 13, 2_000_011
    dt = torch.float32 if kind == "f32" else torch.bfloat16
    x = torch.randn((K, M + 5), device="cuda").to(dt)
    ns = list(range(7, 7 + K))
    default = dict(vpt=0, nt_load=1, nt_store=1, grid_cap=0, unroll=8, pipe=0, tile=1, xcd=0, tpb=1, fa_occ=0, buf=0,
                   fa_blk=0, st_sc1=-1)
    _tuning_only(knobs)
    default = _product(default)
    outs = []
    for kn in (default, dict(default, **knobs)):
        _native.tune(**kn)
        out = torch.empty(M + 5, device="cuda")
        FedAvgPlan(kind, x, fedavg_weights(ns, kind), M, out, [0, 9, M - 1]).launch()
        torch.cuda.synchronize()
        outs.append(out[:M].clone())
    _native.tune(**default)
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))


@pytest.mark.parametrize("knobs", [dict(vpt=0, buf=1), dict(vpt=4, unroll=4, buf=1), dict(vpt=8, unroll=4, buf=1),
                                   dict(vpt=16, unroll=2, buf=1, grid_cap=3), dict(vpt=16, unroll=1, buf=1)])
def test_fp16_buffer_load_variants_bit_identical(torch_gpu, knobs):
    """fp16 FedAvg (fp16 products and sums, N4) over buffer-descriptor loads: same bits as the
    default global-load launch, numel==1 patches and a ragged tail included."""
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    K, M = 11, 1_500_013
    x = torch.randn((K, M + 5), device="cuda").to(torch.float16)
    ns = list(range(20, 20 + K))
    default = dict(vpt=0, nt_load=1, nt_store=1, grid_cap=0, unroll=8, pipe=0, tile=1, xcd=0, tpb=1, fa_occ=0, buf=0)
    _tuning_only(knobs)
    default = _product(default)
    outs = []
    for kn in (default, dict(default, **knobs)):
        _native.tune(**kn)
        out = torch.empty(M + 5, device="cuda", dtype=torch.float16)
        FedAvgPlan("f16", x, fedavg_weights(ns, "f16"), M, out, [4, M - 1]).launch()
        torch.cuda.synchronize()
        outs.append(out[:M].clone())
    _native.tune(**default)
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))


@pytest.mark.parametrize("kind", ["f16", "f64"])
@pytest.mark.parametrize("knobs", [dict(st_sc1=1), dict(st_sc1=0), dict(st_sc1=1, vpt=8, unroll=4),
                                   dict(st_sc1=1, vpt=16, unroll=2), dict(st_sc1=1, grid_cap=5)])
def test_write_through_store_variants_bit_identical(torch_gpu, kind, knobs):
    """Device-scope write-through output stores (fedagg_tune "st_sc1", buffer stores based at the
    first active lane) for fp16 and fp64 (pipelined) tiles: same bits as the default stores,
    ragged tail and numel==1 patches included."""
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    K, M = 9, 1_000_007
    dt = torch.float16 if kind == "f16" else torch.float64
    x = torch.randn((K, M + 7), device="cuda").to(dt)
    ns = list(range(11, 11 + K))
    default = dict(vpt=0, nt_load=1, nt_store=1, grid_cap=0, unroll=8, pipe=0, tile=1, xcd=0, tpb=1, fa_occ=0, buf=0,
                   fa_blk=0, st_sc1=-1)
    _tuning_only(knobs)
    default = _product(default)
    outs = []
    for kn in (default, dict(default, **knobs)):
        _native.tune(**kn)
        out = torch.empty(M + 7, device="cuda", dtype=dt)
        FedAvgPlan(kind, x, fedavg_weights(ns, kind), M, out, [3, M - 2]).launch()
        torch.cuda.synchronize()
        outs.append(out[:M].clone())
    _native.tune(**default)
    iv = torch.int16 if kind == "f16" else torch.int64
    assert torch.equal(outs[0].view(iv), outs[1].view(iv))


def test_auto_shape_many_clients_bit_identical(torch_gpu):
    """K >= 32 over a large bucket picks the 16-KiB-per-stream shape (shape_for); it must agree
    bit for bit with the 8-KiB shape and with the oracle order on sampled elements."""
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    K, M = 33, 16 * 256 * 2048 * 4 + 77  # just past the threshold, ragged tail
    x = torch.randn((K, M + 3), device="cuda")
    ns = list(range(100, 100 + K))
    w = fedavg_weights(ns, "f32")
    outs = []
    shapes = (dict(vpt=0), dict(vpt=8, unroll=4)) if _native.tuning_build() else ({},)  # product: the oracle sample
    for kn in shapes:
        _native.tune(**kn)
        out = torch.empty(M + 3, device="cuda")
        FedAvgPlan("f32", x, w, M, out, [5, M - 1]).launch()
        torch.cuda.synchronize()
        outs.append(out[:M].clone())
    if len(outs) > 1:
        _native.tune(vpt=0, unroll=8)
        assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    idx = np.array([0, 1, 4095, 16 * 256 * 4 * 7 + 3, M // 2, M - 80, M - 2])
    xs = x[:, torch.from_numpy(idx).cuda()].cpu().numpy()
    acc = np.zeros(idx.size, np.float32)
    for k in range(K):
        acc = (acc + (xs[k] * w[k]).astype(np.float32)).astype(np.float32)
    assert np.array_equal(acc.view(np.uint32), outs[0][torch.from_numpy(idx).cuda()].cpu().numpy().view(np.uint32))
    del x


def test_auto_shape_many_clients_bf16_bit_identical(torch_gpu):
    """bf16 from 32 clients over a large bucket: the auto shape (16-KiB tiles, client pairs,
    buffer-descriptor loads) against the 8-KiB global-load shape and the oracle order (exact
    upcast, fp32 products and client-order sums, N8)."""
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    K, M = 34, 16 * 256 * 2048 * 8 + 45  # bf16: 8 elements per 16-B vector; just past the threshold
    x = torch.randn((K, M + 3), device="cuda").to(torch.bfloat16)
    ns = list(range(50, 50 + K))
    w = fedavg_weights(ns, "bf16")
    outs = []
    shapes = (dict(vpt=0, buf=0), dict(vpt=8, unroll=4, buf=0)) if _native.tuning_build() else ({},)
    for kn in shapes:
        _native.tune(**kn)
        out = torch.empty(M + 3, device="cuda")
        FedAvgPlan("bf16", x, w, M, out, [2, M - 1]).launch()
        torch.cuda.synchronize()
        outs.append(out[:M].clone())
    if len(outs) > 1:
        _native.tune(vpt=0, unroll=8)
        assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    idx = np.array([0, 1, 8191, 16 * 256 * 8 * 5 + 7, M // 3, M - 40, M - 2])
    xs = x[:, torch.from_numpy(idx).cuda()].float().cpu().numpy()
    acc = np.zeros(idx.size, np.float32)
    for k in range(K):
        acc = (acc + (xs[k] * np.float32(w[k])).astype(np.float32)).astype(np.float32)
    assert np.array_equal(acc.view(np.uint32), outs[0][torch.from_numpy(idx).cuda()].cpu().numpy().view(np.uint32))
    del x


@pytest.mark.parametrize("knobs", [dict(sc_vpt=1), dict(sc_vpt=2, sc_unroll=2), dict(nt_store=0), dict(nt_load=0),
                                   dict(grid_cap=3), dict(sc_vpt=4, sc_unroll=2), dict(sc_vpt=2, sc_unroll=4),
                                   dict(sc_vpt=8), dict(sc_vpt=8, grid_cap=2), dict(sc_split=1),
                                   dict(sc_split=1, sc_vpt=4, sc_unroll=8), dict(sc_split=1, sc_vpt=8, sc_unroll=2),
                                   dict(sc_split=1, sc_vpt=8, grid_cap=2), dict(sc_vpt=8, sc_unroll=2),
                                   dict(xcd=1), dict(sc_vpt=8, sc_unroll=2, xcd=1, grid_cap=5),
                                   dict(sc_pipe=1), dict(sc_pipe=1, sc_vpt=2, sc_unroll=4, grid_cap=3),
                                   dict(tpb=3), dict(tpb=5, grid_cap=2, sc_vpt=8, sc_unroll=2),
                                   dict(sc_vpt=2, sc_unroll=8), dict(sc_vpt=1, sc_unroll=8, grid_cap=4),
                                   dict(sc_bsplit=1), dict(sc_bsplit=1, sc_vpt=8, sc_unroll=4),
                                   dict(sc_bsplit=1, sc_vpt=8, sc_unroll=2, grid_cap=3),
                                   dict(sc_bsplit=1, sc_vpt=4, sc_unroll=8), dict(sc_bsplit=1, sc_vpt=2, sc_unroll=8),
                                   dict(sc_bsplit=1, nt_store=0), dict(sc_buf=1), dict(sc_buf=1, sc_vpt=4, sc_unroll=2),
                                   dict(sc_buf=1, sc_vpt=8, sc_unroll=2, grid_cap=3), dict(sc_buf=1, sc_vpt=8, sc_unroll=4),
                                   dict(sc_buf=1, sc_vpt=2), dict(sc_buf=1, nt_store=0),
                                   dict(sc_vpt=4, sc_unroll=4, sc_cpf=1), dict(sc_vpt=4, sc_unroll=4, sc_cpf=1, K=12),
                                   dict(sc_vpt=4, sc_unroll=4, sc_occ=4), dict(sc_vpt=4, sc_unroll=4, sc_blk=512),
                                   dict(sc_vpt=4, sc_unroll=4, sc_cpf=1, sc_occ=4, K=16),
                                   dict(sc_vpt=4, sc_unroll=4, sc_cpf=1, sc_blk=512, grid_cap=3, K=8),
                                   dict(sc_vpt=4, sc_unroll=4, sc_occ=2, sc_blk=512, K=16),
                                   dict(sc_vpt=4, sc_unroll=4, sc_sc1=1), dict(sc_sc1=1, K=16),
                                   dict(sc_buf=1, sc_vpt=4, sc_unroll=4, sc_sc1=1, K=32),
                                   dict(sc_sc1=1, grid_cap=3, K=8),
                                   dict(sc_2l=1), dict(sc_2l=1, sc_vpt=8, sc_unroll=4), dict(sc_2l=1, K=70),
                                   dict(sc_2l=1, sc_vpt=16, sc_unroll=2, K=16), dict(sc_2l=1, sc_vpt=8, sc_unroll=2, sc_sc1=1),
                                   dict(sc_2l=1, nt_store=0, K=5), dict(sc_2l=1, grid_cap=3, K=33),
                                   dict(sc_2l=1, sc_vpt=4, sc_unroll=8), dict(sc_2l=1, sc_vpt=16, sc_unroll=1, K=12),
                                   dict(sc_2l=2, sc_vpt=8, sc_unroll=4), dict(sc_2l=2, K=70, grid_cap=5),
                                   dict(sc_2l=1, sc_pipe=1, sc_vpt=8, sc_unroll=2), dict(sc_2l=1, sc_pipe=1, K=70),
                                   dict(sc_2l=1, sc_pipe=1, sc_vpt=4, sc_unroll=2, K=7)])
def test_scaffold_launch_variants_bit_identical(torch_gpu, knobs):
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import ScaffoldPlan, scaffold_weights

    knobs = dict(knobs)
    K, M = knobs.pop("K", 11), 300_007
    d = torch.randn((K, M + 1), device="cuda")
    cv = torch.randn((K, M + 1), device="cuda")
    c = torch.randn(M + 1, device="cuda")
    w = scaffold_weights(list(range(5, 5 + K)))
    default = dict(sc_vpt=0, sc_unroll=4, sc_split=0, sc_bsplit=0, sc_buf=0, sc_pipe=0, nt_store=1, nt_load=1, grid_cap=0,
                   xcd=0, tpb=1, sc_cpf=0, sc_occ=0, sc_blk=256, sc_sc1=0, sc_2l=-1)
    _tuning_only(knobs)
    default = _product(default)
    outs = []
    for kn in (default, knobs):
        _native.tune(**kn)
        do = torch.empty(M + 1, dtype=torch.float64, device="cuda")
        co = torch.empty(M + 1, dtype=torch.float64, device="cuda")
        ScaffoldPlan("f32", [d[k].data_ptr() for k in range(K)], [cv[k].data_ptr() for k in range(K)], c, w, M, 0.9,
                     do, co, [3, M - 1]).launch()
        torch.cuda.synchronize()
        outs.append((do[:M].clone(), co[:M].clone()))
    _native.tune(**default)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a.view(torch.int64), b.view(torch.int64))
    # and against the oracle on a sample of elements (fp64 sequential order)
    idx = np.array([0, 1, 2, 3, 4, 1000, M // 2, M - 2, M - 1])
    hd, hc, hcc = d.cpu().numpy(), cv.cpu().numpy(), c.cpu().numpy()
    for i in idx:
        pu = [[hd[k, i:i + 1].copy()] for k in range(K)]
        cu = [[hc[k, i:i + 1].copy()] for k in range(K)]
        if i in (3, M - 1):
            rc, ra = scaffold_reference_structure(pu, cu, [hcc[i:i + 1].copy()], list(range(5, 5 + K)), 0.9)
        else:  # numel >= 2 order: use a 2-element layer holding the element twice
            pu2 = [[np.repeat(p[0], 2)] for p in pu]
            cu2 = [[np.repeat(p[0], 2)] for p in cu]
            rc, ra = scaffold_reference_structure(pu2, cu2, [np.repeat(hcc[i:i + 1], 2)], list(range(5, 5 + K)), 0.9)
        assert _bits(ra[0].reshape(-1)[0]) == _bits(outs[0][0][i].cpu().numpy())
        assert _bits(rc[0].reshape(-1)[0]) == _bits(outs[0][1][i].cpu().numpy())


@pytest.mark.parametrize("K", [32, 40, 70])
def test_scaffold_auto_shape_many_clients_bit_identical(torch_gpu, K):
    """From 32 clients the Scaffold auto shape is 8 x 4 over buffer descriptors (two launch chunks
    at 70); it must agree bit for bit with the 4 x 4 global-load shape."""
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import ScaffoldPlan, scaffold_weights

    M = 1_000_003
    d = torch.randn((K, M + 1), device="cuda")
    cv = torch.randn((K, M + 1), device="cuda")
    c = torch.randn(M + 1, device="cuda")
    w = scaffold_weights(list(range(9, 9 + K)))
    outs = []
    pair = (dict(sc_vpt=0), dict(sc_vpt=4, sc_unroll=4, sc_buf=0)) if _native.tuning_build() else \
        (dict(sc_2l=-1), dict(sc_2l=0))  # product: the one-bucket pair against the fused 8 x 4 walk
    for kn in pair:
        _native.tune(**kn)
        do = torch.empty(M + 1, dtype=torch.float64, device="cuda")
        co = torch.empty(M + 1, dtype=torch.float64, device="cuda")
        ScaffoldPlan("f32", [d[k].data_ptr() for k in range(K)], [cv[k].data_ptr() for k in range(K)], c, w, M, 0.7,
                     do, co, [1, M - 1]).launch()
        torch.cuda.synchronize()
        outs.append((do[:M].clone(), co[:M].clone()))
    _native.tune(**_product(dict(sc_vpt=0, sc_unroll=4, sc_buf=0, sc_2l=-1)))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a.view(torch.int64), b.view(torch.int64))


@pytest.mark.parametrize("K", [9, 67])
@pytest.mark.parametrize("knobs", [dict(sc_2l=1), dict(sc_2l=1, sc_vpt=8, sc_unroll=2, sc_sc1=1), dict(sc_2l=2),
                                   dict(sc_2l=-1), dict(sc_2l=1, sc_pipe=1, sc_vpt=4, sc_unroll=4)])
def test_scaffold_one_bucket_launches_fp64_bit_identical(torch_gpu, K, knobs):
    """fp64 inputs through the one-bucket launch pair (sc_2l): same bits as the fused walk, with a
    ragged tail, numel==1 elements and (K = 67) two client chunks."""
    torch = torch_gpu
    from substrafl_amd import _native
    from substrafl_amd.engine import ScaffoldPlan, scaffold_weights

    M = 200_003
    d = torch.randn((K, M + 1), device="cuda", dtype=torch.float64)
    cv = torch.randn((K, M + 1), device="cuda", dtype=torch.float64)
    c = torch.randn(M + 1, device="cuda", dtype=torch.float64)
    w = scaffold_weights(list(range(4, 4 + K)))
    base = dict(sc_2l=0, sc_vpt=0, sc_unroll=4, sc_sc1=0, sc_pipe=0)
    _tuning_only(knobs)
    base = _product(base)
    outs = []
    for kn in (base, dict(base, **knobs)):
        _native.tune(**kn)
        do = torch.empty(M + 1, dtype=torch.float64, device="cuda")
        co = torch.empty(M + 1, dtype=torch.float64, device="cuda")
        ScaffoldPlan("f64", [d[k].data_ptr() for k in range(K)], [cv[k].data_ptr() for k in range(K)], c, w, M, 1.3,
                     do, co, [2, M - 1]).launch()
        torch.cuda.synchronize()
        outs.append((do[:M].clone(), co[:M].clone()))
    _native.tune(**dict(base, sc_2l=-1))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a.view(torch.int64), b.view(torch.int64))


def test_golden_fedpca(golden, torch_gpu, dummy_algo_class):
    """FedPCA average (bit-exact, same kernel as FedAvg) and the QR variant (fed_pca.py:210-299)."""
    from substrafl_amd.schemas import FedPCASharedState
    from substrafl_amd.strategies import FedPCA

    arrays, meta = golden
    cases = [c for c in meta["cases"] if c["strategy"] == "fedpca"]
    assert cases
    s = FedPCA(algo=dummy_algo_class())
    for case in cases:
        key, K, L = case["key"], case["K"], case["layers"]
        ns = [int(v) for v in arrays[f"{key}/n_samples"]]
        states = [FedPCASharedState(n_samples=ns[k], parameters_update=[arrays[f"{key}/x{li}"][k] for li in range(L)])
                  for k in range(K)]
        _assert_same(s.avg_shared_states(states, _skip=True).avg_parameters_update,
                     [arrays[f"{key}/avg{li}"] for li in range(L)])
        _assert_same(s.avg_shared_states_with_qr(states, _skip=True).avg_parameters_update,
                     [arrays[f"{key}/qr{li}"] for li in range(L)])


@pytest.mark.parametrize("all_flat", [True, False])
def test_flat_wire_format_inputs(torch_gpu, dummy_algo_class, all_flat):
    """Shared states in the flat wire format (substrafl_amd.wire), through the reference's pickle
    (protocol 4), staged one segment per client; bit-exact, and the result pickles as one buffer."""
    from substrafl_amd import wire
    from substrafl_amd.schemas import FedAvgSharedState, ScaffoldSharedState
    from substrafl_amd.strategies import FedAvg, Scaffold

    rng = np.random.default_rng(5)
    shapes = [(257, 33), (1,), (33,), (1, 1), (4099,)]
    K = 9
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    rows = [wire.pack(p) if (all_flat or k % 2) else p for k, p in enumerate(pus)]
    states = [pickle.loads(pickle.dumps(FedAvgSharedState(n_samples=n, parameters_update=r), protocol=4))
              for n, r in zip(ns, rows)]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(states, _skip=True)
    _assert_same(got.avg_parameters_update, fedavg_reference_structure(pus, ns))
    assert wire.flat_of(got.avg_parameters_update) is not None
    back = pickle.loads(pickle.dumps(got))
    _assert_same(back.avg_parameters_update, got.avg_parameters_update)

    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    sstates = [ScaffoldSharedState(parameters_update=wire.pack(pus[k]), control_variate_update=wire.pack(cvs[k]),
                                   n_samples=ns[k], server_control_variate=wire.pack(c)) for k in range(K)]
    res = Scaffold(algo=dummy_algo_class(), aggregation_lr=0.3).avg_shared_states(sstates, _skip=True)
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.3)
    _assert_same(res.server_control_variate, rc)
    _assert_same(res.avg_parameters_update, ra)


def test_ingest_overlapped_staging(torch_gpu, dummy_algo_class, tmp_path):
    """engine.ingest (threaded unpickling + per-client H2D as each file lands) feeds the next
    aggregation; results stay bit-exact, and arrays other than the ingested ones are re-staged."""
    from substrafl_amd.engine import engine_for
    from substrafl_amd.remote import PickleSerializer
    from substrafl_amd.schemas import FedAvgSharedState, ScaffoldSharedState
    from substrafl_amd.strategies import FedAvg, Scaffold

    rng = np.random.default_rng(21)
    shapes = [(300, 17), (1,), (17,), (4097,)]
    K = 7
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    paths = []
    for k in range(K):
        paths.append(tmp_path / f"f{k}")
        PickleSerializer.save(FedAvgSharedState(n_samples=ns[k], parameters_update=pus[k]), paths[-1])
    strategy = FedAvg(algo=dummy_algo_class())
    eng = engine_for(None)
    states = strategy.ingest_shared_states("avg_shared_states", paths, PickleSerializer.load)
    assert eng.last_ingest["prestaged_clients"] == K
    got = strategy.avg_shared_states(states, _skip=True).avg_parameters_update
    assert eng.last_timing.get("prestaged") is True
    _assert_same(got, fedavg_reference_structure(pus, ns))
    # ingest, then aggregate DIFFERENT arrays of the same shapes: must not reuse the staged rows
    states = strategy.ingest_shared_states("avg_shared_states", paths, PickleSerializer.load)
    other = [FedAvgSharedState(n_samples=s.n_samples, parameters_update=[a * np.float32(2) for a in s.parameters_update])
             for s in states]
    got = strategy.avg_shared_states(other, _skip=True).avg_parameters_update
    assert not eng.last_timing.get("prestaged")
    _assert_same(got, fedavg_reference_structure([o.parameters_update for o in other], ns))

    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    spaths = []
    for k in range(K):
        spaths.append(tmp_path / f"s{k}")
        PickleSerializer.save(ScaffoldSharedState(parameters_update=pus[k], control_variate_update=cvs[k],
                                                  n_samples=ns[k], server_control_variate=c), spaths[-1])
    sc = Scaffold(algo=dummy_algo_class(), aggregation_lr=0.4)
    sstates = sc.ingest_shared_states("avg_shared_states", spaths, PickleSerializer.load)
    assert eng.last_ingest["prestaged_clients"] == K
    res = sc.avg_shared_states(sstates, _skip=True)
    assert eng.last_timing.get("prestaged") is True
    # every file carries its own copy of c: one copy staged, the others checked while loading
    assert eng.last_timing["c_check"] == "host-ingest"
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.4)
    _assert_same(res.server_control_variate, rc)
    _assert_same(res.avg_parameters_update, ra)
    # a client whose c differs in one element fails the check
    c_bad = [a.copy() for a in c]
    c_bad[3][7] += 1.0
    PickleSerializer.save(ScaffoldSharedState(parameters_update=pus[2], control_variate_update=cvs[2], n_samples=ns[2],
                                              server_control_variate=c_bad), spaths[2])
    sstates = sc.ingest_shared_states("avg_shared_states", spaths, PickleSerializer.load)
    with pytest.raises(AssertionError):
        sc.avg_shared_states(sstates, _skip=True)
    assert eng.last_timing["c_check"] == "host-ingest"


def test_fedavg_layout_edge_cases(torch_gpu, dummy_algo_class):
    """Fortran-ordered, strided (non-contiguous) and empty layers: same values, shapes and dtypes
    as the reference's np.sum over the K products."""
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    rng = np.random.default_rng(99)
    K = 6
    pus = []
    for _ in range(K):
        base = rng.standard_normal((40, 30)).astype(np.float32)
        pus.append([
            np.asfortranarray(rng.standard_normal((17, 9)).astype(np.float32)),  # F order
            base[::2, ::3],  # strided view
            np.zeros((0,), np.float32),  # empty
            rng.standard_normal((3, 0, 2)).astype(np.float32),  # empty, 3-d
            rng.standard_normal((1,)).astype(np.float32),
        ])
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    states = [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, pus)]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(states, _skip=True).avg_parameters_update
    _assert_same(got, fedavg_reference_structure(pus, ns))


def test_fedavg_only_empty_layers(torch_gpu, dummy_algo_class):
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    pus = [[np.zeros((0, 4), np.float32)] for _ in range(3)]
    states = [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip([1, 2, 3], pus)]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(states, _skip=True).avg_parameters_update
    _assert_same(got, fedavg_reference_structure(pus, [1, 2, 3]))


def test_ingest_mixed_dtypes_round2_scaffold_and_int_layers(torch_gpu, dummy_algo_class, tmp_path):
    """Scaffold from round 2 on ships fp32 deltas with fp64 control variates and fp64 c (the
    aggregator's fp64 output comes back; tests/golden plumbing call1+): the rows are staged raw
    and cast once on the device, prestaged by ingest, bit-exact.  Same for int64 FedAvg layers."""
    from substrafl_amd.engine import engine_for
    from substrafl_amd.remote import PickleSerializer
    from substrafl_amd.schemas import FedAvgSharedState, ScaffoldSharedState
    from substrafl_amd.strategies import FedAvg, Scaffold

    rng = np.random.default_rng(8)
    shapes = [(64, 9), (1,), (9,), (1, 1), (2049,)]
    K = 5
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    cvs = [[rng.standard_normal(s) for s in shapes] for _ in range(K)]  # fp64
    c = [rng.standard_normal(s) for s in shapes]  # fp64
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    paths = []
    for k in range(K):
        paths.append(tmp_path / f"s{k}")
        PickleSerializer.save(ScaffoldSharedState(parameters_update=pus[k], control_variate_update=cvs[k],
                                                  n_samples=ns[k], server_control_variate=c), paths[-1])
    eng = engine_for(None)
    sc = Scaffold(algo=dummy_algo_class(), aggregation_lr=1.3)
    states = sc.ingest_shared_states("avg_shared_states", paths, PickleSerializer.load)
    assert eng.last_ingest["prestaged_clients"] == K
    res = sc.avg_shared_states(states, _skip=True)
    assert eng.last_timing.get("prestaged") is True
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 1.3)
    _assert_same(res.server_control_variate, rc)
    _assert_same(res.avg_parameters_update, ra)
    # the same inputs without ingest (staged by the aggregation call) agree bit for bit
    res2 = sc.avg_shared_states(states, _skip=True)
    _assert_same(res2.avg_parameters_update, ra)

    ints = [[rng.integers(-1000, 1000, s) for s in shapes] for _ in range(K)]
    ipaths = []
    for k in range(K):
        ipaths.append(tmp_path / f"i{k}")
        PickleSerializer.save(FedAvgSharedState(n_samples=ns[k], parameters_update=ints[k]), ipaths[-1])
    fa = FedAvg(algo=dummy_algo_class())
    istates = fa.ingest_shared_states("avg_shared_states", ipaths, PickleSerializer.load)
    assert eng.last_ingest["prestaged_clients"] == K
    got = fa.avg_shared_states(istates, _skip=True).avg_parameters_update
    assert eng.last_timing.get("prestaged") is True
    _assert_same(got, fedavg_reference_structure(ints, ns))


def test_sharding_over_rccl_world1(torch_gpu):
    """The RCCL code paths of substrafl_amd.sharding (all_gather of parameter-range slices, reduce
    of client-block partials) on a one-rank nccl group: with one rank both are exact."""
    import socket

    import torch.distributed as dist

    from substrafl_amd.sharding import client_sharded_fedavg, param_range_fedavg

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(4)
        shapes = [(37, 29), (1,), (700,), (1, 1)]
        pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(6)]
        ns = [int(v) for v in rng.integers(1, 5000, 6)]
        ref = fedavg_reference_structure(pus, ns)
        _assert_same(param_range_fedavg(pus, ns), ref)
        _assert_same(client_sharded_fedavg(pus, ns, combine="rccl"), ref)
        _assert_same(client_sharded_fedavg(pus, ns, combine="ordered"), ref)
    finally:
        dist.destroy_process_group()


# ------------------------------------------------------------------------------------------
# non-finite and extreme values (a diverged client: NaN / Inf updates, overflow, denormals)
# ------------------------------------------------------------------------------------------
# Contract: every NaN of the reference is a NaN here and every other value (Inf, max, denormal,
# signed zero) is bit-exact.  NaN payload and sign bits are NOT part of the reference's
# behaviour: NumPy's x86 loops keep the first operand's NaN in the scalar path and the second
# operand's in the SIMD path (fp32: arrays of <= 16 vs >= 17 elements on the box this was
# measured on), and invalid operations give the negative "indefinite" NaN; the GPU picks its own.
def _assert_same_nan_aware(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert isinstance(g, np.ndarray)
        assert g.dtype == r.dtype and g.shape == r.shape, (g.dtype, r.dtype, g.shape, r.shape)
        rn = np.isnan(r)
        assert np.array_equal(np.isnan(g), rn)
        assert np.array_equal(_bits(g)[~rn], _bits(r)[~rn])


def _nonfinite_updates(dtype, K, rng):
    info = np.finfo(dtype)
    bits = {np.float16: np.uint16, np.float32: np.uint32, np.float64: np.uint64}[dtype]
    specials = [np.nan, -np.nan, np.inf, -np.inf, info.max, -info.max, info.tiny, info.tiny / 4, -0.0, 0.0,
                info.smallest_subnormal]
    # NaNs with payloads: quiet with a payload, and signalling (NumPy quiets them in arithmetic)
    qpay = np.array([np.nan], dtype).view(bits) | bits(5)
    spay = (np.array([np.inf], dtype).view(bits) | bits(3))
    specials += [qpay.view(dtype)[0], spay.view(dtype)[0], (qpay | np.array([np.inf], dtype).view(bits) * 0 | (bits(1) << bits(8 * np.dtype(dtype).itemsize - 1))).view(dtype)[0]]
    specials = np.array(specials, dtype)
    shapes = [(257,), (1,), (16, 9), (1, 1)]
    ups = []
    for k in range(K):
        row = []
        for s in shapes:
            a = (rng.standard_normal(s) * 10.0).astype(dtype)
            flat = a.reshape(-1)
            n = flat.size
            pick = rng.random(n) < 0.3  # 30 % specials, per client
            flat[pick] = specials[rng.integers(0, specials.size, int(pick.sum()))]
            row.append(a)
        ups.append(row)
    return ups


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.float16])
@pytest.mark.parametrize("K", [1, 2, 7, 9, 33])
def test_fedavg_nonfinite_bit_exact(torch_gpu, dummy_algo_class, dtype, K):
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    rng = np.random.default_rng(1000 + K)
    ups = _nonfinite_updates(dtype, K, rng)
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    with np.errstate(all="ignore"):
        ref = fedavg_reference_structure(ups, ns)
    states = [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, ups)]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(shared_states=states, _skip=True).avg_parameters_update
    _assert_same_nan_aware(got, ref)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_scaffold_nonfinite_bit_exact(torch_gpu, dummy_algo_class, dtype):
    from substrafl_amd.schemas import ScaffoldSharedState
    from substrafl_amd.strategies import Scaffold

    rng = np.random.default_rng(77)
    K = 6
    pus = _nonfinite_updates(dtype, K, rng)
    cvs = _nonfinite_updates(dtype, K, rng)
    c = [(rng.standard_normal(a.shape) * 3).astype(dtype) for a in pus[0]]
    c[0].reshape(-1)[:3] = [np.inf, -np.inf, -0.0]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    with np.errstate(all="ignore"):
        ref_c, ref_avg = scaffold_reference_structure(pus, cvs, c, ns, 0.5)
    states = [ScaffoldSharedState(parameters_update=pus[k], control_variate_update=cvs[k], n_samples=ns[k],
                                  server_control_variate=c) for k in range(K)]
    got = Scaffold(algo=dummy_algo_class(), aggregation_lr=0.5).avg_shared_states(shared_states=states, _skip=True)
    _assert_same_nan_aware(got.avg_parameters_update, ref_avg)
    _assert_same_nan_aware(got.server_control_variate, ref_c)


@pytest.mark.parametrize("ns", [[5, -3, 7], [0, 0, 9, 0], [-1, -2, -4], [2**62, 3, 2**61 + 1], [1, 10**18, 7, 10**18 - 5],
                                [True, 3, 4]])
def test_n_samples_edge_values(torch_gpu, dummy_algo_class, ns):
    """negative and zero n_k are accepted, totals are exact Python ints (so huge
    counts keep their exact double ratio), True counts as 1 -- weights computed as the reference."""
    from substrafl_amd.schemas import FedAvgSharedState, ScaffoldSharedState
    from substrafl_amd.strategies import FedAvg, Scaffold

    rng = np.random.default_rng(len(ns))
    K = len(ns)
    shapes = [(33, 5), (1,), (1000,)]
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    states = [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, pus)]
    nsi = [s.n_samples for s in states]  # after the schema's coercion
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(shared_states=states, _skip=True).avg_parameters_update
    _assert_same(got, fedavg_reference_structure(pus, nsi))
    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    sst = [ScaffoldSharedState(parameters_update=pus[k], control_variate_update=cvs[k], n_samples=ns[k],
                               server_control_variate=c) for k in range(K)]
    sg = Scaffold(algo=dummy_algo_class(), aggregation_lr=0.3).avg_shared_states(shared_states=sst, _skip=True)
    ref_c, ref_avg = scaffold_reference_structure(pus, cvs, c, nsi, 0.3)
    _assert_same(sg.avg_parameters_update, ref_avg)
    _assert_same(sg.server_control_variate, ref_c)


# ------------------------------------------------------------------------------------------
# seeded random sweep: client counts, layer lists, dtypes and counts drawn together
# ------------------------------------------------------------------------------------------
def _random_case(seed):
    rng = np.random.default_rng(9000 + seed)
    K = int(rng.choice([1, 2, 3, 5, 8, 9, 16, 17, 31, 64, 127, 128, 129, 200, 257]))
    L = int(rng.integers(1, 10))
    shapes = []
    for _ in range(L):
        kind = rng.integers(0, 6)
        if kind == 0:
            shapes.append((1,))
        elif kind == 1:
            shapes.append((int(rng.integers(0, 3)), int(rng.integers(1, 40))))  # may be empty
        elif kind == 2:
            shapes.append((int(rng.integers(1, 9000)),))
        elif kind == 3:
            shapes.append(tuple(int(v) for v in rng.integers(1, 12, 3)))
        else:
            shapes.append((int(rng.integers(1, 300)), int(rng.integers(1, 300))))
    base = rng.choice([np.float32, np.float32, np.float64, np.float16])
    mixed = rng.random() < 0.2
    pus = []
    for _ in range(K):
        row = []
        for li, s in enumerate(shapes):
            dt = np.float64 if (mixed and li == 0) else base
            if mixed and li == 1 and len(shapes) > 1:
                row.append(rng.integers(-50, 50, s).astype(np.int64))
            else:
                row.append((rng.standard_normal(s) * 10.0 ** rng.integers(-3, 3)).astype(dt))
        pus.append(row)
    ns = [int(v) for v in rng.integers(0, 3000, K)]
    if sum(ns) == 0:
        ns[0] = 1
    return pus, ns


@pytest.mark.parametrize("seed", range(40))
def test_random_sweep_fedavg(torch_gpu, dummy_algo_class, seed):
    from substrafl_amd.schemas import FedAvgSharedState
    from substrafl_amd.strategies import FedAvg

    pus, ns = _random_case(seed)
    states = [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, pus)]
    got = FedAvg(algo=dummy_algo_class()).avg_shared_states(shared_states=states, _skip=True).avg_parameters_update
    _assert_same(got, fedavg_reference_structure(pus, ns))


@pytest.mark.parametrize("seed", range(40))
def test_random_sweep_scaffold(torch_gpu, dummy_algo_class, seed):
    from substrafl_amd.schemas import ScaffoldSharedState
    from substrafl_amd.strategies import Scaffold

    pus, ns = _random_case(100 + seed)
    rng = np.random.default_rng(seed)
    pus = [[np.asarray(a, dtype=np.float64 if seed % 3 == 0 else np.float32) for a in row] for row in pus]
    cvs = [[(rng.standard_normal(a.shape)).astype(a.dtype) for a in row] for row in pus]
    c = [rng.standard_normal(a.shape).astype(a.dtype) for a in pus[0]]
    lr = float(rng.choice([0.0, 0.5, 1.0, 2.5]))
    states = [ScaffoldSharedState(parameters_update=pus[k], control_variate_update=cvs[k], n_samples=ns[k],
                                  server_control_variate=c) for k in range(len(ns))]
    got = Scaffold(algo=dummy_algo_class(), aggregation_lr=lr).avg_shared_states(shared_states=states, _skip=True)
    ref_c, ref_avg = scaffold_reference_structure(pus, cvs, c, ns, lr)
    _assert_same(got.avg_parameters_update, ref_avg)
    _assert_same(got.server_control_variate, ref_c)


@pytest.mark.parametrize("seed", range(12))
def test_random_sweep_multi_device(torch_gpu, seed):
    from substrafl_amd.multi_device import MultiDeviceEngine

    pus, ns = _random_case(300 + seed)
    devices = (0,) * (1 + seed % 4)
    cap = [None, 20_000, 150_000, 1_000_000][seed % 4]
    got = MultiDeviceEngine(devices, max_shard_bytes=cap).fedavg(pus, ns)
    _assert_same(got, fedavg_reference_structure(pus, ns))


@pytest.mark.parametrize("copy_streams", [1, 2])
@pytest.mark.parametrize("chunk", [1 << 16, (1 << 20) + 4096, 4 << 20])
def test_session_staging_knobs_round_trip(torch_gpu, copy_streams, chunk):
    """The native session's staging (pinned ring, one or two H2D queues, any chunk size, byte
    ranges) lands every byte of every client's row where it belongs, before work enqueued after it
    on the session stream runs: staged rows come back bit-identical through fetch."""
    from substrafl_amd.runtime import Session

    rng = np.random.default_rng(chunk + copy_streams)
    K = 5
    sizes = [3, 1_000_003, 1, 777_777, 2_500_000]
    rows = [[rng.standard_normal(n).astype(np.float32) for n in sizes] for _ in range(K)]
    M = sum(sizes)
    ld = (M + 127) // 128 * 128
    s = Session(0, threads=4)
    try:
        s.set("chunk_bytes", chunk)
        s.set("copy_streams", copy_streams)
        d = s.buffer(0, K * ld * 4)
        s.memset(d, 0xFF, K * ld * 4)
        s.stage(d, ld * 4, rows)
        got = np.empty(K * ld, np.float32)
        s.fetch(d, got)
        for k in range(K):
            assert np.array_equal(got[k * ld: k * ld + M].view(np.uint32), np.concatenate(rows[k]).view(np.uint32))
            assert np.all(got[k * ld + M: (k + 1) * ld].view(np.uint32) == 0xFFFFFFFF)  # padding untouched
        lo, hi = 999_999, 3_100_001  # a parameter-range shard: bytes [4*lo, 4*hi) of every row
        d2 = s.buffer(1, K * (hi - lo) * 4)
        s.stage(d2, (hi - lo) * 4, rows, byte_range=(lo * 4, hi * 4))
        got2 = np.empty(K * (hi - lo), np.float32)
        s.fetch(d2, got2)
        for k in range(K):
            assert np.array_equal(got2[k * (hi - lo): (k + 1) * (hi - lo)], np.concatenate(rows[k])[lo:hi])
    finally:
        s.close()


def test_scaffold_0d_server_control_variate(torch_gpu, dummy_algo_class):
    """A client whose server control variate layer is 0-d and equal to every element of client 0's
    layer passes the reference's np.testing.assert_array_equal (scaffold.py:193-196); the average
    (which adds client 0's c, scaffold.py:262-263) is bit-exact; an unequal 0-d value is refused."""
    from substrafl_amd.schemas import ScaffoldSharedState
    from substrafl_amd.strategies import Scaffold

    rng = np.random.default_rng(77)
    shapes = [(40, 3), (7,), (1,)]
    K = 4
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c0 = [np.full((40, 3), 0.375, np.float32), rng.standard_normal(7).astype(np.float32), np.ones(1, np.float32)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]

    def states(c2):
        cs = [c0, [a.copy() for a in c0], c2, [a.copy() for a in c0]]
        return [ScaffoldSharedState(parameters_update=pus[k], control_variate_update=cvs[k], n_samples=ns[k],
                                    server_control_variate=cs[k]) for k in range(K)]

    good = [np.array(0.375, np.float32), c0[1].copy(), c0[2].copy()]
    res = Scaffold(algo=dummy_algo_class(), aggregation_lr=0.8).avg_shared_states(states(good), _skip=True)
    rc, ra = scaffold_reference_structure(pus, cvs, c0, ns, 0.8)
    _assert_same(res.server_control_variate, rc)
    _assert_same(res.avg_parameters_update, ra)
    bad = [np.array(0.5, np.float32), c0[1].copy(), c0[2].copy()]
    with pytest.raises(AssertionError, match="server_control_variate"):
        Scaffold(algo=dummy_algo_class(), aggregation_lr=0.8).avg_shared_states(states(bad), _skip=True)


@pytest.mark.parametrize("kind", ["f32", "bf16"])
@pytest.mark.parametrize("M", [300_001, 1_000_003, 2_500_007, 3_500_011])
def test_short_buckets_many_clients_vs_torch_sequential(torch_gpu, kind, M):
    """The short-bucket tiles of shape_for (from 32 clients: 2 x 8 under 1.5M fp32 elements, 4 x 4
    under 3M -- the runs of the client-sharded schedules): bit-exact against torch eager ops applied
    client by client, as a first launch and as a chain continuing an accumulator."""
    torch = torch_gpu
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights
    from substrafl_amd.sharding import GpuShardOps

    K = 64
    dt = torch.bfloat16 if kind == "bf16" else torch.float32
    x = torch.randn((K, M + 9), device="cuda").to(dt)
    ns = [int(v) for v in np.random.default_rng(M).integers(100, 10000, K)]
    w = fedavg_weights(ns, kind)
    out = torch.empty(M + 9, device="cuda")
    FedAvgPlan(kind, x, w, M, out, None).launch()
    acc = torch.zeros(M, device="cuda")
    for k in range(K):
        acc = acc + x[k, :M].float() * torch.tensor(w[k], device="cuda")
    half = torch.zeros(M, device="cuda")  # the chain form: clients 0..31, then 32..63 continuing it
    ops = GpuShardOps()
    ops.fedavg_run(kind, x[:32, :M], w[:32], True, half)
    ops.fedavg_run(kind, x[32:, :M], w[32:], False, half)
    torch.cuda.synchronize()
    assert torch.equal(out[:M].view(torch.int32), acc.view(torch.int32))
    assert torch.equal(half.view(torch.int32), acc.view(torch.int32))


@pytest.mark.parametrize("device", [None, "all"])
def test_non_native_byte_order_layers(torch_gpu, dummy_algo_class, device):
    """Arrays in big-endian byte order (a pickle written on a big-endian host): NumPy's ufuncs
    read them by value and give native-order results, so the engine converts them on the host
    (exactly) before staging -- FedAvg fp32/fp64/int layers and Scaffold, one GPU and the
    multi-device engine."""
    from substrafl_amd.schemas import FedAvgSharedState, ScaffoldSharedState
    from substrafl_amd.strategies import FedAvg, Scaffold

    rng = np.random.default_rng(11)
    K = 6
    mk = lambda s, dt: (rng.standard_normal(s) * 30).astype(dt)  # noqa: E731
    pus = [[mk((40, 3), ">f4"), mk((1,), ">f4"), mk((17,), ">f8"), mk((5,), ">i4"), mk((9,), np.float32)]
           for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    states = [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, pus)]
    got = FedAvg(algo=dummy_algo_class(), device=device).avg_shared_states(states, _skip=True).avg_parameters_update
    _assert_same(got, fedavg_reference_structure(pus, ns))

    shapes = [(13, 7), (1,), (130,)]
    sk = lambda: [mk(s, ">f4") for s in shapes]  # noqa: E731
    dpus, cvs, c = [sk() for _ in range(K)], [sk() for _ in range(K)], sk()
    sstates = [ScaffoldSharedState(parameters_update=dpus[k], control_variate_update=cvs[k], n_samples=ns[k],
                                   server_control_variate=c) for k in range(K)]
    res = Scaffold(algo=dummy_algo_class(), aggregation_lr=0.7, device=device).avg_shared_states(
        shared_states=sstates, _skip=True)
    rc, ra = scaffold_reference_structure(dpus, cvs, c, ns, 0.7)
    _assert_same(res.server_control_variate, rc)
    _assert_same(res.avg_parameters_update, ra)


BIG = 2 ** 32 + 4099  # a client row past 2^32 elements: every 32-bit element or vector index would wrap


@pytest.mark.parametrize("kind, K, layout", [("f32", 2, "rows"), ("f32", 2, "tiles"), ("bf16", 3, "rows")])
def test_rows_beyond_2_32_elements(torch_gpu, kind, K, layout):
    """Maximum sizes: client rows of 2^32 + 4099 elements (17 GB fp32 each), a ragged tail for
    the scalar remainder and a numel == 1 layer at index 2^32 + 4098 for the fused pairwise
    patch; bit-exact on every element against torch eager ops in list order, built in place so
    the check's own temporaries stay within one GPU's 288 GB."""
    torch = torch_gpu
    from substrafl_amd.engine import (FedAvgPlan, TiledFedAvgPlan, fedavg_weights, tiled_client_view, tiled_elems,
                                      tiled_tile)
    from substrafl_amd.layout import BucketLayout

    M = BIG
    lay = BucketLayout(range(2), [(M - 1,), (1,)], np.float32)
    assert lay.pairwise_idx.tolist() == [M - 1]
    dt = torch.bfloat16 if kind == "bf16" else torch.float32
    g = torch.Generator(device="cuda").manual_seed(23)
    ns = [int(v) for v in np.random.default_rng(23).integers(100, 10000, K)]
    w = fedavg_weights(ns, kind)
    out = torch.empty(lay.ld, device="cuda")
    if layout == "tiles":
        tv = tiled_tile(kind, K, M)
        x = torch.zeros(tiled_elems(kind, K, M, tv), device="cuda", dtype=dt)
        for k in range(K):
            view = tiled_client_view(x, kind, K, k, tv)  # strided: filled through a contiguous row
            row = torch.zeros(view.numel(), device="cuda", dtype=dt)
            row[:M].normal_(generator=g)
            view.copy_(row.view(view.shape))
            del row

        def row_of(k):
            return tiled_client_view(x, kind, K, k, tv).reshape(-1)  # a contiguous copy
        TiledFedAvgPlan(kind, x, K, w, M, out, lay.pairwise_idx, tv=tv).launch()
    else:
        x = torch.empty((K, lay.ld), device="cuda", dtype=dt)
        for k in range(K):
            x[k].normal_(generator=g)

        def row_of(k):
            return x[k]
        FedAvgPlan(kind, x, w, M, out, lay.pairwise_idx).launch()
    acc = torch.zeros(M - 1, device="cuda")
    prods = np.zeros(K, np.float32)
    for k in range(K):
        r = row_of(k)
        acc.add_(r[: M - 1].float() * torch.tensor(w[k], device="cuda"))
        prods[k] = (r[M - 1: M].float().cpu().numpy() * w[k]).astype(np.float32)[0]
        del r
    torch.cuda.synchronize()
    same = torch.equal(out[: M - 1].view(torch.int32), acc.view(torch.int32))
    same = same and _bits(np.float32(0.0) + numpy_pairwise_sum(prods)) == _bits(out[M - 1].cpu().numpy())
    del x, acc, out
    torch.cuda.empty_cache()
    assert same


def test_scaffold_rows_beyond_2_31_elements(torch_gpu):
    """Scaffold with rows of 2^31 + 4097 elements (fp64 outputs of 17 GB each): every element
    bit-exact against torch fp64 eager ops (w*x, +, c last, lr*) on the device."""
    torch = torch_gpu
    from substrafl_amd.engine import ScaffoldPlan, scaffold_weights

    K, M = 2, 2 ** 31 + 4097
    ld = (M + 63) // 64 * 64
    g = torch.Generator(device="cuda").manual_seed(29)
    d = torch.randn((K, ld), device="cuda", generator=g)
    cv = torch.randn((K, ld), device="cuda", generator=g)
    c = torch.randn(ld, device="cuda", generator=g)
    w = scaffold_weights([int(v) for v in np.random.default_rng(29).integers(100, 10000, K)])
    do = torch.empty(ld, dtype=torch.float64, device="cuda")
    co = torch.empty(ld, dtype=torch.float64, device="cuda")
    ScaffoldPlan("f32", d, cv, c, w, M, 0.7, do, co).launch()
    acc = torch.zeros(M, dtype=torch.float64, device="cuda")
    for k in range(K):
        acc.add_(torch.tensor(w[k], dtype=torch.float64, device="cuda") * d[k, :M].double())
    acc.mul_(torch.tensor(0.7, dtype=torch.float64, device="cuda"))  # lr * sum (lr first operand: same product)
    same = torch.equal(do[:M].view(torch.int64), acc.view(torch.int64))
    acc.zero_()
    for k in range(K):
        acc.add_(torch.tensor(w[k], dtype=torch.float64, device="cuda") * cv[k, :M].double())
    acc.add_(c[:M].double())
    torch.cuda.synchronize()
    same = same and torch.equal(co[:M].view(torch.int64), acc.view(torch.int64))
    del d, cv, c, do, co, acc
    torch.cuda.empty_cache()
    assert same


def test_host_path_rows_beyond_2_32_elements(torch_gpu):
    """The drop-in host path (pinned-ring staging, kernel, fetch) with two clients whose one layer
    holds 2^32 + 4099 fp32 elements (17 GB each): every element bit-exact against the reference's
    arithmetic (fed_avg.py:217-222: fl32(x * fl32(n_k / n)), summed in list order), checked in
    chunks.  The values repeat with a period of 1_000_003 elements, which does not divide 2^32:
    a wrapped 32-bit index would read the wrong value."""
    from substrafl_amd.engine import AggregationEngine, fedavg_weights

    M, P = BIG, 1_000_003
    rng = np.random.default_rng(31)
    rows = []
    for _ in range(2):
        base = rng.standard_normal(P).astype(np.float32)
        a = np.empty(M, np.float32)
        for lo in range(0, M, P * 64):  # block copies: no full-size temporaries
            hi = min(M, lo + P * 64)
            a[lo:hi] = np.resize(base, hi - lo) if hi - lo < P * 64 else np.tile(base, 64)
        rows.append([a])
    ns = [3, 5]
    (out,) = AggregationEngine(0).fedavg(rows, ns)
    w = fedavg_weights(ns, "f32")
    assert out.shape == (M,) and out.dtype == np.float32
    step = 1 << 28
    for lo in range(0, M, step):
        hi = min(M, lo + step)
        ref = np.float32(0.0) + rows[0][0][lo:hi] * w[0]
        ref += rows[1][0][lo:hi] * w[1]
        assert np.array_equal(ref.view(np.uint32), out[lo:hi].view(np.uint32)), lo
