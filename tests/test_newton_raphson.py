"""``accelerate(NewtonRaphson)``: the weighted Hessian / gradient sums of
``NewtonRaphson.compute_averaged_states`` (substrafl/strategies/newton_raphson.py:195-211) on the
engine (``engine.sequential_sum``: client 0's product by ``fedagg_scale_cast``, then the chain
kernel continuing it -- the reference's explicit ``+=`` order, no ``+0.0`` seed, no pairwise
order for ``numel == 1``), the dense solve and unflatten as the reference on the host.  Driven
through the builder-written stand-in package (tests/standin_substrafl) whose own averaging body
refuses to run; bit-exact to the reference's own outputs (golden_newton_raphson.npz) and to the
oracle's restatement on random inputs."""

import json
from pathlib import Path

import numpy as np
import pytest

import standin_substrafl.exceptions as sx
import standin_substrafl.strategies as ss
from standin_substrafl.strategies import schemas as sch

from oracle import newton_raphson_reference_structure, newton_raphson_sums

D = Path(__file__).resolve().parent / "golden"


class _Algo:
    pass


@pytest.fixture(scope="module")
def NR():
    from substrafl_amd.integration import accelerate

    return accelerate(ss.NewtonRaphson)


def _states(grads, hess, ns):
    return [sch.NewtonRaphsonSharedState(gradients=g, hessian=h, n_samples=n) for g, h, n in zip(grads, hess, ns)]


def _bits(a):
    a = np.asarray(a)
    return a.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize])


def _same(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        g, r = np.asarray(g), np.asarray(r)
        assert g.dtype == r.dtype and g.shape == r.shape, (g.dtype, r.dtype, g.shape, r.shape)
        assert np.array_equal(_bits(g), _bits(r))


# ---------------------------------------------------------------------------- CPU
def test_class_shape_and_host_errors(NR):
    s = NR(algo=_Algo(), damping_factor=0.5)
    assert isinstance(s, ss.NewtonRaphson) and s.name == sch.StrategyName.NEWTON_RAPHSON
    assert s._aggregation_methods == {"compute_averaged_states": "sequential"}
    with pytest.raises(ValueError):
        NR(algo=_Algo(), damping_factor=0)
    with pytest.raises(sx.EmptySharedStatesError):  # the package's own check, before any device work
        s.compute_averaged_states(shared_states=[], _skip=True)
    bad = _states([[np.ones(3, np.float32)]], [np.eye(2)], [1])
    with pytest.raises(sx.SharedStatesError):
        s.compute_averaged_states(shared_states=bad, _skip=True)
    zero = _states([[np.ones(2, np.float32)]] * 2, [np.eye(2)] * 2, [0, 0])
    with pytest.raises(ZeroDivisionError):
        s.compute_averaged_states(shared_states=zero, _skip=True)


def test_oracle_keeps_negative_zero_columns():
    """The reference's chain starts from client 0's product: an all -0.0 column stays -0.0 (FedAvg's
    np.sum would start from +0.0)."""
    g = [[np.array([-0.0, 1.0], np.float32)], [np.array([-0.0, 2.0], np.float32)]]
    h = [np.array([[2.0, -0.0], [-0.0, 2.0]])] * 2
    H, G = newton_raphson_sums(g, h, [1, 3])
    assert np.signbit(H[0, 1]) and np.signbit(G[0])


# ---------------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from substrafl_amd import _native

    _native.load()


@pytest.mark.gpu
def test_golden_outputs_bit_exact(NR, gpu):
    arrays = np.load(D / "golden_newton_raphson.npz", allow_pickle=False)
    meta = json.loads((D / "golden_newton_raphson_meta.json").read_text())
    for c in meta["cases"]:
        key, K, L = c["key"], c["K"], c["layers"]
        grads = [[arrays[f"{key}/k{k}/g{li}"] for li in range(L)] for k in range(K)]
        hess = [arrays[f"{key}/k{k}/h"] for k in range(K)]
        ns = [int(v) for v in arrays[f"{key}/n_samples"]]
        res = NR(algo=_Algo(), damping_factor=c["damping_factor"]).compute_averaged_states(
            shared_states=_states(grads, hess, ns), _skip=True)
        assert isinstance(res, sch.NewtonRaphsonAveragedStates)
        # the sums bit for bit against the oracle on this box; the output against the reference's
        # own bits (the solve is the reference's np.linalg.solve on the same sums)
        from substrafl_amd.integration import newton_raphson_sums as engine_sums

        H, G = engine_sums(_states(grads, hess, ns))
        Hr, Gr = newton_raphson_sums(grads, hess, ns)
        _same([H, G], [Hr, Gr])
        _same(res.parameters_update, newton_raphson_reference_structure(grads, hess, ns, c["damping_factor"]))


@pytest.mark.gpu
@pytest.mark.parametrize("K,P", [(1, 300), (2, 1), (9, 64), (33, 700), (130, 257)])
def test_random_sums_bit_exact(gpu, K, P):
    """Client counts across the chain kernel's client chunks (K > 128), P = 1 (numel == 1: no
    pairwise order here), signed zeros and a zero-sample client."""
    from substrafl_amd.integration import newton_raphson_sums as engine_sums

    rng = np.random.default_rng(K * 1000 + P)
    shapes = [(P - 1,), (1,)] if P > 1 else [(1,)]
    grads = [[np.where(rng.random(s) < 0.1, np.float32(-0.0), rng.standard_normal(s).astype(np.float32))
              for s in shapes] for _ in range(K)]
    hess = []
    for _ in range(K):
        h = rng.standard_normal((P, P))
        h[rng.random((P, P)) < 0.1] = -0.0
        hess.append(h)
    ns = [int(v) for v in rng.integers(0, 5000, K)]
    ns[0] = max(ns[0], 1)
    H, G = engine_sums(_states(grads, hess, ns))
    _same([H, G], list(newton_raphson_sums(grads, hess, ns)))


@pytest.mark.gpu
def test_integer_inputs_and_large_hessian(gpu):
    """Integer arrays (int64 x Python float multiplies as float64, cast on the device) and a
    2048 x 2048 float64 Hessian per client (4M elements, 8 clients)."""
    from substrafl_amd.integration import newton_raphson_sums as engine_sums

    rng = np.random.default_rng(3)
    gi = [[rng.integers(-5, 5, (3,))] for _ in range(3)]
    hi = [rng.integers(-5, 5, (3, 3)) for _ in range(3)]
    H, G = engine_sums(_states(gi, hi, [2, 5, 1]))
    _same([H, G], list(newton_raphson_sums(gi, hi, [2, 5, 1])))
    P, K = 2048, 8
    grads = [[rng.standard_normal(P).astype(np.float32)] for _ in range(K)]
    hess = [rng.standard_normal((P, P)) for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 100, K)]
    H, G = engine_sums(_states(grads, hess, ns))
    _same([H, G], list(newton_raphson_sums(grads, hess, ns)))


_DT = {"f16": np.float16, "f32": np.float32, "f64": np.float64, "i64": np.int64}


@pytest.mark.gpu
@pytest.mark.parametrize("dts", [("f32", "f64"), ("f64", "f32", "f32"), ("f16", "f16", "f16"), ("f16", "f32", "f16"),
                                 ("f32", "i64", "f64", "f32"), ("f16", "f64"), ("i64", "f32")])
def test_mixed_and_half_client_dtypes_bit_exact(gpu, dts):
    """the reference's ``total += x_k * c_k`` casts every later client into client 0's
    type (NumPy adds in the promoted type, then rounds back) and takes float16 arrays; the engine
    does the same on the device, bit for bit -- no input the reference accepts is refused."""
    from substrafl_amd.integration import newton_raphson_sums as engine_sums

    rng = np.random.default_rng(len(dts) * 7 + sum(map(len, dts)))
    P = 37

    def arr(shape, dt):
        x = rng.standard_normal(shape) * 3
        x[rng.random(shape) < 0.1] = -0.0
        return (np.round(x) if dt == "i64" else x).astype(_DT[dt])

    grads = [[arr((P - 1,), dt), arr((1,), dt)] for dt in dts]
    hess = [arr((P, P), dt) for dt in dts]
    ns = [int(v) for v in rng.integers(1, 5000, len(dts))]
    H, G = engine_sums(_states(grads, hess, ns))
    Hr, Gr = newton_raphson_sums(grads, hess, ns)
    assert H.dtype == Hr.dtype and G.dtype == Gr.dtype
    _same([H, G], [Hr, Gr])
