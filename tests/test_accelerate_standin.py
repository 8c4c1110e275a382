"""``substrafl_amd.integration.accelerate`` with the REAL engine (VERDICT r03 "Next 3"): the drop-in
and the kernels had each been tested, never together -- the container has no GPU (its
reference-driven test swaps in an oracle engine, tests/reference_drop_in.py) and the GPU box has no
reference.  Here ``accelerate`` takes the classes of ``tests/standin_substrafl`` -- a builder-written
package with the reference's module paths, class and field names and ``@remote`` convention, whose
own aggregation bodies refuse to run -- and the accelerated methods go through libfedagg on the GPU:
bit-exact to the golden vectors the reference itself produced (``golden_aggregation.npz``: G1-G5,
G8 FedAvg, G3 Scaffold, G9 FedPCA) and to every aggregation of the G7 plumbing runs
(``golden_plumbing.npz``; fed_avg.py:176-224, scaffold.py:297-337, fed_pca.py:210-299)."""

import json
from pathlib import Path

import numpy as np
import pytest

import standin_substrafl.exceptions as sx
import standin_substrafl.strategies as ss
from standin_substrafl.remote import RemoteOperation
from standin_substrafl.strategies import schemas as sch

D = Path(__file__).resolve().parent / "golden"


def _bits(a):
    a = np.asarray(a)
    return a.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize])


def _same(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert isinstance(g, np.ndarray)
        assert g.dtype == r.dtype and g.shape == r.shape, (g.dtype, r.dtype, g.shape, r.shape)
        assert np.array_equal(_bits(g), _bits(r))


class _Algo:
    pass


@pytest.fixture(scope="module")
def acc():
    from substrafl_amd.integration import accelerate

    return {"fedavg": accelerate(ss.FedAvg), "scaffold": accelerate(ss.Scaffold), "fedpca": accelerate(ss.FedPCA)}


# ---------------------------------------------------------------------------- CPU: the class shape
def test_accelerate_keeps_the_standin_class(acc):
    """The accelerated classes are subclasses of the package's own, keep its constructor, name and
    kwargs, and name the engine kind of each aggregation method."""
    f = acc["fedavg"](algo=_Algo(), metric_functions={"m": len})
    assert isinstance(f, ss.FedAvg) and f.name == sch.StrategyName.FEDERATED_AVERAGING
    assert f.metric_functions == {"m": len}
    s = acc["scaffold"](algo=_Algo(), aggregation_lr=0.7)
    assert isinstance(s, ss.Scaffold) and s._aggregation_lr == 0.7
    with pytest.raises(ValueError):
        acc["scaffold"](algo=_Algo(), aggregation_lr=-1)
    assert acc["fedpca"]._aggregation_methods == {"avg_shared_states": "fedavg", "avg_shared_states_with_qr": "fedavg"}
    assert acc["scaffold"]._aggregation_methods == {"avg_shared_states": "scaffold"}
    from substrafl_amd.integration import accelerate

    with pytest.raises(TypeError):
        accelerate(ss.Strategy)


def test_graph_mode_returns_the_packages_remote_operation(acc):
    """Without ``_skip`` the package's own ``@remote`` records the operation (compute-plan
    building): no engine call, no GPU."""
    states = [sch.FedAvgSharedState(n_samples=1, parameters_update=[np.ones(3, np.float32)])]
    op = acc["fedavg"](algo=_Algo()).avg_shared_states(shared_states=states)
    assert isinstance(op, RemoteOperation) and op.method_name == "avg_shared_states"
    assert issubclass(op.cls, ss.FedAvg)


def test_empty_input_raises_the_packages_error_before_any_device_work(acc):
    with pytest.raises(sx.EmptySharedStatesError):
        acc["fedavg"](algo=_Algo()).avg_shared_states(shared_states=[], _skip=True)
    with pytest.raises(sx.EmptySharedStatesError):
        acc["fedpca"](algo=_Algo()).avg_shared_states(shared_states=[], _skip=True)


# ---------------------------------------------------------------------------- GPU: the real engine
@pytest.fixture(scope="module")
def gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from substrafl_amd import _native

    _native.load()  # no fallback: the accelerated bodies run on libfedagg


@pytest.mark.gpu
def test_accelerated_goldens_bit_exact(acc, golden, gpu):
    arrays, meta = golden
    fa, sc, pca = acc["fedavg"](algo=_Algo()), None, acc["fedpca"](algo=_Algo())
    counts = {"fedavg": 0, "scaffold": 0, "fedpca": 0}
    for case in meta["cases"]:
        key, K, L = case.get("key"), case.get("K"), case.get("layers")
        if case["strategy"] == "fedavg":
            ns = [int(v) for v in arrays[f"{key}/n_samples"]]
            states = [sch.FedAvgSharedState(n_samples=ns[k],
                                            parameters_update=[arrays[f"{key}/x{li}"][k] for li in range(L)])
                      for k in range(K)]
            _same(fa.avg_shared_states(shared_states=states, _skip=True).avg_parameters_update,
                  [arrays[f"{key}/out{li}"] for li in range(L)])
        elif case["strategy"] == "scaffold":
            lr = int(case["lr"]) if case["lr_is_int"] else float(case["lr"])
            ns = [int(v) for v in arrays[f"{key}/n_samples"]]
            c = [arrays[f"{key}/c{li}"] for li in range(L)]
            states = [sch.ScaffoldSharedState(parameters_update=[arrays[f"{key}/pu{li}"][k] for li in range(L)],
                                              control_variate_update=[arrays[f"{key}/cv{li}"][k] for li in range(L)],
                                              n_samples=ns[k], server_control_variate=c) for k in range(K)]
            sc = acc["scaffold"](algo=_Algo(), aggregation_lr=lr)
            res = sc.avg_shared_states(shared_states=states, _skip=True)
            assert isinstance(res, sch.ScaffoldAveragedStates)
            _same(res.avg_parameters_update, [arrays[f"{key}/avg{li}"] for li in range(L)])
            _same(res.server_control_variate, [arrays[f"{key}/newc{li}"] for li in range(L)])
        elif case["strategy"] == "fedpca":
            ns = [int(v) for v in arrays[f"{key}/n_samples"]]
            states = [sch.FedPCASharedState(n_samples=ns[k],
                                            parameters_update=[arrays[f"{key}/x{li}"][k] for li in range(L)])
                      for k in range(K)]
            res = pca.avg_shared_states(shared_states=states, _skip=True)
            assert isinstance(res, sch.FedPCAAveragedState)
            _same(res.avg_parameters_update, [arrays[f"{key}/avg{li}"] for li in range(L)])
            _same(pca.avg_shared_states_with_qr(shared_states=states, _skip=True).avg_parameters_update,
                  [arrays[f"{key}/qr{li}"] for li in range(L)])
        else:
            continue
        counts[case["strategy"]] += 1
    assert counts["fedavg"] >= 40 and counts["scaffold"] >= 6 and counts["fedpca"] >= 1, counts


@pytest.mark.gpu
def test_accelerated_plumbing_runs_bit_exact(acc, gpu):
    """Every aggregation of the reference's own 2-org FedAvg / Scaffold known-answer runs and of the
    MNIST-shaped run (G7), replayed through the accelerated stand-in classes."""
    arrays = np.load(D / "golden_plumbing.npz", allow_pickle=False)
    meta = json.loads((D / "golden_plumbing_meta.json").read_text())
    n = 0
    for name, cfg in meta["configs"].items():
        for call in cfg["calls"]:
            key, K, L = call["key"], call["K"], call["layers"]
            ns = [int(v) for v in arrays[f"{key}/n_samples"]]
            pu = [[arrays[f"{key}/k{k}/pu{li}"] for li in range(L)] for k in range(K)]
            if call["kind"] == "fedavg":
                res = acc["fedavg"](algo=_Algo()).avg_shared_states(
                    shared_states=[sch.FedAvgSharedState(n_samples=a, parameters_update=b) for a, b in zip(ns, pu)],
                    _skip=True)
                _same(res.avg_parameters_update, [arrays[f"{key}/out_avg{li}"] for li in range(L)])
            else:
                states = [sch.ScaffoldSharedState(
                    parameters_update=pu[k], control_variate_update=[arrays[f"{key}/k{k}/cv{li}"] for li in range(L)],
                    n_samples=ns[k], server_control_variate=[arrays[f"{key}/k{k}/c{li}"] for li in range(L)])
                    for k in range(K)]
                res = acc["scaffold"](algo=_Algo(), aggregation_lr=call["aggregation_lr"]).avg_shared_states(
                    shared_states=states, _skip=True)
                _same(res.avg_parameters_update, [arrays[f"{key}/out_avg{li}"] for li in range(L)])
                _same(res.server_control_variate, [arrays[f"{key}/out_c{li}"] for li in range(L)])
            n += 1
    assert n == 8


@pytest.mark.gpu
def test_accelerated_errors_on_the_gpu_path(acc, gpu):
    """The reference's error behaviour through the accelerated bodies: zero samples, layer-count
    and shape mismatches, a differing server control variate."""
    fa = acc["fedavg"](algo=_Algo())
    one = np.ones(2, np.float32)
    with pytest.raises(ZeroDivisionError):
        fa.avg_shared_states(shared_states=[sch.FedAvgSharedState(n_samples=0, parameters_update=[one])] * 2,
                             _skip=True)
    with pytest.raises(AssertionError):
        fa.avg_shared_states(shared_states=[sch.FedAvgSharedState(n_samples=1, parameters_update=[one]),
                                            sch.FedAvgSharedState(n_samples=1, parameters_update=[])], _skip=True)
    with pytest.raises(ValueError):
        fa.avg_shared_states(shared_states=[sch.FedAvgSharedState(n_samples=1, parameters_update=[one]),
                                            sch.FedAvgSharedState(n_samples=1, parameters_update=[np.ones(3, np.float32)])],
                             _skip=True)
    sc = acc["scaffold"](algo=_Algo())
    mk = lambda c: sch.ScaffoldSharedState(parameters_update=[one], control_variate_update=[one], n_samples=3,  # noqa: E731
                                           server_control_variate=[c])
    with pytest.raises(AssertionError):
        sc.avg_shared_states(shared_states=[mk(one), mk(one * 2)], _skip=True)


@pytest.mark.gpu
def test_accelerated_calls_load_the_native_library(acc, gpu):
    """The accelerated body ran on libfedagg (the stand-in's own body would have raised)."""
    fa = acc["fedavg"](algo=_Algo())
    res = fa.avg_shared_states(shared_states=[sch.FedAvgSharedState(n_samples=n, parameters_update=[np.full(
        (3,), float(n), np.float32)]) for n in (1, 3)], _skip=True)
    assert [float(v) for v in res.avg_parameters_update[0]] == [2.5, 2.5, 2.5]  # (1*1 + 3*3) / 4
    maps = Path("/proc/self/maps").read_text()
    assert "libfedagg.so" in maps


def test_accelerate_takes_a_user_subclass_defined_anywhere():
    """A user's own FedAvg subclass (defined in the user's module, not the package's) finds the
    package's modules through its MRO."""
    from substrafl_amd.integration import accelerate

    class MyFedAvg(ss.FedAvg):
        pass

    acc = accelerate(MyFedAvg)
    assert issubclass(acc, MyFedAvg) and acc._aggregation_methods == {"avg_shared_states": "fedavg"}
    with pytest.raises(sx.EmptySharedStatesError):
        acc(algo=_Algo()).avg_shared_states(shared_states=[], _skip=True)
