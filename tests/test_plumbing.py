"""G7 plumbing: every aggregation of the reference's own 2-org linear FedAvg / Scaffold known-answer
experiments (final MAE 0.0127768361 / 0.0127768706, tests/algorithms/pytorch/test_fed_avg.py:25,
test_scaffold.py:26) and of an MNIST-shaped 2-org FedAvg, captured from the reference
(tests/golden/gen_plumbing.py), replayed through the oracle (CPU) and through substrafl_amd (GPU).
Bit-identical aggregates at every round => the experiment run with the MI355X aggregator produces
exactly the reference's models and known answers (client training is deterministic given them)."""

import json
from pathlib import Path

import numpy as np
import pytest

from oracle import fedavg_reference_structure, scaffold_reference_structure

D = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def plumbing():
    arrays = np.load(D / "golden_plumbing.npz", allow_pickle=False)
    meta = json.loads((D / "golden_plumbing_meta.json").read_text())
    return arrays, meta


def _calls(arrays, meta):
    for name, cfg in meta["configs"].items():
        for call in cfg["calls"]:
            key, K, L = call["key"], call["K"], call["layers"]
            ns = [int(v) for v in arrays[f"{key}/n_samples"]]
            pu = [[arrays[f"{key}/k{k}/pu{li}"] for li in range(L)] for k in range(K)]
            out = {"avg": [arrays[f"{key}/out_avg{li}"] for li in range(L)]}
            extra = {}
            if call["kind"] == "scaffold":
                extra["cv"] = [[arrays[f"{key}/k{k}/cv{li}"] for li in range(L)] for k in range(K)]
                extra["c"] = [[arrays[f"{key}/k{k}/c{li}"] for li in range(L)] for k in range(K)]
                out["c"] = [arrays[f"{key}/out_c{li}"] for li in range(L)]
            yield name, call, ns, pu, extra, out


def _bits(a):
    a = np.asarray(a)
    return a.view({4: np.uint32, 8: np.uint64}[a.dtype.itemsize])


def test_known_answers_recorded(plumbing):
    _, meta = plumbing
    cfg = meta["configs"]
    assert abs(cfg["linear_fedavg"]["final_performance"] - 0.0127768361) <= 1e-5 * 0.0127768361
    assert abs(cfg["linear_scaffold"]["final_performance"] - 0.0127768706) <= 1e-5 * 0.0127768706
    assert len(cfg["linear_fedavg"]["calls"]) == 3 and len(cfg["mnist_fedavg"]["calls"]) == 2
    shapes = cfg["mnist_fedavg"]["calls"][0]["shapes"]
    assert [8, 1, 3, 3] in shapes and [8] in shapes and [10, 1352] in shapes


def test_oracle_replays_every_aggregation(plumbing):
    arrays, meta = plumbing
    n = 0
    for name, call, ns, pu, extra, out in _calls(arrays, meta):
        if call["kind"] == "fedavg":
            got = {"avg": fedavg_reference_structure(pu, ns)}
        else:
            new_c, avg = scaffold_reference_structure(pu, extra["cv"], extra["c"][0], ns, call["aggregation_lr"])
            got = {"avg": avg, "c": new_c}
        for k in out:
            for g, r in zip(got[k], out[k]):
                assert g.dtype == r.dtype and np.array_equal(_bits(g), _bits(r)), (name, call["key"], k)
        n += 1
    assert n == 8


@pytest.mark.gpu
def test_mi355x_replays_every_aggregation(plumbing, dummy_algo_class):
    import torch

    assert torch.cuda.is_available()
    from substrafl_amd.schemas import FedAvgSharedState, ScaffoldSharedState
    from substrafl_amd.strategies import FedAvg, Scaffold

    arrays, meta = plumbing
    for name, call, ns, pu, extra, out in _calls(arrays, meta):
        if call["kind"] == "fedavg":
            res = FedAvg(algo=dummy_algo_class()).avg_shared_states(
                [FedAvgSharedState(n_samples=n, parameters_update=p) for n, p in zip(ns, pu)], _skip=True)
            got = {"avg": res.avg_parameters_update}
        else:
            states = [ScaffoldSharedState(parameters_update=pu[k], control_variate_update=extra["cv"][k], n_samples=ns[k],
                                          server_control_variate=extra["c"][k]) for k in range(len(ns))]
            res = Scaffold(algo=dummy_algo_class(), aggregation_lr=call["aggregation_lr"]).avg_shared_states(
                states, _skip=True)
            got = {"avg": res.avg_parameters_update, "c": res.server_control_variate}
        for k in out:
            for g, r in zip(got[k], out[k]):
                assert g.dtype == r.dtype and g.shape == r.shape and np.array_equal(_bits(g), _bits(r)), (name, k)
