"""CONTAINER-ONLY checker (imports /root/reference; never runs on the GPU box): the reference's own
experiment driver runs with ``substrafl_amd.integration.accelerate``'d strategy classes.

``simulate_experiment`` (substrafl/experiment.py) drives ``accelerate(FedAvg)`` and
``accelerate(Scaffold)`` through the reference's graph building (``perform_round``,
``build_compute_plan``), ``@remote`` / ``RemoteStruct`` and aggregation node -- the 2-org linear
known-answer setup of tests/golden/gen_plumbing.py -- and the final performance must equal, to the
last bit, the one the unmodified reference produced when the G7 fixtures were captured
(tests/golden/golden_plumbing_meta.json).  There is no GPU in this container, so the engine behind
the accelerated methods is a test double that computes with the oracle's explicit-order
restatement (oracle/aggregation.py, pinned bit-exact by the golden vectors); the GPU side of the
same calls is the G7 replay in tests/test_plumbing.py.  Also checked: the generated class is
carried by value through cloudpickle (the task process's ``RemoteStruct``), and the reference's
error types surface unchanged.  Prints one JSON line.
"""

from __future__ import annotations

import json
import sys
import tempfile
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True  # never write into /root/reference
HERE = Path(__file__).resolve().parent
ROOT = HERE.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(HERE / "golden"))
sys.path.insert(0, str(HERE / "refplugin"))
from gen_golden import REF, _install_stubs  # noqa: E402
from gen_plumbing import linear_data  # noqa: E402



from oracle_engine import OracleEngine  # noqa: E402  (tests/refplugin/oracle_engine.py)


def main():
    if not REF.exists():
        raise SystemExit("reference_drop_in.py needs /root/reference (build container only)")
    _install_stubs()
    import types

    sys.modules["substra"].BackendType = types.SimpleNamespace(REMOTE="remote", LOCAL_SUBPROCESS="subprocess",
                                                               LOCAL_DOCKER="docker")
    sys.path.insert(0, str(REF))
    import cloudpickle
    import torch

    import substrafl.nodes.test_data_node as tdn
    import substrafl.nodes.train_data_node as trn
    from substrafl import exceptions as ref_exceptions
    from substrafl import simulate_experiment
    from substrafl.algorithms.pytorch import TorchFedAvgAlgo, TorchScaffoldAlgo
    from substrafl.evaluation_strategy import EvaluationStrategy
    from substrafl.index_generator import NpIndexGenerator
    from substrafl.nodes import AggregationNode, TestDataNode, TrainDataNode
    from substrafl.remote.operations import RemoteOperation
    from substrafl.strategies import FedAvg, Scaffold
    from substrafl.strategies.schemas import FedAvgSharedState

    import substrafl_amd.integration as integ
    import substrafl_amd.strategies.fed_avg as mirror_fedavg

    engine = OracleEngine()
    integ.engine_for = mirror_fedavg.engine_for = lambda device=None: engine

    data = {}
    trn.preload_data = tdn.preload_data = lambda client, data_manager_key, data_sample_keys: data[data_sample_keys[0]]

    class Client:
        backend_mode = "subprocess"

    class TorchDataset(torch.utils.data.Dataset):  # tests/conftest.py:424-441
        def __init__(self, data_from_opener, is_inference=False):
            self.x, self.y, self.is_inference = data_from_opener[0], data_from_opener[1], is_inference

        def __getitem__(self, index):
            x = torch.from_numpy(self.x[index]).float()
            if self.is_inference:
                return x
            return x, torch.as_tensor(self.y[index]).float()

        def __len__(self):
            return len(self.x)

    class Perceptron(torch.nn.Module):  # tests/conftest.py:322-341
        def __init__(self):
            super().__init__()
            self.linear1 = torch.nn.Linear(2, 1)

        def forward(self, x):
            return self.linear1(x)

    def mae_score(data_from_opener, predictions):  # tests/conftest.py:133-144
        return abs(np.array(predictions) - data_from_opener[1]).mean()

    split = lambda d: (d[:, :-1], d[:, -1:])  # noqa: E731
    train = [split(linear_data(n_col=3, n_samples=1024, weights_seed=42, noise_seed=i)) for i in range(2)]
    test = split(linear_data(n_col=3, n_samples=64, weights_seed=42, noise_seed=42))

    def run(strategy_cls, algo_base, rounds=3):
        data.clear()
        for i, d in enumerate(train):
            data[f"train{i}"] = d
        data["test0"] = test
        torch.manual_seed(42)
        model = Perceptron()
        nig = NpIndexGenerator(batch_size=32, num_updates=100)

        class MyAlgo(algo_base):
            def __init__(self):
                super().__init__(optimizer=torch.optim.SGD(model.parameters(), lr=0.1), criterion=torch.nn.MSELoss(),
                                 model=model, index_generator=nig, dataset=TorchDataset)

        strategy = strategy_cls(algo=MyAlgo(), metric_functions=mae_score)
        perf, _, _ = simulate_experiment(
            client=Client(), strategy=strategy,
            train_data_nodes=[TrainDataNode(f"org{i}", "ds", [f"train{i}"]) for i in range(2)],
            evaluation_strategy=EvaluationStrategy(test_data_nodes=[TestDataNode("org0", "ds", ["test0"])],
                                                   eval_rounds=[0, rounds]),
            aggregation_node=AggregationNode("org0"), num_rounds=rounds, clean_models=True,
            experiment_folder=tempfile.mkdtemp())
        return float(perf.performance[-1]), strategy

    meta = json.loads((HERE / "golden" / "golden_plumbing_meta.json").read_text())["configs"]
    out = {}
    AccFedAvg, AccScaffold = integ.accelerate(FedAvg), integ.accelerate(Scaffold)
    assert issubclass(AccFedAvg, FedAvg) and issubclass(AccScaffold, Scaffold)
    assert AccScaffold._aggregation_methods == {"avg_shared_states": "scaffold"}
    assert callable(AccFedAvg.prewarm_aggregation) and callable(AccFedAvg.ingest_shared_states)
    perf, strat = run(AccFedAvg, TorchFedAvgAlgo)
    out["linear_fedavg"] = {"final": perf, "reference_final": meta["linear_fedavg"]["final_performance"],
                            "engine_calls": engine.calls["fedavg"]}
    perf, _ = run(AccScaffold, TorchScaffoldAlgo)
    out["linear_scaffold"] = {"final": perf, "reference_final": meta["linear_scaffold"]["final_performance"],
                              "engine_calls": engine.calls["scaffold"]}

    # the client half: accelerate_algo over the reference's own algorithm classes (the user
    # subclasses the accelerated class), both halves accelerated in one simulate_experiment
    AccFedAvgAlgo, AccScaffoldAlgo = integ.accelerate_algo(TorchFedAvgAlgo), integ.accelerate_algo(TorchScaffoldAlgo)
    assert issubclass(AccFedAvgAlgo, TorchFedAvgAlgo) and issubclass(AccScaffoldAlgo, TorchScaffoldAlgo)
    calls0 = dict(engine.calls)
    perf, strat_algo = run(AccFedAvg, AccFedAvgAlgo)
    out["linear_fedavg_accelerate_algo"] = {
        "final": perf, "reference_final": meta["linear_fedavg"]["final_performance"],
        "engine_calls": engine.calls["fedavg"] - calls0["fedavg"],
        "train_is_accelerated": type(strat_algo.algo).train.__qualname__.startswith("_fedavg_train")}
    perf, strat_algo = run(AccScaffold, AccScaffoldAlgo)
    out["linear_scaffold_accelerate_algo"] = {
        "final": perf, "reference_final": meta["linear_scaffold"]["final_performance"],
        "engine_calls": engine.calls["scaffold"] - calls0["scaffold"],
        "train_is_accelerated": type(strat_algo.algo).train.__qualname__.startswith("_scaffold_train")}
    # the algo's RemoteDataStruct carries the generated class (and its train) by value too
    blob = cloudpickle.dumps(type(strat_algo.algo))
    out["algo_class_by_value"] = b"_scaffold_train.<locals>.train" in blob

    # @remote: without _skip the call is a RemoteOperation naming the generated class, which
    # cloudpickle carries by value (the task process re-creates it from the RemoteStruct)
    states = [FedAvgSharedState(n_samples=n, parameters_update=[np.full((3,), float(n), np.float32)])
              for n in (1, 3)]
    op = strat.avg_shared_states(shared_states=states)
    assert isinstance(op, RemoteOperation) and op.remote_struct._method_name == "avg_shared_states"
    blob = cloudpickle.dumps(op.remote_struct)
    inst = cloudpickle.loads(blob).get_remote_instance()
    res = inst.instance.avg_shared_states(shared_states=states, _skip=True)
    out["remote_struct_roundtrip"] = {"bytes": len(blob), "class_by_value": b"accelerate.<locals>" in blob,
                                      "result": [float(v) for v in res.avg_parameters_update[0]]}

    # FedPCA: both aggregation methods against the unmodified reference class on the same states
    from substrafl.algorithms.algo import Algo
    from substrafl.strategies import FedPCA
    from substrafl.strategies.schemas import FedPCASharedState, StrategyName

    class PcaAlgo(Algo):
        strategies = property(lambda self: list(StrategyName))
        model = property(lambda self: None)

        def train(self, data_from_opener, shared_state):  # never called here
            return None

        def predict(self, data_from_opener, shared_state):
            return None

        def load_local_state(self, path):
            return self

        def save_local_state(self, path):
            pass

    rng = np.random.default_rng(5)
    pca_states = [FedPCASharedState(n_samples=int(n), parameters_update=[rng.standard_normal((6, 4)),
                                                                          rng.standard_normal((3,))])
                  for n in (17, 5, 230)]
    ref_pca, acc_pca = FedPCA(algo=PcaAlgo()), integ.accelerate(FedPCA)(algo=PcaAlgo())
    same = {}
    for meth in ("avg_shared_states", "avg_shared_states_with_qr"):
        states = pca_states if meth == "avg_shared_states" else [
            FedPCASharedState(n_samples=st.n_samples, parameters_update=[st.parameters_update[0]]) for st in pca_states]
        r = getattr(ref_pca, meth)(shared_states=states, _skip=True).avg_parameters_update
        a = getattr(acc_pca, meth)(shared_states=states, _skip=True).avg_parameters_update
        same[meth] = len(r) == len(a) and all(x.dtype == y.dtype and np.array_equal(x.view(np.uint64), y.view(np.uint64))
                                               for x, y in zip(r, a))
    out["fedpca_bit_identical"] = same

    # NewtonRaphson: accelerate(NewtonRaphson) against the unmodified class on the same states
    # (the reference's own unit-test inputs and the golden file's), bit for bit
    from substrafl.strategies import NewtonRaphson
    from substrafl.strategies.schemas import NewtonRaphsonSharedState

    nr_arrays = np.load(HERE / "golden" / "golden_newton_raphson.npz", allow_pickle=False)
    nr_meta = json.loads((HERE / "golden" / "golden_newton_raphson_meta.json").read_text())
    nr_same = []
    AccNR = integ.accelerate(NewtonRaphson)
    for c in nr_meta["cases"]:
        key, K, L = c["key"], c["K"], c["layers"]
        states = [NewtonRaphsonSharedState(gradients=[nr_arrays[f"{key}/k{k}/g{li}"] for li in range(L)],
                                           hessian=nr_arrays[f"{key}/k{k}/h"], n_samples=int(nr_arrays[f"{key}/n_samples"][k]))
                  for k in range(K)]
        r = NewtonRaphson(algo=PcaAlgo(), damping_factor=c["damping_factor"]).compute_averaged_states(
            shared_states=states, _skip=True).parameters_update
        a = AccNR(algo=PcaAlgo(), damping_factor=c["damping_factor"]).compute_averaged_states(
            shared_states=states, _skip=True).parameters_update
        nr_same.append(len(r) == len(a) and all(x.dtype == y.dtype and np.array_equal(x.view(np.uint64), y.view(np.uint64))
                                                for x, y in zip(r, a)))
    out["newton_raphson_bit_identical"] = {"cases": len(nr_same), "all": all(nr_same),
                                           "engine_calls": engine.calls.get("sequential", 0)}

    # ... and in the reference's simulate_experiment with its TorchNewtonRaphsonAlgo (2-org linear
    # data): the accelerated run's final performance equals the unmodified one's
    from substrafl.algorithms.pytorch import TorchNewtonRaphsonAlgo

    def run_nr(strategy_cls, rounds=2):
        data.clear()
        for i, d in enumerate(train):
            data[f"train{i}"] = d
        data["test0"] = test
        torch.manual_seed(42)
        model = Perceptron()

        class NRAlgo(TorchNewtonRaphsonAlgo):
            def __init__(self):
                super().__init__(model=model, criterion=torch.nn.MSELoss(), batch_size=64, dataset=TorchDataset,
                                 l2_coeff=0)

        strategy = strategy_cls(algo=NRAlgo(), metric_functions=mae_score, damping_factor=0.8)
        perf, _, _ = simulate_experiment(
            client=Client(), strategy=strategy,
            train_data_nodes=[TrainDataNode(f"org{i}", "ds", [f"train{i}"]) for i in range(2)],
            evaluation_strategy=EvaluationStrategy(test_data_nodes=[TestDataNode("org0", "ds", ["test0"])],
                                                   eval_rounds=[rounds]),
            aggregation_node=AggregationNode("org0"), num_rounds=rounds, clean_models=True,
            experiment_folder=tempfile.mkdtemp())
        return float(perf.performance[-1])

    calls0 = engine.calls.get("sequential", 0)
    ref_perf = run_nr(NewtonRaphson)
    acc_perf = run_nr(AccNR)
    out["newton_raphson_simulate"] = {"reference": ref_perf, "accelerated": acc_perf,
                                      "engine_calls": engine.calls.get("sequential", 0) - calls0}

    # the reference's error types
    errs = {}
    for name, call, exc in (
            ("empty", lambda: strat.avg_shared_states(shared_states=[], _skip=True),
             ref_exceptions.EmptySharedStatesError),
            ("zero_samples", lambda: strat.avg_shared_states(
                shared_states=[FedAvgSharedState(n_samples=0, parameters_update=[np.ones(2, np.float32)])] * 2,
                _skip=True), ZeroDivisionError),
            ("layer_count", lambda: strat.avg_shared_states(
                shared_states=[FedAvgSharedState(n_samples=1, parameters_update=[np.ones(2, np.float32)]),
                               FedAvgSharedState(n_samples=1, parameters_update=[])], _skip=True), AssertionError)):
        try:
            call()
            errs[name] = "no exception"
        except exc:
            errs[name] = exc.__name__
    out["errors"] = errs
    print(json.dumps(out))


if __name__ == "__main__":
    main()
