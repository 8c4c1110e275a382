"""G7 plumbing fixtures: every aggregation of two small end-to-end SubstraFL simulations, captured
from the REFERENCE running in this container.

CONTAINER-ONLY (imports /root/reference; never runs on the GPU box).  Configs (BASELINE.json
configs[0] "MNIST FedAvg, 2 train orgs", plumbing only):

* ``linear_fedavg`` / ``linear_scaffold``: the reference's own 2-org linear known-answer setup
  (tests/algorithms/pytorch/test_fed_avg.py:25-120, test_scaffold.py; data
  tests/assets_factory.py:149-173 via tests/conftest.py:191-246, perceptron conftest.py:322-341,
  SGD lr 0.1, MSE, batch 32, 100 updates, 3 rounds, seed 42).  Its final MAE must equal
  EXPECTED_PERFORMANCE = 0.0127768361 (rtol 1e-5) -- checked here before anything is written.
* ``mnist_fedavg``: an MNIST-shaped synthetic set (1x28x28, 10 classes; MNIST/torchvision are not
  available offline) with a small CNN incl. BatchNorm running statistics, 2 orgs, 2 rounds.

For every call of ``avg_shared_states`` the K input shared states and the output are stored;
tests/test_gpu_plumbing.py replays them through substrafl_amd and requires bit-identical outputs,
i.e. the reference experiment with the MI355X aggregator produces exactly the same models.
The Substra client/opener layer is replaced by an in-memory ``preload_data`` (no Substra backend
here); ``substra``/``substratools`` are permissive import stubs.  Run:
    python tests/golden/gen_plumbing.py
"""

from __future__ import annotations

import json
import sys
import tempfile
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True  # never write into /root/reference
sys.path.insert(0, str(Path(__file__).resolve().parent))
from gen_golden import REF, _install_stubs  # noqa: E402

OUT = Path(__file__).resolve().parent
RECORD = []


def linear_data(n_col=3, n_samples=11, weights_seed=42, noise_seed=12):
    """tests/assets_factory.py:149-173 (restated: same NumPy calls and seeds)."""
    np.random.seed(weights_seed)
    random_content = np.random.uniform(0, 1, (n_samples, n_col - 1))
    np.random.seed(noise_seed)
    noise = np.random.normal(0, 0.01, (n_samples, n_col - 1))
    target = (random_content + noise).sum(axis=1)
    return np.c_[random_content, target]


def main():
    if not REF.exists():
        raise SystemExit("gen_plumbing.py needs /root/reference (build container only)")
    _install_stubs()
    import types

    sys.modules["substra"].BackendType = types.SimpleNamespace(REMOTE="remote", LOCAL_SUBPROCESS="subprocess",
                                                               LOCAL_DOCKER="docker")
    sys.path.insert(0, str(REF))
    import torch

    import substrafl.nodes.test_data_node as tdn
    import substrafl.nodes.train_data_node as trn
    from substrafl import simulate_experiment
    from substrafl.algorithms.pytorch import TorchFedAvgAlgo, TorchScaffoldAlgo
    from substrafl.evaluation_strategy import EvaluationStrategy
    from substrafl.index_generator import NpIndexGenerator
    from substrafl.nodes import AggregationNode, TestDataNode, TrainDataNode
    from substrafl.remote import remote
    from substrafl.strategies import FedAvg, Scaffold

    DATA = {}

    def fake_preload(client, data_manager_key, data_sample_keys):
        return DATA[data_sample_keys[0]]

    trn.preload_data = fake_preload
    tdn.preload_data = fake_preload

    class Client:
        backend_mode = "subprocess"

    class RecFedAvg(FedAvg):
        @remote
        def avg_shared_states(self, shared_states):
            out = FedAvg.avg_shared_states(self, shared_states=shared_states, _skip=True)
            RECORD.append(("fedavg", None, shared_states, out))
            return out

    class RecScaffold(Scaffold):
        @remote
        def avg_shared_states(self, shared_states):
            out = Scaffold.avg_shared_states(self, shared_states=shared_states, _skip=True)
            RECORD.append(("scaffold", self._aggregation_lr, shared_states, out))
            return out

    class TorchDataset(torch.utils.data.Dataset):  # tests/conftest.py:424-441
        def __init__(self, data_from_opener, is_inference=False):
            self.x = data_from_opener[0]
            self.y = data_from_opener[1]
            self.is_inference = is_inference

        def __getitem__(self, index):
            x = torch.from_numpy(self.x[index]).float()
            if not self.is_inference:
                y = torch.as_tensor(self.y[index])
                y = y.float() if y.dtype.is_floating_point else y.long()
                return x, y
            return x

        def __len__(self):
            return len(self.x)

    def mae_score(data_from_opener, predictions):  # tests/conftest.py:133-144
        return abs(np.array(predictions) - data_from_opener[1]).mean()

    def acc_score(data_from_opener, predictions):
        return float((np.array(predictions).argmax(axis=1) == data_from_opener[1]).mean())

    arrays, meta = {}, {"numpy": np.__version__, "torch": torch.__version__, "configs": {}}

    def run(name, strategy_cls, algo_base, model, criterion, data_train, data_test, metric, rounds, lr=0.1,
            updates=100, batch=32, strategy_kwargs=None, algo_kwargs=None):
        DATA.clear()
        for i, d in enumerate(data_train):
            DATA[f"train{i}"] = d
        DATA["test0"] = data_test
        nig = NpIndexGenerator(batch_size=batch, num_updates=updates)

        class MyAlgo(algo_base):
            def __init__(self):
                super().__init__(optimizer=torch.optim.SGD(model.parameters(), lr=lr), criterion=criterion,
                                 model=model, index_generator=nig, dataset=TorchDataset, **(algo_kwargs or {}))

        train_nodes = [TrainDataNode(f"org{i}", "ds", [f"train{i}"]) for i in range(len(data_train))]
        test_nodes = [TestDataNode("org0", "ds", ["test0"])]
        strategy = strategy_cls(algo=MyAlgo(), metric_functions=metric, **(strategy_kwargs or {}))
        RECORD.clear()
        perf, _, _ = simulate_experiment(
            client=Client(),
            strategy=strategy,
            train_data_nodes=train_nodes,
            evaluation_strategy=EvaluationStrategy(test_data_nodes=test_nodes, eval_rounds=[0, rounds]),
            aggregation_node=AggregationNode("org0"),
            num_rounds=rounds,
            clean_models=True,
            experiment_folder=tempfile.mkdtemp(),
        )
        final = float(perf.performance[-1])
        calls = []
        for ci, (kind, alr, states, out) in enumerate(RECORD):
            key = f"{name}/call{ci}"
            arrays[f"{key}/n_samples"] = np.array([s.n_samples for s in states], dtype=np.int64)
            L = len(states[0].parameters_update)
            for k, s in enumerate(states):
                for li in range(L):
                    arrays[f"{key}/k{k}/pu{li}"] = s.parameters_update[li]
                    if kind == "scaffold":
                        arrays[f"{key}/k{k}/cv{li}"] = s.control_variate_update[li]
                        arrays[f"{key}/k{k}/c{li}"] = s.server_control_variate[li]
            for li in range(L):
                arrays[f"{key}/out_avg{li}"] = out.avg_parameters_update[li]
                if kind == "scaffold":
                    arrays[f"{key}/out_c{li}"] = out.server_control_variate[li]
            calls.append({"key": key, "K": len(states), "layers": L, "kind": kind, "aggregation_lr": alr,
                          "shapes": [list(a.shape) for a in states[0].parameters_update],
                          "dtypes": [str(a.dtype) for a in states[0].parameters_update]})
        meta["configs"][name] = {"calls": calls, "final_performance": final, "rounds": rounds}
        print(f"{name}: {len(calls)} aggregations, final performance {final!r}")
        return final

    # --- the reference's own linear known answer (FedAvg, then Scaffold) ---
    train = [linear_data(n_col=3, n_samples=1024, weights_seed=42, noise_seed=i) for i in range(2)]
    test = linear_data(n_col=3, n_samples=64, weights_seed=42, noise_seed=42)
    split = lambda d: (d[:, :-1], d[:, -1:])  # noqa: E731  (the NumpyOpener, assets_factory.py:23-31)

    class Perceptron(torch.nn.Module):  # tests/conftest.py:322-341
        def __init__(self):
            super().__init__()
            self.linear1 = torch.nn.Linear(2, 1)

        def forward(self, x):
            return self.linear1(x)

    torch.manual_seed(42)
    perf = run("linear_fedavg", RecFedAvg, TorchFedAvgAlgo, Perceptron(), torch.nn.MSELoss(),
               [split(d) for d in train], split(test), mae_score, rounds=3)
    assert abs(perf - 0.0127768361) <= 1e-5 * 0.0127768361, perf  # test_fed_avg.py:25
    torch.manual_seed(42)
    perf = run("linear_scaffold", RecScaffold, TorchScaffoldAlgo, Perceptron(), torch.nn.MSELoss(),
               [split(d) for d in train], split(test), mae_score, rounds=3)
    assert abs(perf - 0.0127768706) <= 1e-5 * 0.0127768706, perf  # test_scaffold.py:26

    # --- MNIST-shaped synthetic FedAvg (conv + BatchNorm running stats + linear) ---
    g = np.random.default_rng(2024)
    mk = lambda n: (g.standard_normal((n, 1, 28, 28)).astype(np.float32), g.integers(0, 10, n))  # noqa: E731

    class SmallCNN(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = torch.nn.Conv2d(1, 8, 3)
            self.bn = torch.nn.BatchNorm2d(8)
            self.fc = torch.nn.Linear(8 * 13 * 13, 10)

        def forward(self, x):
            x = torch.nn.functional.max_pool2d(torch.relu(self.bn(self.conv(x))), 2)
            return self.fc(x.flatten(1))

    torch.manual_seed(7)
    run("mnist_fedavg", RecFedAvg, TorchFedAvgAlgo, SmallCNN(), torch.nn.CrossEntropyLoss(),
        [mk(256), mk(192)], mk(64), acc_score, rounds=2, lr=0.05, updates=8, batch=32,
        algo_kwargs={"with_batch_norm_parameters": True})

    np.savez_compressed(OUT / "golden_plumbing.npz", **arrays)
    (OUT / "golden_plumbing_meta.json").write_text(json.dumps(meta, indent=1))
    print(f"wrote {len(arrays)} arrays ({sum(a.nbytes for a in arrays.values()) / 1e6:.2f} MB raw)")


if __name__ == "__main__":
    main()
