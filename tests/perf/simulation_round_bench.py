"""One federated round of simulation mode, end to end in one process on one GPU: K clients'
``train`` (one optimizer step each, so the weight moves and the aggregation are what is timed)
and the aggregation of their states, as ``simulate_experiment`` runs them
(nodes/train_data_node.py:336-382, nodes/aggregation_node.py:197-227).  Three paths on the same
model, data and seeds:

* ``reference``: the builder-written stand-ins of ``TorchFedAvgAlgo`` / ``TorchScaffoldAlgo``
  (the reference's torch ops) and the reference's NumPy aggregation (oracle: the same calls as
  fed_avg.py:217-222 / scaffold.py:204-337) -- the reference's own path;
* ``accelerated``: ``accelerate_algo`` clients and an ``accelerate``d strategy (host arrays
  between them, staged over PCIe both ways);
* ``handoff``: the same with the simulation-mode device hand-off (substrafl_amd/handoff.py): the
  exports reach the aggregator, and the average the clients, device to device.

Every round's average is compared bit for bit across the paths.  One JSON line per path.

    python3 tests/perf/simulation_round_bench.py --strategy fedavg --clients 8 --params 25000000 --rounds 5
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
    ap.add_argument("--strategy", default="fedavg", choices=["fedavg", "scaffold"])
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--paths", default="reference,accelerated,handoff")
    args = ap.parse_args()

    import torch

    import standin_substrafl.strategies as ss
    from oracle import fedavg_reference_structure, scaffold_reference_structure
    from standin_substrafl.algorithms.pytorch import TorchFedAvgAlgo, TorchScaffoldAlgo
    from standin_substrafl.index_generator import NpIndexGenerator
    from standin_substrafl.strategies import schemas as sch
    from substrafl_amd import handoff
    from substrafl_amd.integration import accelerate, accelerate_algo

    torch.backends.cudnn.enabled = False
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    width = int((args.params / args.layers) ** 0.5)
    scaffold = args.strategy == "scaffold"
    base_cls = TorchScaffoldAlgo if scaffold else TorchFedAvgAlgo

    class DS(torch.utils.data.Dataset):
        def __init__(self, data_from_opener, is_inference=False):
            self.x, self.y = data_from_opener

        def __getitem__(self, i):
            return torch.from_numpy(self.x[i]), torch.from_numpy(self.y[i])

        def __len__(self):
            return len(self.x)

    rng = np.random.default_rng(0)
    data = [(rng.standard_normal((32 + 8 * k, width)).astype(np.float32),
             rng.standard_normal((32 + 8 * k, width)).astype(np.float32)) for k in range(args.clients)]

    def make(k, accelerated):
        torch.manual_seed(3)  # every client starts from the same weights
        model = torch.nn.Sequential(*[torch.nn.Linear(width, width) for _ in range(args.layers)])

        class Algo(base_cls):
            def __init__(self):
                super().__init__(model=model, criterion=torch.nn.MSELoss(),
                                 optimizer=torch.optim.SGD(model.parameters(), lr=1e-3 * (1 + 0.1 * k)),
                                 index_generator=NpIndexGenerator(batch_size=8, num_updates=1, seed=5 + k),
                                 dataset=DS)

        return (accelerate_algo(Algo) if accelerated else Algo)()

    params = None
    averages, results = {}, []
    for path in args.paths.split(","):
        handoff.enable(path == "handoff")
        algos = [make(k, path != "reference") for k in range(args.clients)]
        params = sum(p.numel() for p in algos[0].model.parameters())
        if path == "reference":
            strategy = None
        elif scaffold:
            strategy = accelerate(ss.Scaffold)(algo=algos[0], aggregation_lr=1.0)
        else:
            strategy = accelerate(ss.FedAvg)(algo=algos[0])
        avg, prev, times, train_t, agg_t, avgs = None, None, [], [], [], []
        taken0 = handoff.stats["taken"]
        for r in range(args.rounds + 1):
            sync()
            t0 = time.perf_counter()
            states = [a.train(data_from_opener=d, shared_state=avg, _skip=True) for a, d in zip(algos, data)]
            sync()
            t1 = time.perf_counter()
            if strategy is not None:
                avg = strategy.avg_shared_states(shared_states=states, _skip=True)
            elif scaffold:
                new_c, upd = scaffold_reference_structure([list(s.parameters_update) for s in states],
                                                          [list(s.control_variate_update) for s in states],
                                                          list(states[0].server_control_variate),
                                                          [s.n_samples for s in states], 1.0)
                avg = sch.ScaffoldAveragedStates(server_control_variate=new_c, avg_parameters_update=upd)
            else:
                avg = sch.FedAvgAveragedState(avg_parameters_update=fedavg_reference_structure(
                    [list(s.parameters_update) for s in states], [s.n_samples for s in states]))
            sync()
            t2 = time.perf_counter()
            prev = states  # the strategy keeps the last train states until the next ones return
            if r:  # round 0 pays the allocations and the code objects
                times.append(t2 - t0)
                train_t.append(t1 - t0)
                agg_t.append(t2 - t1)
            avgs.append(np.concatenate([np.asarray(a, np.float64).reshape(-1)[:4096] for a in avg.avg_parameters_update]))
        del prev
        averages[path] = avgs
        results.append({"strategy": args.strategy, "path": path, "clients": args.clients, "params": params,
                        "layers": args.layers, "optimizer_steps_per_round": 1, "rounds_timed": len(times),
                        "round_ms_median": round(1e3 * float(np.median(times)), 2),
                        "round_ms_min": round(1e3 * float(np.min(times)), 2),
                        "train_ms_median_all_clients": round(1e3 * float(np.median(train_t)), 2),
                        "aggregate_ms_median": round(1e3 * float(np.median(agg_t)), 2),
                        "handoff_taken": handoff.stats["taken"] - taken0})
        del algos, strategy, avg, states
        handoff.enable(False)
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    ref = averages.get("reference")
    for res in results:
        if ref is not None:
            res["averages_bit_identical_to_reference"] = all(
                np.array_equal(a.view(np.uint64), b.view(np.uint64)) for a, b in zip(averages[res["path"]], ref))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
