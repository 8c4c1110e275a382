"""Client-side cost of one federated round's ``train`` (VERDICT r04 "Next 1"): the reference's
``TorchFedAvgAlgo.train`` / ``TorchScaffoldAlgo.train`` sequence in per-layer torch ops (the
builder-written stand-ins of tests/standin_substrafl) against ``accelerate_algo`` of the same
class, on a model of --params parameters in --layers Linear layers, with ONE optimizer step per
round (so the weight moves -- apply the average, snapshot, delta, reset, export -- are what is
timed, not the training).  Both start from the same weights and see the same data; every
exported update is compared bit for bit.  One JSON line per (strategy, path).

    python3 tools/accelerate_algo_bench.py --params 25000000 --layers 24 --rounds 5
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--strategies", default="fedavg,scaffold")
    ap.add_argument("--breakdown", action="store_true",
                    help="also time each weight_manager call of the accelerated train (synchronised "
                         "before and after: the total then includes those syncs)")
    args = ap.parse_args()

    import torch

    from standin_substrafl.algorithms.pytorch import TorchFedAvgAlgo, TorchScaffoldAlgo
    from standin_substrafl.index_generator import NpIndexGenerator
    from substrafl_amd.integration import accelerate_algo

    torch.backends.cudnn.enabled = False
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    width = int((args.params / args.layers) ** 0.5)

    class DS(torch.utils.data.Dataset):
        def __init__(self, data_from_opener, is_inference=False):
            self.x, self.y = data_from_opener

        def __getitem__(self, i):
            return torch.from_numpy(self.x[i]), torch.from_numpy(self.y[i])

        def __len__(self):
            return len(self.x)

    rng = np.random.default_rng(0)
    data = (rng.standard_normal((64, width)).astype(np.float32), rng.standard_normal((64, width)).astype(np.float32))

    def make(base, accelerated):
        torch.manual_seed(3)
        model = torch.nn.Sequential(*[torch.nn.Linear(width, width) for _ in range(args.layers)])

        class Algo(base):
            def __init__(self):
                super().__init__(model=model, criterion=torch.nn.MSELoss(),
                                 optimizer=torch.optim.SGD(model.parameters(), lr=1e-3),
                                 index_generator=NpIndexGenerator(batch_size=8, num_updates=1, seed=5), dataset=DS)

        return (accelerate_algo(Algo) if accelerated else Algo)()

    phases: dict = {}
    if args.breakdown:
        import functools

        from substrafl_amd.algorithms import weight_manager as wm

        def timed(name, fn):
            @functools.wraps(fn)
            def inner(*a, **k):
                sync()
                t = time.perf_counter()
                try:
                    return fn(*a, **k)
                finally:
                    sync()
                    phases.setdefault(name, []).append(time.perf_counter() - t)
            return inner

        for name in ("increment_parameters", "to_device", "get_parameters", "subtract_parameters",
                     "weighted_sum_parameters", "add_parameters", "set_parameters", "export_numpy"):
            setattr(wm, name, timed(name, getattr(wm, name)))

    params = sum(p.numel() for p in make(TorchFedAvgAlgo, False).model.parameters())
    for strat in args.strategies.split(","):
        base = TorchScaffoldAlgo if strat == "scaffold" else TorchFedAvgAlgo
        results, exports = {}, {}
        for path in ("reference_torch_loops", "accelerate_algo"):
            algo = make(base, path == "accelerate_algo")
            times, shared, outs = [], None, []
            for r in range(args.rounds + 1):
                if r == 1:
                    phases.clear()
                sync()
                t0 = time.perf_counter()
                st = algo.train(data_from_opener=data, shared_state=shared, _skip=True)
                sync()
                if r:  # round 0 pays the allocations and the code objects
                    times.append(time.perf_counter() - t0)
                outs.append([np.array(a, copy=True) for a in st.parameters_update])
                # the "average" of one client is its own update (the aggregation is not timed here)
                if strat == "scaffold":
                    from standin_substrafl.strategies.schemas import ScaffoldAveragedStates

                    shared = ScaffoldAveragedStates(avg_parameters_update=[a.astype(np.float64) for a in outs[-1]],
                                                    server_control_variate=[np.asarray(a, np.float64)
                                                                            for a in st.control_variate_update])
                else:
                    from standin_substrafl.strategies.schemas import FedAvgAveragedState

                    shared = FedAvgAveragedState(avg_parameters_update=outs[-1])
            results[path] = times
            exports[path] = outs
            if phases and path == "accelerate_algo":
                print(json.dumps({"strategy": strat, "path": path, "breakdown_ms_per_round": {
                    k: round(1e3 * sum(v) / len(times), 2) for k, v in phases.items()},
                    "calls_per_round": {k: len(v) / len(times) for k, v in phases.items()}}), flush=True)
            phases.clear()
        same = all(np.array_equal(a.view(np.uint32), b.view(np.uint32))
                   for ra, rb in zip(exports["reference_torch_loops"], exports["accelerate_algo"]) for a, b in zip(ra, rb))
        for path, times in results.items():
            print(json.dumps({"strategy": strat, "path": path, "params": params, "layers": args.layers,
                              "optimizer_steps_per_round": 1, "rounds_timed": len(times),
                              "train_ms_median": round(1e3 * float(np.median(times)), 2),
                              "train_ms_min": round(1e3 * float(np.min(times)), 2),
                              "train_ms_rounds": [round(1e3 * t, 2) for t in times],
                              "exports_bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()
