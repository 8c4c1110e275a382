#!/usr/bin/env python3
"""Subprocess-mode aggregate task, timed as Substra runs it: a FRESH Python process
per task that unpickles K shared-state files, aggregates and pickles the result.

  parent: writes K reference-format pickles once, then runs --reps fresh children per mode and
          prints one JSON line per child (wall time of the whole child, measured by the parent).
  child --mode engine:    substrafl_amd's RemoteMethod.generic_function (prewarm + threaded load +
                          GPU engine), exactly the drop-in task path.
  child --mode engine-noprewarm: same, with the prewarm hook disabled.
  child --mode engine-copyload: same, loading with pickle.load instead of the mapped loader.
  child --mode numpy:     the reference's own sequence (sequential pickle.load, NumPy FedAvg in the
                          reference call structure from oracle/, pickle.dump) -- the CPU baseline.
  --strategy scaffold: ScaffoldSharedState files, each carrying its own pickled copy of the server
                          control variate (as K clients send it); child --mode engine-devcheck stages
                          all K copies and checks them on the GPU (the round-1 path) where the default
                          engine stages one copy and checks the others on the host.
"""

import argparse
import json
import os
import pickle
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def np_testing_assert_array_equal(a, b):
    import numpy as np

    np.testing.assert_array_equal(a, b)


def child(mode: str, d: Path, K: int, strategy_name: str = "fedavg") -> None:
    t0 = time.perf_counter()
    paths = [d / f"shared_{k}" for k in range(K)]
    out = d / f"out_{mode}"
    if mode == "engine-devcheck":
        os.environ["FEDAGG_C_CHECK"] = "device"
    if mode == "numpy" and strategy_name == "scaffold":
        from oracle import scaffold_reference_structure
        from substrafl_amd.schemas import ScaffoldAveragedStates

        states = []
        t1 = time.perf_counter()
        for p in paths:
            with open(p, "rb") as f:
                states.append(pickle.load(f))
        t1b = time.perf_counter()
        c0 = states[0].server_control_variate
        for s_ in states[1:]:  # scaffold.py:193-196
            for a_, b_ in zip(c0, s_.server_control_variate):
                np_testing_assert_array_equal(a_, b_)
        new_c, avg = scaffold_reference_structure([s_.parameters_update for s_ in states],
                                                  [s_.control_variate_update for s_ in states], c0,
                                                  [s_.n_samples for s_ in states], 1.0)
        t2 = time.perf_counter()
        with open(out, "wb") as f:
            pickle.dump(ScaffoldAveragedStates(server_control_variate=new_c, avg_parameters_update=avg), f)
        t3 = time.perf_counter()
    elif mode == "numpy":
        from oracle import fedavg_reference_structure
        from substrafl_amd.schemas import FedAvgAveragedState

        states = []
        t1 = time.perf_counter()
        for p in paths:
            with open(p, "rb") as f:
                states.append(pickle.load(f))
        t1b = time.perf_counter()
        avg = fedavg_reference_structure([s.parameters_update for s in states], [s.n_samples for s in states])
        t2 = time.perf_counter()
        with open(out, "wb") as f:
            pickle.dump(FedAvgAveragedState(avg_parameters_update=avg), f)
        t3 = time.perf_counter()
    else:
        # RemoteMethod.generic_function's steps, timed one by one
        from substrafl_amd import runtime
        from substrafl_amd.engine import default_engine
        from substrafl_amd.remote.substratools_methods import RemoteMethod
        from substrafl_amd.strategies import FedAvg, Scaffold

        class _Algo:
            strategies = ["Federated Averaging", "Scaffold"]

        strategy = Scaffold(algo=_Algo()) if strategy_name == "scaffold" else FedAvg(algo=_Algo())
        if mode == "engine-noprewarm":
            strategy.prewarm_aggregation = None
        if mode == "engine-copyload":  # pickle.load instead of the mapped loader
            os.environ["FEDAGG_MAPPED_LOAD"] = "0"
        t1 = time.perf_counter()
        rm = RemoteMethod(strategy, "avg_shared_states", {})
        rm.register_substratools_function()  # function.py's next step: starts the prewarm
        ta = time.perf_counter()
        inputs = rm.load_method_inputs({"shared": paths}, {})
        tb = time.perf_counter()
        res = strategy.avg_shared_states(**inputs, _skip=True)
        tc = time.perf_counter()
        rm.save_method_output(res, {"shared": out})
        t2 = t3 = time.perf_counter()
        phases = {"load_s": round(tb - ta, 4), "aggregate_s": round(tc - tb, 4), "save_s": round(t2 - tc, 4),
                  "engine": {k: (round(v, 4) if isinstance(v, float) else v)
                             for k, v in default_engine().last_timing.items()}}
        if 0 in runtime.warm_times:
            w0, w1 = runtime.warm_times[0]
            phases["prewarm_s"] = round(w1 - w0, 4)
            phases["prewarm_done_after_load_s"] = round(w1 - tb, 4)
            phases["prewarm_started_after_setup_s"] = round(w0 - t1, 4)
            # where the prewarm's time went (VERDICT r05 "Next 4"): library load, HIP runtime start,
            # streams, pinned ring, worker pool, HBM buffers, code-object load
            phases["prewarm_phases"] = runtime.warm_phases.get(0)
    line = {"child": mode, "strategy": strategy_name, "in_child_total_s": round(t3 - t0, 4), "setup_s": round(t1 - t0, 4),
            "task_s": round(t3 - t1, 4)}
    if mode == "numpy":
        phases = {"load_s": round(t1b - t1, 4), "aggregate_s": round(t2 - t1b, 4), "save_s": round(t3 - t2, 4)}
    line.update(phases)
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=8)
    ap.add_argument("--M", type=int, default=25_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--child", default=None)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--strategy", default="fedavg", choices=["fedavg", "scaffold"])
    args = ap.parse_args()
    if args.child:
        return child(args.child, Path(args.dir), args.K, args.strategy)

    import numpy as np

    from substrafl_amd.layout import synthetic_state_dict_shapes
    from substrafl_amd.schemas import FedAvgSharedState, ScaffoldSharedState

    d = Path(tempfile.mkdtemp(prefix="task_", dir=os.environ.get("TMPDIR", "/tmp")))
    rng = np.random.default_rng(0)
    ns = [int(v) for v in np.random.default_rng(7).integers(100, 10000, args.K)]
    shapes = synthetic_state_dict_shapes(args.M)
    c = [rng.standard_normal(s, dtype=np.float32) for s in shapes]
    for k in range(args.K):
        pu = [rng.standard_normal(s, dtype=np.float32) for s in shapes]
        if args.strategy == "scaffold":
            st = ScaffoldSharedState(parameters_update=pu, n_samples=ns[k], server_control_variate=c,
                                     control_variate_update=[rng.standard_normal(s, dtype=np.float32) for s in shapes])
        else:
            st = FedAvgSharedState(n_samples=ns[k], parameters_update=pu)
        with open(d / f"shared_{k}", "wb") as f:
            pickle.dump(st, f)
    modes = ("numpy", "engine", "engine-devcheck") if args.strategy == "scaffold" else \
        ("numpy", "engine", "engine-noprewarm", "engine-copyload")
    for rep in range(args.reps):
        for mode in modes:
            t0 = time.perf_counter()
            r = subprocess.run([sys.executable, __file__, "--child", mode, "--dir", str(d), "--K", str(args.K),
                                "--strategy", args.strategy], capture_output=True, text=True, timeout=600)
            wall = time.perf_counter() - t0
            if r.returncode != 0:
                print(r.stdout, r.stderr, file=sys.stderr)
                raise SystemExit(r.returncode)
            line = json.loads(r.stdout.strip().splitlines()[-1])
            line.update(K=args.K, M=args.M, rep=rep, process_wall_s=round(wall, 4))
            print(json.dumps(line), flush=True)
    ra, rb = pickle.load(open(d / "out_numpy", "rb")), pickle.load(open(d / "out_engine", "rb"))
    a, b = ra.avg_parameters_update, rb.avg_parameters_update
    if args.strategy == "scaffold":
        a, b = a + ra.server_control_variate, b + rb.server_control_variate
    same = all(np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8)) for x, y in zip(a, b))
    print(json.dumps({"bit_exact_engine_vs_numpy": bool(same)}), flush=True)
    for p in d.iterdir():
        p.unlink()
    d.rmdir()


if __name__ == "__main__":
    main()
