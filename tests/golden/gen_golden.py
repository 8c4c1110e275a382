"""Generate golden vectors by running the REFERENCE aggregation code itself.

CONTAINER-ONLY: this script imports ``/root/reference`` (SubstraFL v1.0.0 source) and
refuses to run when it is absent, so it never runs on the GPU box.  Its outputs are
small ``.npz`` fixtures committed next to it; the tests read only those.

What it calls (with ``_skip=True``, exactly like ``RemoteMethod.generic_function``,
substrafl/remote/substratools_methods.py:109-116):
  * ``substrafl.strategies.FedAvg.avg_shared_states``   (fed_avg.py:176-224)
  * ``substrafl.strategies.Scaffold.avg_shared_states`` (scaffold.py:297-337)

``substra`` / ``substratools`` (pinned ``~=1.0.0`` in pyproject.toml:24-25) are not
installed and there is no network, so a permissive module stub stands in for them;
they are only needed for module-level imports, never for the arithmetic (which is
NumPy's).  Run:  python tests/golden/gen_golden.py
"""

from __future__ import annotations

import json
import sys
import types
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True  # never write into /root/reference

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent


def _install_stubs():
    class _Stub(types.ModuleType):
        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(name)
            cls = type(name, (), {"__init__": lambda self, *a, **k: None})
            setattr(self, name, cls)
            return cls

    for name in [
        "substra",
        "substra.sdk",
        "substra.sdk.schemas",
        "substra.sdk.models",
        "substra.sdk.client",
        "substra.schemas",
        "substra.models",
        "substratools",
        "docker",
    ]:
        mod = _Stub(name)
        mod.__version__ = "1.0.0-stub"
        mod.__path__ = []
        sys.modules[name] = mod
    for name in list(sys.modules):
        if "." in name and name.split(".")[0] in ("substra",):
            parent, child = name.rsplit(".", 1)
            setattr(sys.modules[parent], child, sys.modules[name])


def _import_reference():
    if not REF.exists():
        raise SystemExit("gen_golden.py needs /root/reference (build container only)")
    _install_stubs()
    sys.path.insert(0, str(REF))
    from substrafl.algorithms.algo import Algo
    from substrafl.remote.decorators import remote_data
    from substrafl.strategies import FedAvg, FedPCA, Scaffold
    from substrafl.strategies.schemas import FedAvgSharedState, FedPCASharedState, ScaffoldSharedState, StrategyName

    class DummyAlgo(Algo):  # tests/conftest.py:395-421 (compatible with every strategy)
        @property
        def strategies(self):
            return list(StrategyName)

        @property
        def model(self):
            return "model"

        @remote_data
        def train(self, data_from_opener, shared_state):
            return None

        def predict(self, data_from_opener, shared_state):
            return None

        def load_local_state(self, path):
            return self

        def save_local_state(self, path):
            pass

    globals()["_FEDPCA"] = (FedPCA, FedPCASharedState)
    return FedAvg, Scaffold, FedAvgSharedState, ScaffoldSharedState, DummyAlgo


def _layers(rng, shapes, kind, k):
    out = []
    for s in shapes:
        x = rng.standard_normal(s).astype(np.float32)
        if kind == "scaled":
            x = (x * np.float32(10.0 ** rng.integers(-3, 3))).astype(np.float32)
        elif kind == "cancel":  # G2: alternating-sign large magnitudes
            x = (x + np.float32(1e4 * (-1) ** k)).astype(np.float32)
        elif kind == "bf16":  # G4: bf16-representable fp32 (exact upcast of bf16)
            x = (x.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32)
        elif kind == "signedzero":  # G8: -0.0 / +0.0 columns, zero-sample clients
            x = np.where(rng.random(s) < 0.5, np.float32(-0.0), x).astype(np.float32)
            if k % 2:
                x = np.where(rng.random(s) < 0.5, np.float32(0.0), x).astype(np.float32)
        out.append(np.ascontiguousarray(x))
    return out


LAYER_SETS = {
    "a": [(3, 5)],
    "b": [(64, 33), (33,), (1,)],
    "c": [(5, 1), (2, 1, 3), (1, 1)],
    "d": [(4096,)],
}


def main():
    FedAvg, Scaffold, FedAvgSharedState, ScaffoldSharedState, DummyAlgo = _import_reference()
    meta = {"numpy": np.__version__, "reference": "Substra/substrafl v1.0.0 @ 2024-10-16", "cases": []}

    # ---------------- G1 / G2 / G4: FedAvg ----------------
    fedavg_cases = []
    for K in (1, 2, 3, 7, 8, 9, 16, 64, 130):
        for ls in ("a", "b", "c", "d"):
            if K >= 64 and ls == "d":
                continue
            fedavg_cases.append(("scaled", K, ls))
    for K in (2, 9, 64):
        fedavg_cases.append(("cancel", K, "b"))
    for K in (2, 8, 128):
        fedavg_cases.append(("bf16", K, "b"))
    for K in (1, 3, 12):
        fedavg_cases.append(("signedzero", K, "c"))

    strategy = FedAvg(algo=DummyAlgo())
    arrays = {}
    for ci, (kind, K, ls) in enumerate(fedavg_cases):
        rng = np.random.default_rng(20241016 + K + 1000 * ci)
        n_samples = [int(v) for v in np.random.default_rng(7 + K).integers(1, 5000, K)]
        if kind == "signedzero" and K > 1:
            n_samples[0] = 0
        shapes = LAYER_SETS[ls]
        clients = [_layers(rng, shapes, kind, k) for k in range(K)]
        states = [FedAvgSharedState(n_samples=n, parameters_update=c) for n, c in zip(n_samples, clients)]
        res = strategy.avg_shared_states(shared_states=states, _skip=True).avg_parameters_update
        key = f"fedavg_{ci:03d}"
        arrays[f"{key}/n_samples"] = np.array(n_samples, dtype=np.int64)
        for li in range(len(shapes)):
            arrays[f"{key}/x{li}"] = np.stack([c[li] for c in clients])
            arrays[f"{key}/out{li}"] = res[li]
        meta["cases"].append({"key": key, "strategy": "fedavg", "kind": kind, "K": K, "layers": len(shapes)})

    # ---------------- G3: Scaffold ----------------
    for ci, (K, lr) in enumerate([(1, 1), (2, 0.7), (4, 2), (16, 1), (16, 0), (4, 0.7)]):
        rng = np.random.default_rng(424242 + ci)
        shapes = [(3, 5), (1,), (7,), (1, 1)]
        n_samples = [int(v) for v in np.random.default_rng(11 + K).integers(1, 5000, K)]
        pu = [_layers(rng, shapes, "scaled", k) for k in range(K)]
        cv = [_layers(rng, shapes, "scaled", k) for k in range(K)]
        c = _layers(rng, shapes, "scaled", 0)
        states = [
            ScaffoldSharedState(
                parameters_update=pu[k], control_variate_update=cv[k], n_samples=n_samples[k], server_control_variate=c
            )
            for k in range(K)
        ]
        res = Scaffold(algo=DummyAlgo(), aggregation_lr=lr).avg_shared_states(shared_states=states, _skip=True)
        key = f"scaffold_{ci:03d}"
        arrays[f"{key}/n_samples"] = np.array(n_samples, dtype=np.int64)
        arrays[f"{key}/lr"] = np.array(lr, dtype=np.float64)
        for li in range(len(shapes)):
            arrays[f"{key}/pu{li}"] = np.stack([p[li] for p in pu])
            arrays[f"{key}/cv{li}"] = np.stack([p[li] for p in cv])
            arrays[f"{key}/c{li}"] = c[li]
            arrays[f"{key}/avg{li}"] = res.avg_parameters_update[li]
            arrays[f"{key}/newc{li}"] = res.server_control_variate[li]
        meta["cases"].append(
            {"key": key, "strategy": "scaffold", "K": K, "lr": lr, "lr_is_int": isinstance(lr, int), "layers": len(shapes)}
        )

    # ---------------- G9: FedPCA (fed_pca.py:210-299): plain average + QR variant ----------------
    FedPCA, FedPCASharedState = globals()["_FEDPCA"]
    pca = FedPCA(algo=DummyAlgo())
    for ci, K in enumerate((2, 5)):
        rng = np.random.default_rng(99 + K)
        shapes = [(4, 30), (3, 17)]  # (n_components, n_features): QR of the transpose
        ns = [int(v) for v in np.random.default_rng(5 + K).integers(1, 5000, K)]
        pcs = [[rng.standard_normal(sh).astype(np.float32) for sh in shapes] for _ in range(K)]
        states = [FedPCASharedState(n_samples=ns[k], parameters_update=pcs[k]) for k in range(K)]
        avg = pca.avg_shared_states(shared_states=states, _skip=True).avg_parameters_update
        qr = pca.avg_shared_states_with_qr(shared_states=states, _skip=True).avg_parameters_update
        key = f"fedpca_{ci:03d}"
        arrays[f"{key}/n_samples"] = np.array(ns, dtype=np.int64)
        for li in range(len(shapes)):
            arrays[f"{key}/x{li}"] = np.stack([c[li] for c in pcs])
            arrays[f"{key}/avg{li}"] = avg[li]
            arrays[f"{key}/qr{li}"] = qr[li]
        meta["cases"].append({"key": key, "strategy": "fedpca", "K": K, "layers": len(shapes)})

    # ---------------- G5: reference unit-test inputs verbatim ----------------
    # tests/strategies/test_fed_avg.py:17-38 (float64 ones/zeros) and :41-54 (int64 layers)
    g5 = {}
    for i, ns in enumerate(([1, 0, 0], [1, 1, 1], [1, 0, 1])):
        states = [
            FedAvgSharedState(parameters_update=[np.ones((5, 10))], n_samples=ns[0]),
            FedAvgSharedState(parameters_update=[np.zeros((5, 10))], n_samples=ns[1]),
            FedAvgSharedState(parameters_update=[2 * np.ones((5, 10))], n_samples=ns[2]),
        ]
        g5[f"unit_fedavg_{i}"] = strategy.avg_shared_states(shared_states=states, _skip=True).avg_parameters_update[0]
    states = [
        FedAvgSharedState(parameters_update=[np.asarray([[0, 1], [2, 4]]), np.asarray([[6, 8], [10, 12]])], n_samples=1),
        FedAvgSharedState(
            parameters_update=[np.asarray([[16, 20], [18, 20]]), np.asarray([[22, 24], [26, 28]])], n_samples=3
        ),
    ]
    r = strategy.avg_shared_states(shared_states=states, _skip=True).avg_parameters_update
    g5["unit_fedavg_int64_0"], g5["unit_fedavg_int64_1"] = r
    for k, v in g5.items():
        arrays[f"g5/{k}"] = v

    # ---------------- G6: error cases ----------------
    errors = {}

    def record(name, fn):
        try:
            fn()
            errors[name] = None
        except Exception as e:  # noqa: BLE001
            errors[name] = type(e).__name__

    record("fedavg_empty", lambda: strategy.avg_shared_states(shared_states=[], _skip=True))
    record(
        "fedavg_zero_samples",
        lambda: strategy.avg_shared_states(
            shared_states=[FedAvgSharedState(parameters_update=[np.ones(3, np.float32)], n_samples=0)] * 2, _skip=True
        ),
    )
    record(
        "fedavg_layer_count",
        lambda: strategy.avg_shared_states(
            shared_states=[
                FedAvgSharedState(parameters_update=[np.ones(3, np.float32)] * 2, n_samples=1),
                FedAvgSharedState(parameters_update=[np.ones(3, np.float32)], n_samples=1),
            ],
            _skip=True,
        ),
    )
    record(
        "fedavg_shape_mismatch",
        lambda: strategy.avg_shared_states(
            shared_states=[
                FedAvgSharedState(parameters_update=[np.ones(3, np.float32)], n_samples=1),
                FedAvgSharedState(parameters_update=[np.ones(4, np.float32)], n_samples=1),
            ],
            _skip=True,
        ),
    )
    record(
        "fedavg_0d",
        lambda: strategy.avg_shared_states(
            shared_states=[FedAvgSharedState(parameters_update=[np.float32(1.0) * np.ones((), np.float32)], n_samples=1)]
            * 2,
            _skip=True,
        ),
    )
    record("fedavg_float_n_samples", lambda: FedAvgSharedState(parameters_update=[np.ones(3)], n_samples=1.5))
    sc = Scaffold(algo=DummyAlgo(), aggregation_lr=1)
    record("scaffold_empty", lambda: sc.avg_shared_states(shared_states=[], _skip=True))
    cA = [np.ones(3, np.float32)]
    cB = [np.array([1, 1, 2], np.float32)]
    record(
        "scaffold_c_mismatch",
        lambda: sc.avg_shared_states(
            shared_states=[
                ScaffoldSharedState(parameters_update=cA, control_variate_update=cA, n_samples=1, server_control_variate=cA),
                ScaffoldSharedState(parameters_update=cA, control_variate_update=cA, n_samples=1, server_control_variate=cB),
            ],
            _skip=True,
        ),
    )
    record("scaffold_negative_lr", lambda: Scaffold(algo=DummyAlgo(), aggregation_lr=-1))
    meta["errors"] = errors

    np.savez_compressed(OUT / "golden_aggregation.npz", **arrays)
    (OUT / "golden_meta.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
    total = sum(v.nbytes for v in arrays.values())
    print(f"wrote {len(arrays)} arrays ({total / 1e6:.2f} MB raw), {len(meta['cases'])} cases, errors={errors}")


if __name__ == "__main__":
    main()
