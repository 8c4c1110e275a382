import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfedagg.so on the GPU)")
    config.addinivalue_line("markers", "tuning: an experiment launch variant; needs the FEDAGG_TUNING build "
                                       "(FEDAGG_LIB=substrafl_amd/libfedagg_tuning.so); deselected otherwise")


# fedagg_tune knobs the product library accepts; any other knob selects an experiment variant
# that only the FEDAGG_TUNING build instantiates (DESIGN.md §5 "Product and tuning builds")
PRODUCT_KNOBS = {"grid_cap", "fuse_pairwise", "eq_vec", "flat_vec", "st_sc1", "tiled_few", "sc_2l"}


def experiment_knobs(*knob_dicts) -> bool:
    keys = set().union(*[set(d) for d in knob_dicts])
    return bool(keys - PRODUCT_KNOBS - {"K"}) or any(d.get("sc_2l") == 2 for d in knob_dicts)


def tuning_requested() -> bool:
    return "tuning" in os.environ.get("FEDAGG_LIB", "") or os.environ.get("FEDAGG_TUNING_TESTS") == "1"


def pytest_collection_modifyitems(config, items):
    """Experiment-variant tests (a ``knobs`` parameter naming experiment knobs) are marked
    ``tuning`` and deselected unless the tuning build is loaded: the product library does not
    instantiate them, so they would only ever skip there."""
    keep, drop = [], []
    for it in items:
        knobs = getattr(getattr(it, "callspec", None), "params", {}).get("knobs")
        if isinstance(knobs, dict) and experiment_knobs(knobs):
            it.add_marker(pytest.mark.tuning)
            if not tuning_requested():
                drop.append(it)
                continue
        keep.append(it)
    if drop:
        config.hook.pytest_deselected(items=drop)
        items[:] = keep


class DummyAlgo:
    """Compatible with every strategy (reference tests/conftest.py:395-421)."""

    def __init__(self, *args, **kwargs):
        self.args = args
        self.kwargs = kwargs

    @property
    def strategies(self):
        from substrafl_amd.schemas import StrategyName

        return list(StrategyName)

    @property
    def model(self):
        return "model"


@pytest.fixture
def dummy_algo_class():
    return DummyAlgo


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    d = ROOT / "tests" / "golden"
    arrays = np.load(d / "golden_aggregation.npz", allow_pickle=False)
    meta = json.loads((d / "golden_meta.json").read_text())
    return arrays, meta
