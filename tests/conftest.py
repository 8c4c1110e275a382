import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfedagg.so on the GPU)")


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
