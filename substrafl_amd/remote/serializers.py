"""Shared-state wire format: one pickle file per state (serializers/pickle_serializer.py:8-33).

Files written here are read back only by this process family (our own outputs); a pickle is
never the format for untrusted inputs in tests.
"""

import pickle
from pathlib import Path
from typing import Any


class PickleSerializer:
    @staticmethod
    def save(state: Any, path: Path) -> None:
        with Path(path).open("wb") as f:
            pickle.dump(state, f)

    @staticmethod
    def load(path: Path) -> Any:
        with Path(path).open("rb") as f:
            return pickle.load(f)
