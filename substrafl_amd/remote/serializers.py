"""Shared-state wire format: one pickle file per state (serializers/pickle_serializer.py:8-33).

Files written here are read back only by this process family (our own outputs); a pickle is
never the format for untrusted inputs in tests.
"""

import os
import pickle
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Any, List, Sequence


class PickleSerializer:
    @staticmethod
    def save(state: Any, path: Path) -> None:
        """pickle_serializer.py:10-18, with protocol 5: NumPy arrays and wire buckets are then
        written straight from their buffers (protocol 4 copies each one with ``tobytes`` first:
        100 MB in 33 ms instead of 133 ms in this container).  Any Python >= 3.8 reads it."""
        with Path(path).open("wb") as f:
            pickle.dump(state, f, protocol=5)

    @staticmethod
    def load(path: Path) -> Any:
        with Path(path).open("rb") as f:
            return pickle.load(f)

    @staticmethod
    def load_mapped(path: Path) -> Any:
        """``load`` with the NumPy array payloads left in a private mapping of the file (no copy,
        no fresh pages: mapped_pickle.py); used by the aggregate task's ingest, whose inputs are
        read-only task inputs.  Same objects as ``load``."""
        if os.environ.get("FEDAGG_MAPPED_LOAD", "1") == "0":  # measurement switch: the copying load
            return PickleSerializer.load(path)
        from .mapped_pickle import load_mapped

        return load_mapped(path)

    @staticmethod
    def load_many(paths: Sequence[Path], max_workers: int = 0) -> List[Any]:
        """``[load(p) for p in paths]`` with the K file reads overlapped on a thread pool (the
        read syscalls, where page faulting of the fresh buffers happens, release the GIL).
        Same objects, same order; the first failing path's exception is raised, as in the
        reference's sequential loop (substratools_methods.py:61-64)."""
        paths = list(paths)
        workers = max_workers or min(len(paths), 16, os.cpu_count() or 1)
        if workers <= 1 or len(paths) <= 1:
            return [PickleSerializer.load(p) for p in paths]
        with ThreadPoolExecutor(workers) as ex:
            futures = [ex.submit(PickleSerializer.load, p) for p in paths]
            return [f.result() for f in futures]
