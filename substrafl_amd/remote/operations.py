"""Deferred operations returned by ``@remote`` methods (substrafl/remote/operations.py:13-27)."""

from dataclasses import dataclass
from typing import Any, List, Optional

from .remote_struct import RemoteStruct


@dataclass
class RemoteOperation:
    """Aggregation operation: what to run (``remote_struct``) on which shared states."""

    remote_struct: RemoteStruct
    shared_states: Optional[List]


@dataclass
class RemoteDataOperation:
    """Data operation (train / predict on an organisation's data samples)."""

    remote_struct: RemoteStruct
    data_samples: List[str]
    shared_state: Any
