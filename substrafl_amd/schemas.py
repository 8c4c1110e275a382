"""Shared-state wire schemas, field-for-field the reference's (substrafl/strategies/schemas.py).

Same class names, field names, types and pydantic validation, so shared states pickled by a
reference client unpickle into these once the module path is aliased, and
a 0-d result fails validation exactly like the reference (``np.sum`` of 0-d arrays yields a
NumPy scalar, not an ``np.ndarray``).
"""

from enum import Enum
from typing import List

import numpy as np
import pydantic


class StrategyName(str, Enum):  # schemas.py:11-16
    FEDERATED_AVERAGING = "Federated Averaging"
    FEDERATED_PCA = "Federated PCA"
    SCAFFOLD = "Scaffold"
    SINGLE_ORGANIZATION = "Single organization"
    NEWTON_RAPHSON = "Newton Raphson"


class _Model(pydantic.BaseModel):  # schemas.py:19-22
    model_config = pydantic.ConfigDict(arbitrary_types_allowed=True)


class FedAvgAveragedState(_Model):  # schemas.py:25-29
    avg_parameters_update: List[np.ndarray]


class FedAvgSharedState(_Model):  # schemas.py:32-38
    n_samples: int
    parameters_update: List[np.ndarray]


class ScaffoldSharedState(_Model):  # schemas.py:57-74
    parameters_update: List[np.ndarray]
    control_variate_update: List[np.ndarray]
    n_samples: int
    server_control_variate: List[np.ndarray]


class ScaffoldAveragedStates(_Model):  # schemas.py:77-87
    server_control_variate: List[np.ndarray]
    avg_parameters_update: List[np.ndarray]


class FedPCAAveragedState(_Model):  # schemas.py:41-45
    avg_parameters_update: List[np.ndarray]


class FedPCASharedState(_Model):  # schemas.py:48-54
    n_samples: int
    parameters_update: List[np.ndarray]
