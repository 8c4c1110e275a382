"""Shared / averaged state models with the reference's class and field names
(substrafl/strategies/schemas.py), written for this stand-in."""

from enum import Enum
from typing import List

import numpy as np
import pydantic


class StrategyName(str, Enum):
    FEDERATED_AVERAGING = "Federated Averaging"
    FEDERATED_PCA = "Federated PCA"
    SCAFFOLD = "Scaffold"
    NEWTON_RAPHSON = "Newton Raphson"


class _State(pydantic.BaseModel):
    model_config = pydantic.ConfigDict(arbitrary_types_allowed=True)


class FedAvgSharedState(_State):
    n_samples: int
    parameters_update: List[np.ndarray]


class FedAvgAveragedState(_State):
    avg_parameters_update: List[np.ndarray]


class FedPCASharedState(_State):
    n_samples: int
    parameters_update: List[np.ndarray]


class FedPCAAveragedState(_State):
    avg_parameters_update: List[np.ndarray]


class ScaffoldSharedState(_State):
    parameters_update: List[np.ndarray]
    control_variate_update: List[np.ndarray]
    n_samples: int
    server_control_variate: List[np.ndarray]


class ScaffoldAveragedStates(_State):
    server_control_variate: List[np.ndarray]
    avg_parameters_update: List[np.ndarray]


class NewtonRaphsonSharedState(_State):
    n_samples: int
    gradients: List[np.ndarray]
    hessian: np.ndarray


class NewtonRaphsonAveragedStates(_State):
    parameters_update: List[np.ndarray]
