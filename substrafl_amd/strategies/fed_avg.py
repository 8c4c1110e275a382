"""FedAvg with the aggregation on MI355X.

Drop-in for ``substrafl.strategies.FedAvg`` (substrafl/strategies/fed_avg.py:23-274) on the
aggregation hot path: same class name, constructor, ``name``, ``@remote`` method
``avg_shared_states(shared_states) -> FedAvgAveragedState``, same exceptions, and results
bit-identical to the reference's NumPy arithmetic (fed_avg.py:217-222): the weighted sum of the
client buckets runs in libfedagg's HIP kernels (substrafl_amd/csrc/fedagg.hip).
"""

from typing import List, Optional

import numpy as np

from ..engine import Devices, engine_for
from ..exceptions import EmptySharedStatesError
from ..remote import remote
from ..schemas import FedAvgAveragedState, FedAvgSharedState, StrategyName
from .strategy import Strategy


def check_same_shapes(per_client_layers: List[List[np.ndarray]]) -> None:
    """``np.sum(list, axis=0)`` raises ValueError when the stacked arrays are inhomogeneous
    (fed_avg.py:222, scaffold.py:263/293)."""
    ref = per_client_layers[0]
    for other in per_client_layers[1:]:
        for a, b in zip(ref, other):
            if np.shape(a) != np.shape(b):
                raise ValueError(
                    "setting an array element with a sequence. The requested array has an inhomogeneous shape "
                    f"({np.shape(a)} vs {np.shape(b)})"
                )


class FedAvg(Strategy):
    """Federated averaging: ``Δw = Σ_k (n_k / n) Δw_k`` (fed_avg.py:23-52)."""

    def __init__(self, algo, metric_functions=None, device: Devices = None):
        if device is None:
            super().__init__(algo=algo, metric_functions=metric_functions)
        else:
            super().__init__(algo=algo, metric_functions=metric_functions, device=device)
        self._device = device
        self._local_states = None
        self._shared_states = None

    @property
    def name(self) -> StrategyName:
        return StrategyName.FEDERATED_AVERAGING

    @remote
    def avg_shared_states(self, shared_states: List[FedAvgSharedState]) -> FedAvgAveragedState:
        """Weighted average of the clients' ``parameters_update`` by ``n_samples`` (fed_avg.py:176-224).

        Raises:
            EmptySharedStatesError: ``shared_states`` is empty (fed_avg.py:207-211).
            AssertionError: clients do not have the same number of layers (fed_avg.py:213-215).
            ZeroDivisionError: ``sum(n_samples) == 0`` (fed_avg.py:221).
            ValueError: a layer's shape differs between clients (``np.sum``, fed_avg.py:222).
            pydantic.ValidationError: a 0-d layer (its average is a scalar, schemas.py:29).
        """
        averaged_states = weighted_average(shared_states, "FedAvgSharedState", self._device)
        return FedAvgAveragedState(avg_parameters_update=averaged_states)


def weighted_average(shared_states, state_name: str, device: Devices = None, wire: bool = True,
                     empty_error=EmptySharedStatesError) -> List[np.ndarray]:
    """fed_avg.py:207-222 (also fed_pca.py:244-257): validation on the host, the weighted sum
    of every layer on the GPU.  ``wire``: layers in the flat wire format (this package's own
    schemas); False: plain NumPy arrays (the reference's schemas, :mod:`substrafl_amd.integration`).
    ``empty_error``: the exception class raised for an empty list (the reference's own there)."""
    if len(shared_states) == 0:
        raise empty_error(
            "Your shared_states is empty. Please ensure that "
            f"the train method of your algorithm returns a {state_name} object."
        )
    parameters_update_len = len(shared_states[0].parameters_update)
    assert all(
        [len(shared_state.parameters_update) == parameters_update_len for shared_state in shared_states]
    ), "Not the same number of layers for every input parameters."

    n_samples = [state.n_samples for state in shared_states]
    n_all_samples = sum(n_samples)
    if parameters_update_len == 0:
        return []
    if n_all_samples == 0:
        raise ZeroDivisionError("division by zero")
    updates = [list(state.parameters_update) for state in shared_states]
    check_same_shapes(updates)
    engine = engine_for(device)
    # substrafl_amd's own schemas already need this package to unpickle: the flat wire format
    return engine.fedavg(updates, n_samples, wire=wire)
