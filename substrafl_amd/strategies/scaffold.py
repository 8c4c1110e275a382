"""Scaffold with the two-bucket aggregation on MI355X.

Drop-in for ``substrafl.strategies.Scaffold`` (substrafl/strategies/scaffold.py:22-387) on the
aggregation hot path.  NumPy 2 (NEP 50) makes the reference compute everything in fp64 -- the
client weights are a float64 array (scaffold.py:319-320) -- and return fp64 arrays; the HIP
kernel does the same, adds the server control variate ``c`` last (scaffold.py:262-263) and
applies ``aggregation_lr`` after the sum (scaffold.py:293).  The check that every client sent
the same ``c`` (scaffold.py:193-196) runs on the host while one copy of ``c`` is staged (the
engine's ``c_check="device"`` keeps the GPU ``equal_count`` kernel as an option).
"""

from typing import List, Optional

import numpy as np

from ..engine import Devices
from ..remote import remote
from ..schemas import ScaffoldAveragedStates, ScaffoldSharedState, StrategyName
from .strategy import Strategy


class Scaffold(Strategy):
    _aggregation_methods = {"avg_shared_states": "scaffold"}

    def __init__(self, algo, aggregation_lr: float = 1, metric_functions=None, device: Devices = None):
        if device is None:
            super().__init__(algo=algo, aggregation_lr=aggregation_lr, metric_functions=metric_functions)
        else:
            super().__init__(algo=algo, aggregation_lr=aggregation_lr, metric_functions=metric_functions,
                             device=device)
        if aggregation_lr < 0:
            raise ValueError("aggregation_lr must be >=0")
        self._aggregation_lr = aggregation_lr
        self._device = device
        self._local_states = None
        self._shared_states = None

    @property
    def name(self) -> StrategyName:
        return StrategyName.SCAFFOLD

    def _check_shared_states(self, shared_states: List[ScaffoldSharedState]) -> None:
        """Host-decidable half of scaffold.py:168-202 (types, list lengths, shapes of ``c``);
        the element-wise ``c`` equality is counted by the engine while it stages ``c``."""
        assert shared_states, "shared_states should contain at least one element"
        assert isinstance(shared_states, (list, tuple)), "shared_states should be a list"
        first = shared_states[0]
        for shared_state in shared_states:
            assert isinstance(shared_state, ScaffoldSharedState) or type(shared_state).__name__ == (
                "ScaffoldSharedState"
            ), "shared_state should be an instance of ScaffoldSharedState"
            assert len(shared_state.control_variate_update) == len(
                first.control_variate_update
            ), "the length of control_variate_update should be the same for each shared_state"
            assert len(shared_state.parameters_update) == len(
                first.parameters_update
            ), "the length of parameters_update should be the same for each shared_state"
            assert len(shared_state.server_control_variate) == len(
                first.server_control_variate
            ), "the length of server_control_variate should be the same for each shared_state"
            for c, ci in zip(first.server_control_variate, shared_state.server_control_variate):
                if np.shape(c) == np.shape(ci):
                    continue  # the element-wise comparison runs in the engine while c is staged
                # np.testing.assert_array_equal (scaffold.py:193-196) broadcasts a 0-d operand against
                # the other one and refuses any other shape mismatch
                assert np.ndim(c) == 0 or np.ndim(ci) == 0, "all server_control_variate in the shared_states are not equal"
                assert _all_equal(c, ci), "all server_control_variate in the shared_states are not equal"
        assert (
            len(first.control_variate_update) == len(first.server_control_variate) == len(first.parameters_update)
        ), "the length of server_control_variate, parameters_update and server_control_variate should be the same"

    @staticmethod
    def _server_control_variates(shared_states) -> List[list]:
        """Every client's c for the engine's element-wise check; a client whose layers differ in
        shape from client 0's (a 0-d layer, already compared value by value on the host) passes
        client 0's arrays instead."""
        c0 = list(shared_states[0].server_control_variate)
        out = []
        for s in shared_states:
            ci = list(s.server_control_variate)
            out.append(ci if all(np.shape(a) == np.shape(b) for a, b in zip(c0, ci)) else c0)
        return out

    @remote
    def avg_shared_states(self, shared_states: List[ScaffoldSharedState]) -> ScaffoldAveragedStates:
        """Scaffold server step (scaffold.py:297-337): averaged weight update times
        ``aggregation_lr`` and updated server control variate, both fp64."""
        from ..integration import scaffold_average

        new_c, avg = scaffold_average(self, shared_states, self._aggregation_lr, self._device, wire=True)
        return ScaffoldAveragedStates(server_control_variate=new_c, avg_parameters_update=avg)


def _all_equal(a, b) -> bool:
    """Value equality as np.testing.assert_array_equal has it (NaN == NaN, +0 == -0), broadcast."""
    a, b = np.asarray(a), np.asarray(b)
    eq = np.asarray(a == b)
    if a.dtype.kind in "fc" and b.dtype.kind in "fc":
        eq = eq | (np.isnan(a) & np.isnan(b))
    return bool(np.all(eq))
