"""FedPCA's aggregation on MI355X (kernel reuse).

``FedPCA.avg_shared_states`` (substrafl/strategies/fed_pca.py:210-259) is, operation for
operation, FedAvg's weighted average (fed_avg.py:217-222), so it runs on the
same bucket kernel and is bit-identical to the reference.  ``avg_shared_states_with_qr``
(:261-299) averages on the GPU the same way and then factorises each averaged matrix with
``np.linalg.qr`` exactly as the reference does -- the QR is a small dense LAPACK call on the
result, not part of the element-wise hot path.  The federated-PCA graph
building (``perform_round``) is Substra control plane and out of scope.
"""

from typing import List, Optional

import numpy as np

from ..engine import Devices
from ..remote import remote
from ..schemas import FedPCAAveragedState, FedPCASharedState, StrategyName
from .fed_avg import weighted_average
from .strategy import Strategy


class FedPCA(Strategy):
    _aggregation_methods = {"avg_shared_states": "fedavg", "avg_shared_states_with_qr": "fedavg"}

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
        return StrategyName.FEDERATED_PCA

    @remote
    def avg_shared_states(self, shared_states: List[FedPCASharedState]) -> FedPCAAveragedState:
        averaged = weighted_average(shared_states, "FedPCASharedState", self._device)
        return FedPCAAveragedState(avg_parameters_update=averaged)

    @remote
    def avg_shared_states_with_qr(self, shared_states: List[FedPCASharedState]) -> FedPCAAveragedState:
        averaged = weighted_average(shared_states, "FedPCASharedState", self._device)
        out = []
        for a in averaged:
            q, _ = np.linalg.qr(a.T)  # fed_pca.py:295-296
            out.append(q.T)
        return FedPCAAveragedState(avg_parameters_update=out)
