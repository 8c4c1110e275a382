"""FedAvg / Scaffold / FedPCA with the reference's constructor arguments, ``name`` and ``@remote``
aggregation methods.  The aggregation bodies refuse to run: ``accelerate`` must replace them."""

import numpy as np

from ..exceptions import EmptySharedStatesError, SharedStatesError
from ..remote import remote
from .schemas import NewtonRaphsonSharedState, StrategyName


class Strategy:
    def __init__(self, algo, metric_functions=None, **kwargs):
        self.algo = algo
        self.metric_functions = metric_functions
        self.kwargs = dict(kwargs, algo=algo, metric_functions=metric_functions)

    @property
    def name(self):
        raise NotImplementedError


def _not_here(self, shared_states):
    raise NotImplementedError("stand-in aggregation body: accelerate() must have replaced it")


class FedAvg(Strategy):
    @property
    def name(self):
        return StrategyName.FEDERATED_AVERAGING

    @remote
    def avg_shared_states(self, shared_states):
        return _not_here(self, shared_states)


class Scaffold(Strategy):
    def __init__(self, algo, aggregation_lr: float = 1, metric_functions=None):
        super().__init__(algo=algo, metric_functions=metric_functions, aggregation_lr=aggregation_lr)
        if aggregation_lr < 0:
            raise ValueError("aggregation_lr must be >= 0")
        self._aggregation_lr = aggregation_lr

    @property
    def name(self):
        return StrategyName.SCAFFOLD

    @remote
    def avg_shared_states(self, shared_states):
        return _not_here(self, shared_states)


class FedPCA(Strategy):
    @property
    def name(self):
        return StrategyName.FEDERATED_PCA

    @remote
    def avg_shared_states(self, shared_states):
        return _not_here(self, shared_states)

    @remote
    def avg_shared_states_with_qr(self, shared_states):
        return _not_here(self, shared_states)


class NewtonRaphson(Strategy):
    """The reference's constructor (``damping_factor`` in (0, 1]), checks and unflatten helper,
    written for this stand-in; its averaging body refuses to run."""

    def __init__(self, algo, damping_factor: float, metric_functions=None):
        super().__init__(algo=algo, metric_functions=metric_functions, damping_factor=damping_factor)
        if not 0 < damping_factor <= 1:
            raise ValueError("damping_factor must be in (0, 1]")
        self._damping_factor = damping_factor

    @property
    def name(self):
        return StrategyName.NEWTON_RAPHSON

    def _check_shared_states(self, shared_states):
        if not shared_states:
            raise EmptySharedStatesError("no shared state")
        for st in shared_states:
            if not isinstance(st, NewtonRaphsonSharedState):
                raise SharedStatesError("expected NewtonRaphsonSharedState")
            if len(st.hessian) != sum(g.size for g in st.gradients):
                raise SharedStatesError("hessian and gradients sizes differ")

    def _unflatten_array(self, flat, like):
        out, i = [], 0
        for a in like:
            out.append(np.array(flat[i: i + a.size].reshape(a.shape)))
            i += a.size
        return out

    @remote
    def compute_averaged_states(self, shared_states):
        return _not_here(self, shared_states)
