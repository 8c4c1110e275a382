"""FedAvg / Scaffold / FedPCA with the reference's constructor arguments, ``name`` and ``@remote``
aggregation methods.  The aggregation bodies refuse to run: ``accelerate`` must replace them."""

from ..remote import remote
from .schemas import StrategyName


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
