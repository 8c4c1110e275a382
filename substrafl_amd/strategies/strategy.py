"""Strategy base: constructor contract of substrafl/strategies/strategy.py:30-73.

Every constructor argument is recorded in ``self.args`` / ``self.kwargs``
(compute_plan_builder.py:15-29) so ``RemoteStruct`` can re-create the strategy with
``cls(*args, **kwargs)`` in the task process, and ``name`` must be in ``algo.strategies``.
Graph building (``build_compute_plan``, ``perform_round``) is Substra control plane and out of
scope for this engine.
"""

from abc import abstractmethod
from typing import Sequence

from ..exceptions import IncompatibleAlgoStrategyError
from ..schemas import StrategyName


class Strategy:
    def __init__(self, algo, metric_functions=None, *args, **kwargs):
        self.args = args
        self.kwargs = dict(kwargs, algo=algo, metric_functions=metric_functions)
        self.algo = algo
        self.metric_functions = metric_functions
        if self.name not in algo.strategies:
            raise IncompatibleAlgoStrategyError(
                f"The algo {algo.__class__.__name__} is not compatible with the strategy "
                f"{self.__class__.__name__}, named {self.name}. Check the algo strategies property: "
                "algo.strategies to see the list of compatible strategies."
            )

    @property
    @abstractmethod
    def name(self) -> StrategyName:
        raise NotImplementedError

    # aggregation methods that stream the shared states through the engine, and the bucket set
    # they use ("fedavg": one bucket; "scaffold": three)
    _aggregation_methods = {"avg_shared_states": "fedavg"}

    def prewarm_aggregation(self, method_name: str, shared_paths: Sequence = ()) -> None:
        """Called by the task adapter (remote/substratools_methods.py) before it loads the shared
        states: opens and warms the GPU session on a background thread (engine.prewarm), so HIP
        start-up overlaps the unpickling.  Not part of the reference interface; a no-op for
        methods that do not aggregate on the engine."""
        if method_name not in self._aggregation_methods:
            return
        from ..engine import engine_for

        engine_for(_engine_device(self)).prewarm()

    def ingest_shared_states(self, method_name: str, shared_paths: Sequence, load):
        """Called by the task adapter instead of its own loading loop: loads the shared states on a
        thread pool and stages each client to the GPU as it arrives (engine.ingest).  Returns
        the states in path order, or None for methods that do not aggregate on the engine."""
        kind = self._aggregation_methods.get(method_name)
        if kind is None:
            return None
        from ..engine import engine_for

        engine = engine_for(_engine_device(self))
        return engine.ingest(shared_paths, kind, load)


def _engine_device(strategy):
    """The engine device of a mirrored strategy (``_device``) or of an ``integration.accelerate``d
    reference class (``_fedagg_device``)."""
    return getattr(strategy, "_fedagg_device", getattr(strategy, "_device", None))
