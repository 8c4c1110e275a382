"""Base class of client algorithms (substrafl/algorithms/algo.py:15-156).

Only the part the strategy plugin surface relies on: ``args``/``kwargs`` capture for
RemoteStruct re-instantiation (algo.py:18-20) and the ``strategies`` compatibility list that
``Strategy.__init__`` checks (strategy.py:67-73).
"""

import abc
from typing import Any, List


class Algo(abc.ABC):
    def __init__(self, *args, **kwargs):
        self.args = args
        self.kwargs = kwargs

    @property
    @abc.abstractmethod
    def model(self) -> Any:
        raise NotImplementedError

    @property
    @abc.abstractmethod
    def strategies(self) -> List[str]:
        raise NotImplementedError

    @abc.abstractmethod
    def train(self, data_from_opener, shared_state: Any) -> Any:
        raise NotImplementedError

    def load_local_state(self, path):  # pragma: no cover - client side, out of scope
        raise NotImplementedError

    def save_local_state(self, path):  # pragma: no cover
        raise NotImplementedError
