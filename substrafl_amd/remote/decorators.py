"""``@remote`` / ``@remote_data`` (substrafl/remote/decorators.py:18-143).

Called without ``_skip`` a decorated method returns a deferred operation describing how to
re-create the instance and call the method in another process; with ``_skip=True`` it runs the
method body.  The aggregation hot path is always entered through the ``_skip=True`` branch
(RemoteMethod.generic_function in a task process, or SimuAggregationNode in simulation).
"""

from functools import wraps
from typing import Any, Callable, List, Optional

from .operations import RemoteDataOperation, RemoteOperation
from .remote_struct import RemoteStruct


def _remote_method_cls():
    from .substratools_methods import RemoteMethod

    return RemoteMethod


def remote(method: Callable):
    @wraps(method)
    def remote_method_inner(
        self,
        shared_states: Optional[List] = None,
        *,
        _skip: bool = False,
        _algo_name: Optional[str] = None,
        **method_parameters,
    ):
        if _skip:
            return method(self=self, shared_states=shared_states, **method_parameters)
        return RemoteOperation(
            RemoteStruct(
                cls=self.__class__,
                cls_args=self.args,
                cls_kwargs=self.kwargs,
                method_name=method.__name__,
                method_parameters=method_parameters,
                algo_name=_algo_name,
                remote_cls=_remote_method_cls(),
            ),
            shared_states,
        )

    return remote_method_inner


def remote_data(method: Callable):
    @wraps(method)
    def remote_method_inner(
        self,
        data_samples: Optional[List[str]] = None,
        shared_state: Any = None,
        *,
        _skip: bool = False,
        _algo_name: Optional[str] = None,
        **method_parameters,
    ):
        if _skip:
            return method(self=self, shared_state=shared_state, **method_parameters)
        assert data_samples is not None
        assert "data_from_opener" not in method_parameters
        return RemoteDataOperation(
            RemoteStruct(
                cls=self.__class__,
                cls_args=self.args,
                cls_kwargs=self.kwargs,
                method_name=method.__name__,
                method_parameters=method_parameters,
                algo_name=_algo_name,
                remote_cls=_remote_method_cls(),
            ),
            data_samples,
            shared_state,
        )

    return remote_method_inner
