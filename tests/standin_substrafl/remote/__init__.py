"""``@remote`` with the reference's calling convention (substrafl/remote/decorators.py): the
aggregation node calls ``method(shared_states=..., _skip=True)`` and gets the result; without
``_skip`` the call only records the operation for the compute plan."""

import functools
from dataclasses import dataclass, field


@dataclass
class RemoteOperation:
    cls: type
    method_name: str
    kwargs: dict = field(default_factory=dict)
    shared_states: object = None


def remote(method):
    @functools.wraps(method)
    def wrapper(self, shared_states=None, _skip: bool = False, **method_parameters):
        if _skip:
            return method(self, shared_states=shared_states, **method_parameters)
        return RemoteOperation(type(self), method.__name__, dict(method_parameters), shared_states)

    return wrapper


@dataclass
class RemoteDataOperation:
    cls: type
    method_name: str
    data_samples: object = None
    shared_state: object = None


def remote_data(method):
    """The train-side convention (decorators.py ``remote_data``): ``_skip=True`` runs
    ``method(data_from_opener=..., shared_state=...)``, otherwise a record for the compute plan."""

    @functools.wraps(method)
    def wrapper(self, data_samples=None, shared_state=None, *, _skip: bool = False, **method_parameters):
        if _skip:
            return method(self=self, shared_state=shared_state, **method_parameters)
        return RemoteDataOperation(type(self), method.__name__, data_samples, shared_state)

    return wrapper
