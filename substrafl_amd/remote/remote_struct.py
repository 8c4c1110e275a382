"""Re-instantiation contract of a remote method (substrafl/remote/remote_struct.py:12-137).

A strategy is cloudpickled as ``(cls, args, kwargs, method_name, method_parameters)`` and
re-created in the task process with ``cls(*args, **kwargs)`` (remote_struct.py:108-114), so
engine options must be plain constructor kwargs and the engine itself is never pickled.
"""

from pathlib import Path
from typing import Any, Dict, Optional, Type

import cloudpickle


class RemoteStruct:
    def __init__(
        self,
        cls: Type,
        cls_args: list,
        cls_kwargs: dict,
        remote_cls: Type,
        method_name: str,
        method_parameters: dict,
        algo_name: Optional[str],
    ):
        self._cls = cls
        self._cls_args = cls_args
        self._cls_kwargs = cls_kwargs
        self._remote_cls = remote_cls
        self._method_name = method_name
        self._method_parameters = method_parameters
        self._algo_name = algo_name or f"{method_name}_{cls.__name__}"

    def __eq__(self, other: object) -> bool:
        if not isinstance(other, RemoteStruct):
            return NotImplemented
        return (self._cls, self._cls_args, self._cls_kwargs, self._remote_cls, self._method_name,
                self._method_parameters) == (other._cls, other._cls_args, other._cls_kwargs, other._remote_cls,
                                             other._method_name, other._method_parameters)

    def __hash__(self):
        return hash((self._cls, self._remote_cls, self._method_name))

    @property
    def algo_name(self) -> str:
        return self._algo_name

    @classmethod
    def load(cls, src: Path) -> "RemoteStruct":
        with (Path(src) / "cls_cloudpickle").open("rb") as f:
            return cloudpickle.load(f)

    def save(self, dest: Path) -> None:
        with (Path(dest) / "cls_cloudpickle").open("wb") as f:
            cloudpickle.dump(self, f)

    def get_instance(self) -> Any:
        return self._cls(*self._cls_args, **self._cls_kwargs)

    def get_remote_instance(self):
        return self._remote_cls(self.get_instance(), method_name=self._method_name,
                                method_parameters=self._method_parameters)

    def summary(self) -> Dict[str, str]:
        return {"type": self._cls.__name__, "method_name": self._method_name}
