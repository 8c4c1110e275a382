"""Task-process adapter (substrafl/remote/substratools_methods.py:18-166).

In subprocess/docker/remote mode Substra spawns ``python function.py --function-name
avg_shared_states`` (remote/register/register.py:96-121); ``generic_function`` then loads the
K shared-state pickles, calls the method with ``_skip=True`` and pickles the result.  This
module reproduces that contract (without ``substratools``, which is not installed here) so
the drop-in can be exercised end to end in a child process.
"""

import os
from enum import Enum
from pathlib import Path
from typing import Any, Dict, Iterable, Union

from .serializers import PickleSerializer


class InputIdentifiers(str, Enum):  # nodes/schemas.py
    local = "local"
    shared = "shared"
    predictions = "predictions"
    opener = "opener"
    datasamples = "datasamples"
    rank = "rank"
    X = "X"
    y = "y"


class OutputIdentifiers(str, Enum):
    local = "local"
    shared = "shared"
    predictions = "predictions"


class RemoteMethod:
    def __init__(self, instance, method_name: str, method_parameters: Dict, shared_state_serializer=PickleSerializer):
        self.instance = instance
        self.method_name = method_name
        self.method_parameters = method_parameters
        self.shared_state_serializer = shared_state_serializer

    def load_method_inputs(self, inputs: Dict, outputs: Dict) -> Dict:
        loaded: Dict[str, Any] = {}
        instance_path = inputs.get(InputIdentifiers.local)
        if instance_path is not None:
            self.instance = self.instance.load_local_state(Path(instance_path))
        if InputIdentifiers.shared in inputs:
            shared = inputs[InputIdentifiers.shared]
            if shared is None:
                loaded["shared_state"] = None
            elif isinstance(shared, (str, Path)):
                loaded["shared_state"] = self.load_shared(shared)
            elif isinstance(shared, Iterable):
                paths = [Path(p) for p in shared]
                states = None
                ingest = getattr(self.instance, "ingest_shared_states", None)
                if callable(ingest):  # load + stage to the GPU, overlapped (engine.ingest)
                    load = getattr(self.shared_state_serializer, "load_mapped", self.shared_state_serializer.load)
                    states = ingest(self.method_name, paths, load)
                if states is None:
                    loader = getattr(self.shared_state_serializer, "load_many", None)
                    states = loader(paths) if loader else [self.load_shared(p) for p in paths]
                loaded["shared_states"] = states
        if InputIdentifiers.datasamples in inputs:
            loaded["data_from_opener"] = inputs[InputIdentifiers.datasamples]
        return loaded

    def save_method_output(self, method_output: Any, outputs: Dict) -> None:
        if OutputIdentifiers.local in outputs:
            self.instance.save_local_state(Path(outputs[OutputIdentifiers.local]))
        if OutputIdentifiers.shared in outputs:
            self.save_shared(method_output, outputs[OutputIdentifiers.shared])

    def _prewarm(self) -> None:
        warm = getattr(self.instance, "prewarm_aggregation", None)
        if callable(warm):
            warm(self.method_name, [])  # idempotent: starts the GPU runtime on a background thread

    def register_substratools_function(self) -> None:
        """substratools_methods.py:160-166.  Only a task process (function.py) calls this, right
        before substratools runs generic_function: for an aggregation the GPU runtime starts
        here, so its start-up overlaps the task's own set-up and input loading.  (Loading a
        finished model through model_loading builds a RemoteMethod too, but never registers it,
        so it never touches the GPU.)"""
        self._prewarm()
        try:
            import substratools as tools
        except ImportError:  # the Substra runtime is not installed here (out of scope)
            return
        tools.register(function=self.generic_function, function_name=self.method_name)

    def generic_function(self, inputs: Dict, outputs: Dict, task_properties: Dict) -> None:
        self._prewarm()  # no-op when register_substratools_function already started it
        method_inputs = self.load_method_inputs(inputs, outputs)
        method_inputs["_skip"] = True
        method_output = getattr(self.instance, self.method_name)(**method_inputs, **self.method_parameters)
        self.save_method_output(method_output, outputs)

    def load_shared(self, path: Union[str, os.PathLike]) -> Any:
        return self.shared_state_serializer.load(Path(path))

    def save_shared(self, shared_state, path: Union[str, os.PathLike]) -> None:
        self.shared_state_serializer.save(shared_state, Path(path))
