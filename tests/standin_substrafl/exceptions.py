"""The exception type ``accelerate`` re-raises for an empty input (substrafl/exceptions.py's name)."""


class EmptySharedStatesError(Exception):
    """No shared state to aggregate."""


class TorchScaffoldAlgoParametersUpdateError(Exception):
    """The per-step Scaffold hook was not called once per update."""


class IndexGeneratorUpdateError(Exception):
    """The index generator was not drawn num_updates times."""


class SharedStatesError(Exception):
    """A shared state of the wrong type or with inconsistent sizes."""
