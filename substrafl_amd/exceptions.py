"""Exceptions raised on the aggregation path, with the reference's names and meaning.

Reference: substrafl/exceptions.py (``EmptySharedStatesError`` :45-47,
``IncompatibleAlgoStrategyError`` :54-55).
"""


class EmptySharedStatesError(Exception):
    """The shared_states is empty. Ensure that the train method of the algorithm returns a
    StrategySharedState object."""


class IncompatibleAlgoStrategyError(Exception):
    """This algo is not compatible with this strategy."""


class LoadMetadataError(Exception):
    """metadata.json must name the ``model_file`` and ``function_file`` (exceptions.py:129-130)."""


class LoadFileNotFoundError(Exception):
    """The folder must hold function.tar.gz, metadata.json and the model file (exceptions.py:133-135)."""
