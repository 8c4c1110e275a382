"""The exception type ``accelerate`` re-raises for an empty input (substrafl/exceptions.py's name)."""


class EmptySharedStatesError(Exception):
    """No shared state to aggregate."""
