"""Client-side surface the aggregation path touches (mirror of substrafl/algorithms/)."""

from .algo import Algo  # noqa: F401
