"""Drop-in strategies whose aggregation runs on MI355X (substrafl/strategies/)."""

from .fed_avg import FedAvg  # noqa: F401
from .fed_pca import FedPCA  # noqa: F401
from .scaffold import Scaffold  # noqa: F401
from .strategy import Strategy  # noqa: F401
