"""substrafl_amd -- MI355X-native aggregation engine for SubstraFL's federated strategies.

The hot path (``FedAvg.avg_shared_states`` / ``Scaffold.avg_shared_states``) runs in hand-written
gfx950 HIP kernels behind a C ABI (``include/fedagg.h``, ``libfedagg.so``); this package is the
Python host side that mirrors the reference's strategy plugin surface.  Importing it never
touches the GPU (HIP initialises on the first aggregation).
"""

__version__ = "0.5.0"

from .schemas import (  # noqa: F401
    FedAvgAveragedState,
    FedAvgSharedState,
    ScaffoldAveragedStates,
    ScaffoldSharedState,
    StrategyName,
)
