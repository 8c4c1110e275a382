from .torch_base_algo import TorchAlgo  # noqa: F401
from .torch_fed_avg_algo import TorchFedAvgAlgo  # noqa: F401
from .torch_scaffold_algo import CUpdateRule, TorchScaffoldAlgo  # noqa: F401
