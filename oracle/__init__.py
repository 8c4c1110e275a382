"""CPU oracle for the FedAvg / Scaffold aggregation hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``substrafl_amd`` imports this package:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may use it, and only as the checker or as the timed CPU baseline -- never as
the thing measured or shipped.

Parity status: PINNED.  The restatements here are checked against golden
vectors captured from the reference itself (``tests/golden/gen_golden.py``
imports ``/root/reference`` in the build container and calls
``FedAvg.avg_shared_states`` / ``Scaffold.avg_shared_states`` with
``_skip=True``) and against the reference's own unit-test known answers
(``tests/strategies/test_fed_avg.py:17-65``,
``tests/strategies/test_scaffold.py:22-198``).
"""

from .aggregation import (  # noqa: F401
    fedavg_reference_structure,
    fedavg_explicit,
    scaffold_reference_structure,
    scaffold_explicit,
    numpy_pairwise_sum,
    fedavg_weights_f32,
    scaffold_weights_f64,
    newton_raphson_sums,
    newton_raphson_reference_structure,
)
