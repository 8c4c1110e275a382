"""The drop-in for SubstraFL's experiment drivers: the reference's own strategy classes with their
aggregation method bodies on the MI355X engine.

``accelerate(substrafl.strategies.FedAvg)`` returns a subclass of the reference class that keeps
everything of it -- constructor, ``name``, graph building (``build_compute_plan``,
``perform_round``; substrafl/strategies/fed_avg.py:79-137, strategy.py:183-246), the reference's
``@remote`` decorator and schemas -- and replaces only the bodies of the aggregation methods:

* ``FedAvg.avg_shared_states`` (fed_avg.py:176-224): the weighted sum of the client layers in
  ``fedavg_kernel`` (bit-identical to fed_avg.py:217-222);
* ``Scaffold.avg_shared_states`` (scaffold.py:297-337): the fp64 two-bucket reduction, ``c`` last
  and ``aggregation_lr`` after the sum, with the ``c`` equality check of scaffold.py:193-196
  counted while ``c`` is staged;
* ``FedPCA.avg_shared_states`` / ``avg_shared_states_with_qr`` (fed_pca.py:210-299): FedAvg's
  reduction (+ the reference's ``np.linalg.qr`` of each averaged matrix);
* ``NewtonRaphson.compute_averaged_states`` (newton_raphson.py:151-216): the weighted sums of the
  clients' Hessians and gradients (the explicit ``+=`` chain, ``engine.sequential_sum``), then the
  reference's own ``np.linalg.solve`` and unflatten on the host.

So the class goes straight into ``simulate_experiment`` / ``execute_experiment``::

    from substrafl.strategies import FedAvg
    from substrafl_amd.integration import accelerate

    strategy = accelerate(FedAvg)(algo=my_algo)      # same arguments as the reference class

Error behaviour is the reference's: its ``EmptySharedStatesError``, the layer-count
``AssertionError``, ``ZeroDivisionError`` for ``sum(n_samples) == 0``, ``ValueError`` for shapes
that differ between clients, ``AssertionError`` for differing server control variates.  The task
process re-creates the strategy from its ``RemoteStruct`` (``cls=self.__class__``): cloudpickle
carries the generated subclass by value, so the task environment needs ``substrafl_amd`` (with its
built ``libfedagg.so``) next to ``substrafl``.  Nothing here imports SubstraFL at module level.
"""

from __future__ import annotations

import importlib
from typing import Optional

import numpy as np

from . import handoff
from .engine import Devices, engine_for
from .strategies.fed_avg import check_same_shapes, weighted_average
from .strategies.scaffold import Scaffold as _MirrorScaffold
from .strategies.strategy import Strategy as _MirrorStrategy


def _reference_modules(strategy_cls):
    """The reference package the class comes from (``substrafl``): its strategies, schemas,
    ``remote`` decorator and exceptions.  Found from the first class in the MRO that lives in a
    ``<pkg>.strategies`` module, so a user subclass defined anywhere (``__main__``) works."""
    mods = [b.__module__ for b in getattr(strategy_cls, "__mro__", ())]
    pkg = next((m.split(".")[0] for m in mods if ".strategies" in m), strategy_cls.__module__.split(".")[0])
    return (importlib.import_module(f"{pkg}.strategies"), importlib.import_module(f"{pkg}.strategies.schemas"),
            importlib.import_module(f"{pkg}.remote").remote, importlib.import_module(f"{pkg}.exceptions"))


def accelerate(strategy_cls, device: Devices = None):
    """A subclass of the reference strategy class ``strategy_cls`` (``FedAvg``, ``Scaffold``,
    ``FedPCA`` or a subclass of one of them) whose aggregation methods run on the engine of
    ``device`` (:func:`engine.engine_for`: None = the current GPU, an index, a list, or "all")."""
    strategies, schemas, remote, exceptions = _reference_modules(strategy_cls)
    empty = exceptions.EmptySharedStatesError
    base_init = strategy_cls.__init__

    def __init__(self, *args, **kwargs):
        base_init(self, *args, **kwargs)
        handoff.register("aggregator", self)  # the clients' exports are recorded for it (handoff.py)

    ns = {"__doc__": f"{strategy_cls.__name__} with its aggregation on MI355X (substrafl_amd.integration).",
          "__init__": __init__,
          "_fedagg_device": device,
          # the task-process hooks of INTEGRATION.md §3 (prewarm, overlapped ingest), as the mirrors have them
          "prewarm_aggregation": _MirrorStrategy.prewarm_aggregation,
          "ingest_shared_states": _MirrorStrategy.ingest_shared_states}

    if issubclass(strategy_cls, strategies.Scaffold):
        averaged_cls = schemas.ScaffoldAveragedStates

        def avg_shared_states(self, shared_states):
            """scaffold.py:297-337 on the engine (``c`` check of :193-196 while ``c`` is staged)."""
            new_c, avg = scaffold_average(self, shared_states, self._aggregation_lr, self._fedagg_device)
            return averaged_cls(server_control_variate=new_c, avg_parameters_update=avg)

        ns["avg_shared_states"] = remote(avg_shared_states)
        ns["_aggregation_methods"] = {"avg_shared_states": "scaffold"}
    elif issubclass(strategy_cls, strategies.FedPCA):
        averaged_cls = schemas.FedPCAAveragedState

        def avg_shared_states(self, shared_states):
            """fed_pca.py:210-259 (FedAvg's reduction) on the engine."""
            out = weighted_average(shared_states, "FedPCASharedState", self._fedagg_device, wire=False,
                                   empty_error=empty)
            return averaged_cls(avg_parameters_update=out)

        def avg_shared_states_with_qr(self, shared_states):
            """fed_pca.py:261-299: the average on the engine, then the reference's QR per layer."""
            out = weighted_average(shared_states, "FedPCASharedState", self._fedagg_device, wire=False,
                                   empty_error=empty)
            return averaged_cls(avg_parameters_update=[np.linalg.qr(a.T)[0].T for a in out])

        ns["avg_shared_states"] = remote(avg_shared_states)
        ns["avg_shared_states_with_qr"] = remote(avg_shared_states_with_qr)
        ns["_aggregation_methods"] = {"avg_shared_states": "fedavg", "avg_shared_states_with_qr": "fedavg"}
    elif issubclass(strategy_cls, strategies.FedAvg):
        averaged_cls = schemas.FedAvgAveragedState

        def avg_shared_states(self, shared_states):
            """fed_avg.py:176-224 on the engine."""
            out = weighted_average(shared_states, "FedAvgSharedState", self._fedagg_device, wire=False,
                                   empty_error=empty)
            return averaged_cls(avg_parameters_update=out)

        ns["avg_shared_states"] = remote(avg_shared_states)
        ns["_aggregation_methods"] = {"avg_shared_states": "fedavg"}
    elif getattr(strategies, "NewtonRaphson", None) is not None and issubclass(strategy_cls, strategies.NewtonRaphson):
        averaged_cls = schemas.NewtonRaphsonAveragedStates

        def compute_averaged_states(self, shared_states):
            """newton_raphson.py:151-216: the reference's checks, the two weighted sums on the
            engine, then the reference's own dense solve and unflatten on the host."""
            self._check_shared_states(shared_states)
            hessian, gradient = newton_raphson_sums(shared_states, self._fedagg_device)
            update = -self._damping_factor * np.linalg.solve(hessian, gradient)
            return averaged_cls(parameters_update=self._unflatten_array(update, shared_states[-1].gradients))

        ns["compute_averaged_states"] = remote(compute_averaged_states)
        ns["_aggregation_methods"] = {"compute_averaged_states": "sequential"}
    else:
        raise TypeError(f"accelerate takes SubstraFL's FedAvg, Scaffold, FedPCA or NewtonRaphson (or a subclass), "
                        f"not {strategy_cls!r}")
    cls = type(strategy_cls.__name__, (strategy_cls,), ns)
    # not importable by name: cloudpickle carries the class by value into the task process
    cls.__qualname__ = f"accelerate.<locals>.{strategy_cls.__name__}"
    return cls


def newton_raphson_sums(shared_states, device: Optional[Devices] = None):
    """The weighted Hessian and gradient sums of NewtonRaphson.compute_averaged_states
    (newton_raphson.py:195-211) on the engine (:meth:`engine.AggregationEngine.sequential_sum`:
    the explicit ``+=`` chain from client 0's product, bit for bit).  Returns ``(total_hessians,
    total_gradient_one_d)``; the gradients are concatenated per client first, as there.
    ``ZeroDivisionError`` for ``sum(n_samples) == 0`` and ``ValueError`` for sizes that differ
    between clients, before any device work."""
    n_samples = [s.n_samples for s in shared_states]
    if sum(int(n) for n in n_samples) == 0:
        raise ZeroDivisionError("division by zero")  # n_samples / n_all_samples (:201)
    hessians = [[np.asarray(s.hessian)] for s in shared_states]
    gradients = [[np.concatenate([np.asarray(g).reshape(-1) for g in s.gradients])] for s in shared_states]
    check_same_shapes(hessians)  # total_hessians += ... (:208)
    check_same_shapes(gradients)
    eng = engine_for(device)
    (total_h,) = eng.sequential_sum(hessians, n_samples)
    (total_g,) = eng.sequential_sum(gradients, n_samples)
    return total_h, total_g


def accelerate_algo(algo_cls, wire: bool = False):
    """The client half: :func:`substrafl_amd.algorithms.accelerate.accelerate_algo`.
    Imported on call, so the aggregation side of this module never imports torch."""
    from .algorithms.accelerate import accelerate_algo as _accelerate_algo

    return _accelerate_algo(algo_cls, wire=wire)


def scaffold_average(strategy, shared_states, aggregation_lr, device: Optional[Devices] = None, wire: bool = False):
    """Scaffold.avg_shared_states' arithmetic (scaffold.py:297-337) for any strategy object:
    the checks of scaffold.py:168-202 (element-wise ``c`` equality counted by the engine), then
    ``(new_server_control_variate, avg_parameters_update)``, both fp64."""
    _MirrorScaffold._check_shared_states(strategy, shared_states=shared_states)
    cvs = [list(s.control_variate_update) for s in shared_states]
    pus = [list(s.parameters_update) for s in shared_states]
    c0 = list(shared_states[0].server_control_variate)
    check_same_shapes([*cvs, c0])  # np.sum([w*cv_k ..., c]) (scaffold.py:263)
    check_same_shapes(pus)  # np.sum([w*Δ_k ...]) (scaffold.py:293)
    mismatches, new_c, avg = engine_for(device).scaffold(
        pus, cvs, _MirrorScaffold._server_control_variates(shared_states), [s.n_samples for s in shared_states],
        aggregation_lr, wire=wire)
    assert mismatches == 0, "all server_control_variate in the shared_states are not equal"
    return new_c, avg
