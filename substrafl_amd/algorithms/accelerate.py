"""The client half of the drop-in: the reference's own torch algorithm classes with the
weight-delta producer / consumer of ``train`` on libfedagg's flat-bucket kernels (SURVEY.md §8(a)
rows a5-a7, §8(f) rows 1 and 3).

``accelerate_algo(TorchFedAvgAlgo)`` (or ``TorchScaffoldAlgo``, or any user subclass of either)
returns a subclass that keeps everything of the class -- constructor, ``_local_train``,
``predict``, checkpointing, ``strategies`` and the reference's ``@remote_data`` decorator -- and
replaces only the steps of ``train`` that move the model's weights around:

* FedAvg (substrafl/algorithms/pytorch/torch_fed_avg_algo.py:154-230): the averaged update goes
  onto the model in one H2D copy plus one ``fedagg_flat_increment`` launch (:186-194); the
  before/after snapshots are single ``fedagg_flat_gather`` launches into flat buckets
  (:198-200, :212-216); the delta is one ``fedagg_flat_wsum`` launch (:212-218); the export is
  one D2H copy of the delta bucket (:227-230);
* Scaffold (torch_scaffold_algo.py:338-482): the same, plus the server control variate brought
  in with one H2D copy (:403-406), ``delta_variate`` / ``control_variate_update`` / the client
  cv step as fused ``fedagg_flat_wsum`` launches (:416-420, :451-466) and the per-step
  ``w += lr * delta_variate`` hook (:256-268) as one ``fedagg_flat_increment`` launch per
  optimizer step.

The order of operations, the assertions and the error types are the reference's; every result
is bit-identical to the reference's torch ops (weight_manager.py semantics, see
:mod:`.weight_manager`).  CPU tensors and dtypes the kernels do not take run the reference's own
torch loops.  The shared states hold plain ``np.ndarray`` layers (per-layer views of one host
buffer), so the reference's schemas, pickles and ``model_loading`` accept them in any process;
``wire=True`` opts into :class:`..wire.BucketArray` layers instead (one buffer per pickle, one
staging segment per client at the aggregator, but the reading process needs ``substrafl_amd``).

Two ways to use it::

    from substrafl.algorithms.pytorch import TorchFedAvgAlgo
    from substrafl_amd.integration import accelerate_algo

    class MyAlgo(accelerate_algo(TorchFedAvgAlgo)):   # instead of (TorchFedAvgAlgo)
        ...

    algo = accelerate_algo(MyAlgo)()                   # or wrap an existing subclass

Nothing here imports SubstraFL at module level: the reference modules are found from the class.
"""

from __future__ import annotations

import importlib

from . import weight_manager as wm

_BASES = {"TorchFedAvgAlgo": "fedavg", "TorchScaffoldAlgo": "scaffold"}


def _reference_base(algo_cls):
    """The reference algorithm class ``algo_cls`` derives from (first in the MRO)."""
    if not isinstance(algo_cls, type):
        raise TypeError(f"accelerate_algo takes a class, not {algo_cls!r}")
    for base in algo_cls.__mro__:
        if base.__name__ in _BASES and base.__module__.rsplit(".", 1)[-1] in ("torch_fed_avg_algo",
                                                                               "torch_scaffold_algo"):
            return base
    raise TypeError(f"accelerate_algo takes SubstraFL's TorchFedAvgAlgo or TorchScaffoldAlgo (or a subclass), "
                    f"not {algo_cls!r}")


def _export(self, tensors, tag="export"):
    return wm.export_numpy(tensors, wire=self._fedagg_wire, tag=tag)


def _fedavg_train(shared_state_cls):
    def train(self, data_from_opener, shared_state=None):
        """TorchFedAvgAlgo.train (torch_fed_avg_algo.py:154-230) with the weight moves on the
        flat-bucket kernels."""
        bn = self._with_batch_norm_parameters
        train_dataset = self._dataset(data_from_opener, is_inference=False)
        gen = self._index_generator
        if shared_state is None:
            assert gen.n_samples is None
            gen.n_samples = len(train_dataset)
        else:
            assert gen.n_samples is not None
            # the host layers go over as one bucket; w += 1.0 * u in one launch
            wm.increment_parameters(self._model, list(shared_state.avg_parameters_update),
                                    with_batch_norm_parameters=bn)
        gen.reset_counter()
        before = wm.get_parameters(self._model, with_batch_norm_parameters=bn)

        self._model.train()
        self._local_train(train_dataset)
        gen.check_num_updates()
        self._model.eval()

        delta = wm.subtract_parameters(wm.get_parameters(self._model, with_batch_norm_parameters=bn), before)
        wm.set_parameters(self._model, before, with_batch_norm_parameters=bn)  # back to the pre-train state
        return shared_state_cls(n_samples=len(train_dataset), parameters_update=_export(self, delta))

    return train


def _scaffold_train(shared_state_cls, fast_rule, update_error):
    def train(self, data_from_opener, shared_state=None):
        """TorchScaffoldAlgo.train (torch_scaffold_algo.py:338-482) with the weight and control
        variate moves on the flat-bucket kernels."""
        bn = self._with_batch_norm_parameters
        train_dataset = self._dataset(data_from_opener, is_inference=False)
        gen = self._index_generator
        if shared_state is None:
            assert gen.n_samples is None
            gen.n_samples = len(train_dataset)
            # both control variates start at zero, shaped like the bucket (one flat allocation each)
            assert self._client_control_variate is None
            self._client_control_variate = wm.zeros_like_parameters(self.model, with_batch_norm_parameters=bn,
                                                                     device=self._device)
            assert self._server_control_variate is None
            self._server_control_variate = wm.zeros_like_parameters(self.model, with_batch_norm_parameters=bn,
                                                                    device=self._device)
            self._fedagg_c_host = None
        else:
            assert self._client_control_variate is not None
            assert gen.n_samples is not None
            # avg_parameters_update already carries aggregation_lr (scaffold.py:293)
            wm.increment_parameters(self._model, list(shared_state.avg_parameters_update),
                                    with_batch_norm_parameters=bn)
            c_host = list(shared_state.server_control_variate)
            self._server_control_variate = wm.to_device(c_host, self._device)
            self._fedagg_c_host = _frozen_source(c_host, self._server_control_variate)
        gen.reset_counter()
        before = wm.get_parameters(self._model, with_batch_norm_parameters=bn)
        # c_i - c, added lr-scaled after every optimizer step by _scaffold_parameters_update
        self._delta_variate = wm.subtract_parameters(self._client_control_variate, self._server_control_variate)

        self._model.train()
        self._local_train(train_dataset)
        gen.check_num_updates()
        if self._scaffold_parameters_update_num_call != gen._num_updates:
            raise update_error(
                f"`_scaffold_parameters_update` method has been called {self._scaffold_parameters_update_num_call} "
                f"time(s) but num_updates is set to {gen._num_updates}. Please check within your "
                "`_local_train` function that `_scaffold_parameters_update` is called at each update (each time "
                "self._model(data) is called) after the `self.optimizer.step()` call.")
        self._reset_scaffold_parameters_update()
        self._model.eval()

        delta = wm.subtract_parameters(wm.get_parameters(self._model, with_batch_norm_parameters=bn), before)
        if self._c_update_rule != fast_rule:
            raise NotImplementedError("rule 1 not implemented")
        # option II of the Scaffold paper: c_i+ - c_i = -c - delta / (lr * num_updates)
        cv_update = wm.weighted_sum_parameters([self._server_control_variate, delta],
                                               [-1.0, -1.0 / (self._current_lr * gen.num_updates)])
        self._client_control_variate = wm.add_parameters(self._client_control_variate, cv_update)
        wm.set_parameters(self._model, before, with_batch_norm_parameters=bn)
        # one recycled host buffer per list: the three are alive together until the next round
        c_out = _unchanged_source(getattr(self, "_fedagg_c_host", None), self._server_control_variate)
        return shared_state_cls(parameters_update=_export(self, delta),
                                control_variate_update=_export(self, cv_update, "export_cv"),
                                server_control_variate=(c_out if c_out is not None else
                                                        _export(self, self._server_control_variate, "export_c")),
                                n_samples=len(train_dataset))

    return train


def _frozen_source(host: list, tensors):
    """Simulation mode with the device hand-off (``handoff``): the server control variate's host
    arrays as received, when they are frozen (an engine output) -- the client's export of c may
    then return them instead of copying the same bytes back from the device."""
    from .. import handoff

    flat = wm.flat_bucket(list(tensors)) if tensors else None
    if not handoff.enabled() or flat is None or not handoff.frozen(host):
        return None
    return host, flat, flat._version


def _unchanged_source(rec, tensors):
    """The recorded host arrays of c (``_frozen_source``) if they are still frozen and the device
    bucket still holds what was copied from them (not modified in place since); else None.  The
    export then returns those very arrays (read-only, the same bytes the reference's
    ``.cpu().numpy()`` would produce), which also lets the aggregator see every client's c as one
    object (its identity shortcut of scaffold.py:193-196)."""
    from .. import handoff

    if rec is None or not handoff.enabled():
        return None
    host, flat, version = rec
    cur = wm.flat_bucket(list(tensors)) if tensors else None
    if cur is None or cur.data_ptr() != flat.data_ptr() or flat._version != version or not handoff.frozen(host):
        return None
    return list(host)


def _scaffold_parameters_update(self):
    """The per-step hook (torch_scaffold_algo.py:256-268): ``w += lr * (c_i - c)`` in one launch."""
    self._update_current_lr()
    self._scaffold_parameters_update_num_call += 1
    wm.increment_parameters(self._model, self._delta_variate, with_batch_norm_parameters=self._with_batch_norm_parameters,
                            updates_multiplier=self._current_lr)


def _registering_init(base_init):
    """The class's own constructor, then the instance registered as a hand-off consumer of the
    engine's outputs (``handoff.register``: only then are they recorded, and frozen, for it)."""

    def __init__(self, *args, **kwargs):
        base_init(self, *args, **kwargs)
        from .. import handoff

        handoff.register("client", self)

    return __init__


def accelerate_algo(algo_cls, wire: bool = False):
    """A subclass of ``algo_cls`` (SubstraFL's ``TorchFedAvgAlgo`` / ``TorchScaffoldAlgo`` or a
    subclass of one) whose ``train`` moves weights with the flat-bucket kernels.  ``wire``:
    export :class:`..wire.BucketArray` layers instead of plain arrays."""
    base = _reference_base(algo_cls)
    pkg = base.__module__.split(".")[0]
    remote_data = importlib.import_module(f"{pkg}.remote").remote_data
    schemas = importlib.import_module(f"{pkg}.strategies.schemas")
    ns = {"__doc__": f"{algo_cls.__name__} with its weight moves on MI355X (substrafl_amd.accelerate_algo).",
          "_fedagg_wire": bool(wire),
          "__init__": _registering_init(algo_cls.__init__),
          "__module__": __name__}  # type() under ABCMeta would otherwise record "abc"
    if _BASES[base.__name__] == "scaffold":
        exceptions = importlib.import_module(f"{pkg}.exceptions")
        fast = importlib.import_module(base.__module__).CUpdateRule.FAST
        ns["train"] = remote_data(_scaffold_train(schemas.ScaffoldSharedState, fast,
                                                  exceptions.TorchScaffoldAlgoParametersUpdateError))
        ns["_scaffold_parameters_update"] = _scaffold_parameters_update
    else:
        ns["train"] = remote_data(_fedavg_train(schemas.FedAvgSharedState))
    cls = type(algo_cls.__name__, (algo_cls,), ns)
    # not importable by name: cloudpickle carries the class by value into the task process
    cls.__qualname__ = f"accelerate_algo.<locals>.{algo_cls.__name__}"
    return cls
