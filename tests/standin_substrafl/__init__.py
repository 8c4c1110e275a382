"""A builder-written stand-in with the SHAPE of the reference package ``substrafl`` -- not its
files or text -- for running ``substrafl_amd.integration.accelerate`` on the GPU box, where the
reference is absent (VERDICT r03 "Next 3").

What ``accelerate`` binds to, under the same module paths as the reference
(substrafl/strategies/__init__.py, strategies/schemas.py, remote/decorators.py, exceptions.py):

* ``strategies.FedAvg`` / ``Scaffold`` / ``FedPCA`` with the reference's constructor arguments
  (``algo``, ``metric_functions``; Scaffold's ``aggregation_lr`` kept as ``_aggregation_lr``),
  ``name`` and ``@remote`` aggregation methods -- whose bodies here refuse to run, so a passing
  test proves the accelerated subclass's bodies (the MI355X engine) did the work;
* ``strategies.schemas``: pydantic shared / averaged state models with the reference's field names;
* ``remote.remote``: ``_skip=True`` calls the method, otherwise a ``RemoteOperation`` record;
* ``exceptions.EmptySharedStatesError``.
"""
