"""``AggregationEngine.fedavg``'s staging resolver (VERDICT r05 "Next 3": ``_resolve_rows``, one
reason per call in ``last_timing["staging"]``): each of the paths the client rows can take into
HBM is driven here by name, and every result is bit-identical to the reference's order
(oracle.fedavg_explicit, fed_avg.py:217-222) -- the path changes where the bytes come from, never
the arithmetic.

* ``host-rows`` / ``host-tiles``: staged over PCIe through the pinned ring ([K, ld] rows, or
  tile-interleaved);
* ``prestaged-rows`` / ``prestaged-tiles``: staged by ``ingest`` while the states were loading;
* ``handoff-in-place`` / ``handoff-partial``: simulation mode, every / some row still on the GPU
  as a client's exported bucket (``handoff``);
* ``out-of-core``: the call streamed through the GPU in parameter ranges."""

import gc
import types

import numpy as np
import pytest

from oracle import fedavg_explicit

pytestmark = pytest.mark.gpu

SHAPES = [(64, 33), (33,), (1,), (1000,), (7, 3)]
K = 4


def _clients(seed=0):
    rng = np.random.default_rng(seed)
    pus = [[(rng.standard_normal(s) * 10.0 ** rng.integers(-2, 2)).astype(np.float32) for s in SHAPES]
           for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    return pus, ns


def _bits_equal(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        g, r = np.asarray(g), np.asarray(r)
        assert g.dtype == r.dtype and g.shape == r.shape
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32))


@pytest.fixture()
def engine():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from substrafl_amd.engine import AggregationEngine

    return AggregationEngine(device=0)


@pytest.mark.parametrize("tiled, reason", [(False, "host-rows"), (True, "host-tiles")])
def test_host_staging(engine, tiled, reason):
    pus, ns = _clients(1)
    engine.tiled = tiled
    _bits_equal(engine.fedavg(pus, ns), fedavg_explicit(pus, ns))
    assert engine.last_timing["staging"] == reason


@pytest.mark.parametrize("tiled, reason", [(False, "prestaged-rows"), (True, "prestaged-tiles")])
def test_prestaged_by_ingest(engine, tiled, reason):
    pus, ns = _clients(2)
    engine.tiled = tiled
    states = [types.SimpleNamespace(parameters_update=pu, n_samples=n) for pu, n in zip(pus, ns)]
    loaded = engine.ingest(list(range(K)), "fedavg", lambda i: states[i])
    assert engine.last_ingest["prestaged_clients"] == K
    _bits_equal(engine.fedavg([list(s.parameters_update) for s in loaded], ns), fedavg_explicit(pus, ns))
    assert engine.last_timing["staging"] == reason
    # the same arrays again: the ingest's rows were taken once, the second call stages them itself
    _bits_equal(engine.fedavg([list(s.parameters_update) for s in loaded], ns), fedavg_explicit(pus, ns))
    assert engine.last_timing["staging"] == ("host-tiles" if tiled else "host-rows")


class _Strategy:
    """Stands for an accelerate-d strategy (the consumer the clients' exports are recorded for)."""


@pytest.mark.parametrize("recorded, reason", [((0, 1, 2, 3), "handoff-in-place"), ((0, 2), "handoff-partial")])
def test_handoff(engine, recorded, reason):
    import torch

    from substrafl_amd import handoff

    pus, ns = _clients(3)
    M = sum(int(np.prod(s)) for s in SHAPES)
    handoff.enable(True)
    strategy = _Strategy()
    handoff.register("aggregator", strategy)
    try:
        rows, keep = [], []
        for k, pu in enumerate(pus):
            host = np.concatenate([a.reshape(-1) for a in pu])  # one buffer, the layers as its views
            if k in recorded:  # the client's exported bucket, still on the GPU (weight_manager.export_numpy)
                flat = torch.from_numpy(host.copy()).cuda()
                handoff.record_tensor(host, flat)  # freezes host: the views below are read-only
                keep.append(flat)
            views, off = [], 0
            for a in pu:
                views.append(host[off: off + a.size].reshape(a.shape))
                off += a.size
            rows.append(views)
        assert host.size == M
        taken = handoff.stats["taken"]
        _bits_equal(engine.fedavg(rows, ns), fedavg_explicit(pus, ns))
        assert engine.last_timing["staging"] == reason
        assert engine.last_timing["handoff_rows"] == len(recorded) == handoff.stats["taken"] - taken
        assert not handoff.records()  # each export taken once, its hold on the device bucket gone
    finally:
        handoff.enable(False)
        del strategy
        gc.collect()


def test_out_of_core(engine):
    pus, ns = _clients(4)
    engine.max_bucket_bytes = 16 << 10  # 16 KiB: the call streams through the GPU in ranges
    try:
        _bits_equal(engine.fedavg(pus, ns), fedavg_explicit(pus, ns))
        assert engine.last_timing["staging"] == "out-of-core"
        assert sum(len(r) for r in engine.last_timing["out_of_core"]["ranges"]) > 1
    finally:
        engine.max_bucket_bytes = None
