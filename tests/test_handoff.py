"""The simulation-mode device hand-off's records (substrafl_amd/handoff.py), on the CPU: when a
record may be used (exact views of the frozen buffer, same device, unmodified source) and when it
must not be (anything else falls back to the host copy).  The copies themselves run on the GPU
(tests/test_accelerate_algo.py::test_*_handoff_*)."""

from __future__ import annotations

import gc

import numpy as np
import pytest

from substrafl_amd import handoff, runtime


class _Session:
    def __init__(self, device=0):
        self.device, self.gen = device, {}

    def generation(self, slot):
        return self.gen.get(slot, 0)


class _Tensor:
    """What record_tensor reads of a torch tensor on a GPU."""

    is_cuda = True

    def __init__(self, n, isz=4, device=0):
        self.n, self.isz, self._version = n, isz, 0
        self.device = type("D", (), {"index": device})()

    def numel(self):
        return self.n

    def element_size(self):
        return self.isz

    def data_ptr(self):
        return 0xABC000


class _Consumer:
    """Stands for an accelerated client / strategy (handoff.register)."""


@pytest.fixture()
def on():
    handoff.enable(True)
    consumers = [_Consumer(), _Consumer()]  # an accelerate_algo client and an accelerate-d strategy
    handoff.register("client", consumers[0])
    handoff.register("aggregator", consumers[1])
    yield consumers
    handoff.enable(False)
    del consumers
    gc.collect()


def _export(n=100, tag="handoff_t"):
    host = runtime.reusable_host_array(n, np.float32, tag)
    host[:] = np.arange(n, dtype=np.float32)
    return host


def _views(host, sizes=(60, 30, 10)):
    out, off = [], 0
    for k in sizes:
        out.append(host[off: off + k])
        off += k
    return out


def test_disabled_records_nothing():
    handoff.enable(False)
    host = _export()
    handoff.record_slot(host, _Session(), 1, 0x1000)
    assert handoff.lookup(_views(host), 0) is None and host.flags.writeable


def test_slot_record_lookup_and_freeze(on):
    s = _Session()
    host = _export()
    handoff.record_slot(host, s, 1, 0x1000)
    views = _views(host)  # made after the record, as the engine's per-layer outputs are
    assert not host.flags.writeable and not any(v.flags.writeable for v in views)
    with pytest.raises(ValueError):
        views[0].flags.writeable = True  # the buffer under them is frozen too
    hit = handoff.lookup(views, 0)
    assert hit is not None and hit[0] == 0x1000 and hit[1] == 400 and hit[2] is s
    # anything but exact, in-order views of the recorded bytes on the recorded device misses
    assert handoff.lookup(views, 1) is None
    assert handoff.lookup(views[:2], 0) is None
    assert handoff.lookup([views[1], views[0], views[2]], 0) is None
    assert handoff.lookup([v.copy() for v in views], 0) is None
    # the slot written again (generation), or an engine call on the device: unusable
    s.gen[1] = 5
    assert handoff.lookup(views, 0) is None
    s.gen[1] = 0
    assert handoff.lookup(views, 0) is not None
    handoff.invalidate_slots([0])
    assert handoff.lookup(views, 0) is None


def test_tensor_record_and_in_place_change(on):
    host = _export()
    t = _Tensor(100)
    handoff.record_tensor(host, t)
    views = _views(host)
    handoff.invalidate_slots([0])  # engine calls leave tensor records alone
    hit = handoff.lookup(views, 0)
    assert hit[0] == 0xABC000 and hit[2] is t
    # a client export is consumed once -- the record (and its hold on the device
    # bucket) goes with the aggregation that took it
    assert handoff.lookup(views, 0) is None and not handoff.records()
    handoff.record_tensor(host, t)
    t._version += 1  # modified in place since the export
    assert handoff.lookup(views, 0) is None
    handoff.record_tensor(_export(50, "handoff_u"), _Tensor(100))  # size mismatch: not recorded
    assert all(r["bytes"] != 200 for r in handoff.records())


def test_unfrozen_buffer_is_refused(on):
    host = _export()
    handoff.record_slot(host, _Session(), 1, 0x1000)
    views = _views(host)
    base = views[0].base
    base.flags.writeable = True  # a user who thaws the buffer may have written into it
    assert handoff.lookup(views, 0) is None


def test_recycled_buffer_is_thawed_and_refused_until_recorded_again(on):
    host = _export(tag="handoff_r")
    ptr = host.__array_interface__["data"][0]
    handoff.record_slot(host, _Session(), 1, 0x1000)
    del host
    gc.collect()
    again = runtime.reusable_host_array(100, np.float32, "handoff_r")
    assert again.__array_interface__["data"][0] == ptr and again.flags.writeable
    assert handoff.lookup(_views(again), 0) is None
    handoff.record_slot(again, _Session(), 1, 0x2000)
    assert handoff.lookup(_views(again), 0)[0] == 0x2000


def test_record_goes_with_its_buffer(on):
    buf = np.empty(100, np.float32)  # not a pooled buffer: dies with its last view
    handoff.record_tensor(buf[:100], _Tensor(100))
    start = buf.__array_interface__["data"][0]
    assert any(r["start"] == start for r in handoff.records())
    del buf
    gc.collect()
    assert not any(r["start"] == start for r in handoff.records())


def test_stable_slot_survives_engine_calls_not_writes(on):
    """A stable slot (written only by the runtime's own copies) outlives the invalidation of an
    engine call on its device -- the next Scaffold call reads it back as the clients' c -- and is
    refused once the slot is written again (its generation)."""
    s = _Session()
    host = _export(tag="handoff_s")
    handoff.record_slot(host, s, 12, 0x3000, stable=True)
    views = _views(host)
    handoff.invalidate_slots([0])
    assert handoff.lookup(views, 0)[0] == 0x3000
    s.gen[12] = 1
    assert handoff.lookup(views, 0) is None


def test_records_only_for_a_live_consumer():
    """VERDICT r05 "Next 3": the engine's outputs are recorded (and frozen) only while an
    accelerated client lives to take them on the device, a client's exports only while an
    accelerated strategy lives -- the reference's own algorithms next to an accelerated strategy
    get writable arrays, exactly the reference's (torch.from_numpy warns on read-only ones)."""
    handoff.enable(True)
    try:
        assert handoff.consumers() == {"client": 0, "aggregator": 0}
        out = _export(tag="handoff_c1")
        handoff.record_slot(out, _Session(), 1, 0x1000)  # no accelerated client: not recorded
        exp = _export(tag="handoff_c2")
        handoff.record_tensor(exp, _Tensor(100))  # no accelerated strategy: not recorded
        assert out.flags.writeable and exp.flags.writeable and not handoff.records()
        strategy = _Consumer()
        handoff.register("aggregator", strategy)
        handoff.record_slot(out, _Session(), 1, 0x1000)
        assert out.flags.writeable  # still no client consumer for the engine's outputs
        handoff.record_tensor(exp, _Tensor(100))
        assert not exp.flags.writeable and len(handoff.records()) == 1
        client = _Consumer()
        handoff.register("client", client)
        handoff.record_slot(out, _Session(), 1, 0x1000)
        assert not out.flags.writeable and len(handoff.records()) == 2
        # the experiment's strategy and clients released: every record and pooled buffer goes
        del strategy
        gc.collect()
        assert len(handoff.records()) == 2
        del client
        gc.collect()
        assert handoff.consumers() == {"client": 0, "aggregator": 0}
        assert not handoff.records() and not runtime._host_cache
        with pytest.raises(ValueError):
            handoff.register("server", _Consumer())
    finally:
        handoff.enable(False)
