"""Flat-bucket wire format (substrafl_amd.wire): pickles stay plain pickles,
layers stay np.ndarrays, results are bit-identical to per-layer arrays."""

import pickle

import numpy as np
import pytest

from oracle import fedavg_reference_structure
from substrafl_amd import wire
from substrafl_amd.layout import BucketLayout
from substrafl_amd.schemas import FedAvgAveragedState, FedAvgSharedState

SHAPES = [(64, 33), (33,), (1,), (5, 1), ()]


def _layers(seed=0, dtypes=None):
    rng = np.random.default_rng(seed)
    dtypes = dtypes or [np.float32] * len(SHAPES)
    return [np.asarray(rng.standard_normal(s)).astype(d) for s, d in zip(SHAPES, dtypes)]


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()


@pytest.mark.parametrize("protocol", [2, 3, 4, 5])
def test_round_trip_every_protocol(protocol):
    arrs = _layers(dtypes=[np.float32, np.float64, np.float16, np.int64, np.float32])
    st = FedAvgSharedState(n_samples=7, parameters_update=wire.pack(arrs))
    back = pickle.loads(pickle.dumps(st, protocol=protocol))
    pu = back.parameters_update
    assert all(isinstance(a, np.ndarray) for a in pu)
    assert all(_same(a, b) for a, b in zip(pu, arrs))
    assert len({id(a._bucket) for a in pu}) == 1  # still one buffer
    assert all(a.flags.writeable for a in pu)
    pu[0][0, 0] = 123.0  # writable, and only this state's buffer changes
    assert arrs[0][0, 0] != 123.0


def test_out_of_band_buffers():
    arrs = _layers()
    st = FedAvgSharedState(n_samples=3, parameters_update=wire.pack(arrs))
    bufs = []
    head = pickle.dumps(st, protocol=5, buffer_callback=bufs.append)
    assert len(bufs) == 1 and len(head) < 1024
    back = pickle.loads(head, buffers=bufs)
    assert all(_same(a, b) for a, b in zip(back.parameters_update, arrs))


def test_one_payload_per_client():
    arrs = [np.ones((1000,), np.float32) for _ in range(40)]
    flat_size = len(pickle.dumps(wire.pack(arrs)))
    per_layer = len(pickle.dumps(arrs))
    assert flat_size < per_layer  # one buffer + 40 small records instead of 40 array pickles
    assert flat_size >= 40 * 4000


def test_arithmetic_returns_plain_arrays_and_reference_bits():
    K = 5
    ns = [3, 9, 1, 4000, 17]
    plain = [_layers(seed=k) for k in range(K)]
    flat = [wire.pack(p) for p in plain]
    assert type(flat[0][0] * 2.0) is np.ndarray and type(flat[0][0][1:3]) is wire.BucketArray
    assert flat[0][0][1:3]._bucket is None  # a slice is not a bucket member
    for a, b in zip(fedavg_reference_structure(flat, ns), fedavg_reference_structure(plain, ns)):
        assert _same(a, b)


def test_flat_of():
    f = np.arange(2 * 3 + 1 + 13, dtype=np.float32)
    v = wire.bucket_views(f, [(2, 3), (1,), (13,)])
    flat = wire.flat_of(v)
    assert flat is not None and flat.size == 20 and np.shares_memory(flat, f)
    assert wire.flat_of(v[1:]).size == 14
    assert wire.flat_of([v[0], v[2]]) is None  # gap
    assert wire.flat_of(list(reversed(v))) is None
    assert wire.flat_of([np.zeros(3, np.float32)]) is None
    mixed = wire.pack([np.zeros(3, np.float32), np.zeros(2, np.float64)])
    assert wire.flat_of(mixed) is None


def test_layout_unpack_gives_one_bucket_and_scalars():
    lay = BucketLayout(list(range(len(SHAPES))), SHAPES, np.float32)
    out = np.arange(lay.M, dtype=np.float32)
    got = lay.unpack(out, wire=True)
    assert wire.flat_of([a for _, a in lay.unpack(out)][:-1]) is None  # default: plain views
    arrs = [a for _, a in got]
    assert not isinstance(arrs[-1], np.ndarray) and isinstance(arrs[-1], np.float32)  # 0-d -> scalar
    assert wire.flat_of(arrs[:-1]) is not None
    avg = FedAvgAveragedState(avg_parameters_update=arrs[:-1])
    back = pickle.loads(pickle.dumps(avg))
    assert all(_same(a, b) for a, b in zip(back.avg_parameters_update, arrs[:-1]))


def test_small_payload_is_copied():
    st = wire.pack([np.zeros(2, np.float32)])
    back = pickle.loads(pickle.dumps(st, protocol=4))
    back[0][0] = 1.0
    assert back[0].flags.writeable
