"""Zero-copy shared-state loading (substrafl_amd/remote/mapped_pickle.py): the objects equal
``pickle.load``'s -- same types, dtypes, shapes, orders, values, shared references -- large
arrays are views of the file mapping, and anything unusual falls back to ``pickle.load``.
CPU only."""

import pickle

import numpy as np
import pytest

from substrafl_amd import wire
from substrafl_amd.remote.mapped_pickle import BIG, load_mapped
from substrafl_amd.schemas import FedAvgSharedState, ScaffoldSharedState


def _same(a, b):
    assert type(a) is type(b)
    if isinstance(a, np.ndarray):
        assert a.dtype == b.dtype and a.shape == b.shape
        assert a.flags.c_contiguous == b.flags.c_contiguous and a.flags.f_contiguous == b.flags.f_contiguous
        assert a.tobytes(order="A") == b.tobytes(order="A")
        assert a.flags.writeable == b.flags.writeable
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            _same(x, y)
    elif hasattr(a, "model_dump"):
        for k in type(a).model_fields:
            _same(getattr(a, k), getattr(b, k))
    else:
        assert a == b


def _root(a):
    while isinstance(a, np.ndarray):
        a = a.base
    return a


def _layers(rng):
    big = BIG // 4 + 1000
    return [
        rng.standard_normal((big,)).astype(np.float32),  # large: mapped
        np.asfortranarray(rng.standard_normal((700, 400))),  # large, F order, fp64
        rng.standard_normal((3, 5)).astype(np.float32),  # small: copied as usual
        np.array(2.5, np.float32),  # 0-d
        np.zeros((0, 7), np.float32),  # empty
        rng.integers(-5, 5, (600_000,)).astype(np.int64),  # large int
        (rng.random(1_200_000) > 0.5),  # large bool
        rng.standard_normal((BIG,)).astype(np.float16),  # large fp16
        np.arange(10, dtype=">f4"),  # non-native byte order
    ]


@pytest.mark.parametrize("protocol", [2, 3, 4, 5])
def test_equal_to_pickle_load(tmp_path, protocol):
    rng = np.random.default_rng(protocol)
    st = FedAvgSharedState(n_samples=17, parameters_update=_layers(rng))
    p = tmp_path / "s"
    p.write_bytes(pickle.dumps(st, protocol=protocol))
    ref = pickle.loads(p.read_bytes())
    got = load_mapped(p)
    _same(got, ref)
    if protocol in (3, 4, 5):  # BINBYTES (3, 4) or in-band PickleBuffer (5) payloads: mapped
        big = got.parameters_update[0]
        assert isinstance(_root(big), memoryview)  # a view of the file mapping, not a copy
        big[0] = 123.0  # copy-on-write: the file is untouched
        assert pickle.loads(p.read_bytes()).parameters_update[0][0] != 123.0


def test_shared_references_and_scaffold(tmp_path):
    rng = np.random.default_rng(3)
    layers = _layers(rng)
    c = [a.copy() for a in layers]
    st = ScaffoldSharedState(parameters_update=layers, control_variate_update=layers, n_samples=5,
                             server_control_variate=c)
    p = tmp_path / "s"
    p.write_bytes(pickle.dumps(st))
    got = load_mapped(p)
    _same(got, pickle.loads(p.read_bytes()))
    # the same array object pickled twice (memo) comes back as one object, as with pickle.load
    assert got.parameters_update[0] is got.control_variate_update[0]


@pytest.mark.parametrize("protocol", [4, 5])
def test_wire_format_mapped(tmp_path, protocol):
    rng = np.random.default_rng(4)
    layers = _layers(rng)
    st = FedAvgSharedState(n_samples=3, parameters_update=wire.pack([layers[0], layers[2]]))  # one dtype
    p = tmp_path / "s"
    p.write_bytes(pickle.dumps(st, protocol=protocol))
    got = load_mapped(p)
    _same([np.asarray(a) for a in got.parameters_update],
          [np.asarray(a) for a in pickle.loads(p.read_bytes()).parameters_update])
    assert wire.flat_of(got.parameters_update) is not None
    assert isinstance(_root(got.parameters_update[0]._bucket.flat), memoryview)  # mapped, not copied


def test_fallbacks(tmp_path):
    # a large bytes payload that is not an array: pickle.load's exact objects (bytes, not a view)
    obj = {"blob": b"x" * (BIG + 5), "arr": np.ones(BIG, np.uint8)}
    p = tmp_path / "b"
    p.write_bytes(pickle.dumps(obj))
    got = load_mapped(p)
    assert type(got["blob"]) is bytes and got["blob"] == obj["blob"]
    assert np.array_equal(got["arr"], obj["arr"])
    # object arrays, empty file and corrupt file behave as pickle.load
    p2 = tmp_path / "o"
    p2.write_bytes(pickle.dumps(np.array([1, "a", None], dtype=object)))
    assert list(load_mapped(p2)) == [1, "a", None]
    p3 = tmp_path / "empty"
    p3.write_bytes(b"")
    with pytest.raises(EOFError):
        load_mapped(p3)
    p4 = tmp_path / "bad"
    p4.write_bytes(b"\x80\x04garbage")
    with pytest.raises(Exception) as e_ref:
        pickle.loads(p4.read_bytes())
    with pytest.raises(type(e_ref.value)):
        load_mapped(p4)
