import numpy as np

from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(0)
    shapes = [(3, 5), (1,), (), (7,), (2, 1, 3), (1, 1)]
    layers = [np.asarray(rng.standard_normal(s), dtype=np.float32) for s in shapes]
    lay = BucketLayout(range(len(shapes)), shapes, np.float32)
    assert lay.M == 15 + 1 + 1 + 7 + 6 + 1
    assert lay.ld % 64 == 0 and lay.ld >= lay.M
    assert list(lay.pairwise_idx) == [15, 16, 30]
    row = np.zeros(lay.ld, np.float32)
    lay.pack_row(layers, row)
    back = lay.unpack(row)
    for (li, a), ref in zip(back, layers):
        if ref.ndim == 0:
            assert not isinstance(a, np.ndarray) and a == ref
        else:
            assert a.shape == ref.shape and np.array_equal(a, ref)


def test_row_alignment_per_dtype():
    for dt, per in ((np.float32, 64), (np.float64, 32), (np.float16, 128)):
        lay = BucketLayout([0], [(1000,)], dt)
        assert lay.ld % per == 0 and lay.ld * np.dtype(dt).itemsize % 256 == 0


def test_synthetic_shapes_sum_to_M():
    for M in (1000, 25_000_000, 125_000_000, 350_000_000):
        shapes = synthetic_state_dict_shapes(M)
        assert sum(int(np.prod(s)) for s in shapes) == M
        assert shapes[-1] == (1,)
