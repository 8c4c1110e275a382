"""Property tests (hypothesis) of the host-side byte plumbing: bucket layout, flat wire format,
shard bounds and the pairwise restatement.  CPU only, seconds."""

import pickle

import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from oracle import numpy_pairwise_sum
from substrafl_amd import wire
from substrafl_amd.layout import BucketLayout
from substrafl_amd.sharding import SHARD_ALIGN, pack_range, shard_bounds

shapes = st.lists(st.lists(st.integers(0, 7), min_size=0, max_size=3).map(tuple), min_size=1, max_size=8)
dtypes = st.sampled_from([np.float16, np.float32, np.float64, np.int32, np.int64, np.uint8, np.bool_])


def _arr(rng, shape, dt):
    a = rng.standard_normal(shape) * 100
    return a.astype(dt)


@settings(max_examples=60, deadline=None)
@given(shapes, st.integers(0, 2**32 - 1))
def test_layout_pack_unpack_round_trip(shp, seed):
    rng = np.random.default_rng(seed)
    layers = [_arr(rng, s, np.float32) for s in shp]
    lay = BucketLayout(list(range(len(shp))), shp, np.float32)
    assert lay.ld % (256 // 4) == 0 and lay.ld >= lay.M
    row = np.full(lay.ld, np.nan, np.float32)
    lay.pack_row(layers, row)
    back = dict(lay.unpack(row))
    for i, a in enumerate(layers):
        b = np.asarray(back[i])
        assert b.shape == a.shape and b.tobytes() == a.tobytes()
    assert sorted(int(i) for i in lay.pairwise_idx) == [s.offset for s in lay.segments if s.numel == 1]


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.lists(st.integers(0, 6), max_size=3).map(tuple), dtypes), min_size=1, max_size=6),
       st.integers(0, 2**32 - 1), st.sampled_from([2, 4, 5]))
def test_wire_round_trip_any_dtypes(spec, seed, protocol):
    rng = np.random.default_rng(seed)
    layers = [_arr(rng, s, d) for s, d in spec]
    packed = wire.pack(layers)
    back = pickle.loads(pickle.dumps(packed, protocol=protocol))
    for a, b in zip(layers, back):
        assert b.dtype == a.dtype and b.shape == a.shape and b.tobytes() == a.tobytes()
    if len({a.dtype for a in layers}) == 1:
        f = wire.flat_of(back)
        assert f is not None and f.size == sum(a.size for a in layers)


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 10**9), st.integers(1, 64))
def test_shard_bounds_partition(M, world):
    b = shard_bounds(M, world)
    assert len(b) == world and b[0][0] == 0 and b[-1][1] == M
    for (lo, hi), (lo2, _) in zip(b, b[1:]):
        assert lo <= hi == lo2
    for lo, hi in b:
        assert lo % SHARD_ALIGN == 0 or lo == M


@settings(max_examples=40, deadline=None)
@given(shapes, st.integers(1, 4), st.integers(0, 2**32 - 1))
def test_pack_range_concatenates_to_the_row(shp, world, seed):
    rng = np.random.default_rng(seed)
    layers = [_arr(rng, s, np.float32) for s in shp]
    lay = BucketLayout(list(range(len(shp))), shp, np.float32)
    full = np.zeros(lay.ld, np.float32)
    lay.pack_row(layers, full)
    parts = []
    for lo, hi in shard_bounds(lay.M, world, align=4):
        dst = np.zeros(max(1, hi - lo), np.float32)
        pack_range(lay, layers, dst, lo, hi)
        parts.append(dst[: hi - lo])
    assert np.concatenate(parts).tobytes() == full[: lay.M].tobytes()


@settings(max_examples=100, deadline=None)
@given(st.integers(0, 600), st.integers(0, 2**32 - 1), st.sampled_from([np.float32, np.float64]))
def test_pairwise_restatement_equals_numpy_sum(n, seed, dt):
    x = (np.random.default_rng(seed).standard_normal(n) * 1e3).astype(dt)
    got = numpy_pairwise_sum(x) if n else dt(0.0)
    ref = np.add.reduce(x) if n else dt(0.0)
    assert np.asarray(dt(0.0) + got).tobytes() == np.asarray(ref).tobytes()


@settings(max_examples=80, deadline=None)
@given(st.integers(0, 5_000_000), st.integers(1, 9), st.integers(1, 64), st.one_of(st.none(), st.integers(1, 10**8)))
def test_multi_device_plan_partitions_the_bucket(M, G, bytes_per_elem, cap):
    """MultiDeviceEngine.plan_ranges: the sub-ranges of all shards tile [0, M) in order, every
    boundary except M is 512-element aligned, and no sub-range exceeds the HBM cap (or the
    512-element minimum step)."""
    from substrafl_amd.multi_device import MultiDeviceEngine
    from substrafl_amd.sharding import SHARD_ALIGN

    eng = MultiDeviceEngine(list(range(G)), max_shard_bytes=cap or 10**15)
    plan = eng.plan_ranges(M, bytes_per_elem)
    assert len(plan) == G
    flat = [r for shard in plan for r in shard]
    if M == 0:
        assert flat == []
        return
    assert flat[0][0] == 0 and flat[-1][1] == M
    for (a, b), (c, _) in zip(flat, flat[1:]):
        assert b == c and b % SHARD_ALIGN == 0
    limit = max(SHARD_ALIGN, (cap or 10**15) // bytes_per_elem)
    assert all(0 < b - a <= limit for a, b in flat)
