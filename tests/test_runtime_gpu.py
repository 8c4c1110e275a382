"""GPU tests of the native session and the engine's staging bookkeeping (ADVICE r01 findings):
error paths of the staging / fetch pipelines, the write generation that guards rows prestaged
by ``ingest``, the pairwise workspace of Scaffold with differently shaped delta / cv layers, the
HBM budget of the out-of-core switch, and the host-side server-control-variate check."""

import numpy as np
import pytest

from oracle import fedavg_reference_structure, scaffold_reference_structure

pytestmark = pytest.mark.gpu


def _bits(a):
    a = np.asarray(a)
    return a.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize])


def _assert_same(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert g.dtype == r.dtype and g.shape == r.shape
        assert np.array_equal(_bits(g), _bits(r))


@pytest.fixture(scope="module")
def lib():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from substrafl_amd import _native

    return _native.load()


@pytest.mark.parametrize("fail_at", [1, 2, 7, 40])
def test_injected_copy_failure_stage_and_fetch(lib, fail_at):
    """A copy failing in the middle of a stage / fetch returns FEDAGG_EHIP after the pack and
    copy-out tasks already handed to the workers have finished (no use of the call's flags or of
    the caller's buffers after the return); the session stays usable."""
    from substrafl_amd._native import NativeLibraryError
    from substrafl_amd.runtime import Session

    rng = np.random.default_rng(fail_at)
    K = 3
    rows = [[rng.standard_normal(n).astype(np.float32) for n in (1_000_003, 7, 2_000_000)] for _ in range(K)]
    M = 3_000_010
    ld = (M + 127) // 128 * 128
    s = Session(0, threads=4)
    try:
        s.set("chunk_bytes", 1 << 18)
        d = s.buffer(0, K * ld * 4)
        s.set("fail_copy_after", fail_at)
        with pytest.raises(NativeLibraryError, match="injected"):
            s.stage(d, ld * 4, rows)
        s.set("fail_copy_after", 0)
        s.stage(d, ld * 4, rows)
        got = np.empty(K * ld, np.float32)
        s.set("fail_copy_after", min(fail_at, 20))  # the fetch moves 36 MB in ~36 super-chunk copies
        with pytest.raises(NativeLibraryError, match="injected"):
            s.fetch(d, got)
        s.set("fail_copy_after", 0)
        s.fetch(d, got)
        for k in range(K):
            assert np.array_equal(got[k * ld: k * ld + M], np.concatenate(rows[k]))
    finally:
        s.close()


def test_prestaged_rows_invalidated_by_another_engine(lib, tmp_path):
    """Rows staged by engine A's ingest live in the per-GPU session every engine shares; engine B
    aggregating on the same GPU overwrites them.  A's next call must notice (write generation of
    the slot) and stage again: bit-exact, not B's bytes."""
    from substrafl_amd.engine import AggregationEngine
    from substrafl_amd.remote import PickleSerializer
    from substrafl_amd.schemas import FedAvgSharedState

    rng = np.random.default_rng(5)
    shapes = [(500, 40), (1,), (3000,)]
    K = 4
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 100, K)]
    paths = []
    for k in range(K):
        p = tmp_path / f"s{k}.pkl"
        PickleSerializer().save(FedAvgSharedState(n_samples=ns[k], parameters_update=pus[k]), p)
        paths.append(p)
    a, b = AggregationEngine(0), AggregationEngine(0)
    states = a.ingest(paths, "fedavg", PickleSerializer().load)
    assert a.last_ingest["prestaged_clients"] == K
    other = [[(x * 3 + 1).astype(np.float32) for x in pu] for pu in pus]
    _assert_same(b.fedavg(other, ns), fedavg_reference_structure(other, ns))
    got = a.fedavg([list(s.parameters_update) for s in states], [s.n_samples for s in states])
    assert not a.last_timing.get("prestaged")
    _assert_same(got, fedavg_reference_structure(pus, ns))
    # and without interference the prestaged rows are used
    states = a.ingest(paths, "fedavg", PickleSerializer().load)
    got = a.fedavg([list(s.parameters_update) for s in states], [s.n_samples for s in states])
    assert a.last_timing.get("prestaged")
    _assert_same(got, fedavg_reference_structure(pus, ns))


def test_scaffold_ws_sized_for_cv_layers(lib):
    """Delta and control-variate layers of different shapes (two kernel passes sharing one
    pairwise workspace): the control variates carry more numel == 1 layers than the deltas and
    K > 64 forces the separate pairwise path -- the workspace must fit the larger of the two."""
    from substrafl_amd.engine import AggregationEngine

    rng = np.random.default_rng(8)
    K, L = 70, 20
    d_shapes = [(5,)] * (L - 1) + [(1,)]
    c_shapes = [(1,)] * (L - 1) + [(9,)]
    pus = [[rng.standard_normal(s).astype(np.float32) for s in d_shapes] for _ in range(K)]
    cvs = [[rng.standard_normal(s).astype(np.float32) for s in c_shapes] for _ in range(K)]
    c = [rng.standard_normal(s).astype(np.float32) for s in c_shapes]
    ns = [int(v) for v in rng.integers(1, 1000, K)]
    mism, new_c, avg = AggregationEngine(0).scaffold(pus, cvs, [c] * K, ns, 0.3)
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.3)
    assert mism == 0
    _assert_same(new_c, rc)
    _assert_same(avg, ra)


def test_held_bytes_counts_only_reused_slots(lib):
    """After a Scaffold call the session still holds its control-variate buffers; a FedAvg call's
    out-of-core budget counts only the bucket / output / workspace slots it reuses."""
    from substrafl_amd.engine import AggregationEngine

    rng = np.random.default_rng(1)
    K = 3
    shapes = [(100_000,), (1,)]
    mk = lambda: [rng.standard_normal(s).astype(np.float32) for s in shapes]  # noqa: E731
    eng = AggregationEngine(0)
    eng.scaffold([mk() for _ in range(K)], [mk() for _ in range(K)], [mk()] * K, [1, 2, 3], 1.0)
    s = eng.session()
    fed = s.held_bytes((eng._B_BUCKET, eng._B_OUT, eng._B_WS))
    assert 0 < fed < s.held_bytes()
    assert s.held_bytes((eng._B_CV,)) >= K * 100_001 * 4


def test_stage_check_counts_like_assert_array_equal(lib):
    """Session.stage_check: one copy staged, the others compared by value on the host (+0 == -0,
    NaN == NaN), over a byte range too."""
    from substrafl_amd.runtime import Session

    rng = np.random.default_rng(2)
    for dt in (np.float32, np.float64):
        base = [rng.standard_normal(n).astype(dt) for n in (300_001, 5, 1 << 20)]
        base[0][:7] = np.nan
        base[1][:] = 0.0
        rows = [base] + [[x.copy() for x in base] for _ in range(4)]
        rows[2][1][:] = -0.0
        rows[3][2][12345] += 1
        rows[4][0][100:110] = 5.0
        rows[4][0][3] = -np.nan
        want = sum(int(np.sum(~((np.concatenate(r) == np.concatenate(base))
                                | (np.isnan(np.concatenate(r)) & np.isnan(np.concatenate(base))))))
                   for r in rows[1:])
        s = Session(0, threads=4)
        try:
            M = sum(x.size for x in base)
            isz = np.dtype(dt).itemsize
            d = s.buffer(0, M * isz)
            assert s.stage_check(d, rows, dt) == want
            got = np.empty(M, dt)
            s.fetch(d, got)
            assert np.array_equal(_bits(got), _bits(np.concatenate(base)))
            lo, hi = 90, 300_050  # a parameter range (element-aligned bytes)
            d2 = s.buffer(1, (hi - lo) * isz)
            n = s.stage_check(d2, rows, dt, byte_range=(lo * isz, hi * isz))
            sub = lambda r: np.concatenate(r)[lo:hi]  # noqa: E731
            assert n == sum(int(np.sum(~((sub(r) == sub(base)) | (np.isnan(sub(r)) & np.isnan(sub(base))))))
                            for r in rows[1:])
        finally:
            s.close()


def test_multi_device_host_c_check(lib):
    """MultiDeviceEngine (repeated GPU 0): the c copies are checked on the host per parameter
    range while one copy is staged; a mismatch is counted once."""
    from substrafl_amd.multi_device import MultiDeviceEngine

    rng = np.random.default_rng(4)
    K = 5
    shapes = [(40_000,), (1,), (123, 7)]
    mk = lambda: [rng.standard_normal(s).astype(np.float32) for s in shapes]  # noqa: E731
    pus, cvs, c = [mk() for _ in range(K)], [mk() for _ in range(K)], mk()
    ns = [int(v) for v in rng.integers(1, 100, K)]
    rows = [[a.copy() for a in c] for _ in range(K)]
    eng = MultiDeviceEngine([0, 0, 0], max_shard_bytes=400_000)
    mism, new_c, avg = eng.scaffold(pus, cvs, rows, ns, 0.8)
    assert mism == 0
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.8)
    _assert_same(new_c, rc)
    _assert_same(avg, ra)
    rows[2][0][39_999] += 1
    assert eng.scaffold(pus, cvs, rows, ns, 0.8)[0] == 1
