"""Per-client staging into the tile-interleaved layout (``fedagg_session_stage_tiled_row``) and
the ingest path that uses it: clients staged one at a time, in any order, land exactly where
``fedagg_session_stage_tiled`` puts them, and a FedAvg over buckets staged by ``ingest`` is
bit-identical to the reference arithmetic (fed_avg.py:217-222, oracle.fedavg_reference_structure)."""

import numpy as np
import pytest

from oracle import fedavg_reference_structure

pytestmark = pytest.mark.gpu


def _same(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        g, r = np.asarray(g), np.asarray(r)
        assert g.dtype == r.dtype and g.shape == r.shape
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32))


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


@pytest.mark.parametrize("K,tv,chunk", [(1, 2048, 1 << 18), (5, 8192, 1 << 17), (33, 2048, 1 << 20), (64, 8192, 1 << 22)])
def test_stage_tiled_row_places_like_stage_tiled(torch_gpu, K, tv, chunk):
    from substrafl_amd.engine import tiled_elems, tiled_index
    from substrafl_amd.runtime import Session

    rng = np.random.default_rng(K)
    sizes = (70_001, 1, 3, 2 * tv * 4 + 5)  # ragged segments, a tail tile
    rows = [[rng.standard_normal(n).astype(np.float32) for n in sizes] for _ in range(K)]
    M = sum(sizes)
    n = tiled_elems("f32", K, M, tv)
    s = Session(0, threads=4)
    try:
        s.set("chunk_bytes", chunk)
        a = s.buffer(0, n * 4)
        b = s.buffer(1, n * 4)
        s.stage_tiled(a, tv * 16, rows)
        for k in rng.permutation(K):
            s.stage_tiled_row(b, tv * 16, K, int(k), rows[k])
        ga, gb = np.empty(n, np.float32), np.empty(n, np.float32)
        s.fetch(a, ga)
        s.fetch(b, gb)
        e = np.arange(M)
        for k in range(K):
            idx = tiled_index("f32", K, k, e, tv)
            want = np.concatenate(rows[k])
            assert np.array_equal(gb[idx], want) and np.array_equal(ga[idx], want)
    finally:
        s.close()


def test_stage_tiled_row_rejects_and_recovers(torch_gpu):
    from substrafl_amd._native import NativeLibraryError
    from substrafl_amd.engine import tiled_elems, tiled_index
    from substrafl_amd.runtime import Session

    rng = np.random.default_rng(3)
    row = [rng.standard_normal(300_000).astype(np.float32)]
    K, tv = 4, 2048
    n = tiled_elems("f32", K, row[0].size, tv)
    s = Session(0, threads=2)
    try:
        s.set("chunk_bytes", 1 << 17)
        d = s.buffer(0, n * 4)
        for bad in ((tv * 16, K, K), (tv * 16, K, -1), (24, K, 0), (1 << 18, K, 0)):
            with pytest.raises(NativeLibraryError):
                s.stage_tiled_row(d, bad[0], bad[1], bad[2], row)
        s.set("fail_copy_after", 3)
        with pytest.raises(NativeLibraryError, match="injected"):
            s.stage_tiled_row(d, tv * 16, K, 2, row)
        s.set("fail_copy_after", 0)
        s.stage_tiled_row(d, tv * 16, K, 2, row)
        got = np.empty(n, np.float32)
        s.fetch(d, got)
        assert np.array_equal(got[tiled_index("f32", K, 2, np.arange(row[0].size), tv)], row[0])
    finally:
        s.close()


def _save_states(tmp_path, pus, ns, wire=False):
    from substrafl_amd.remote import PickleSerializer
    from substrafl_amd.schemas import FedAvgSharedState

    paths = []
    for k, (pu, n) in enumerate(zip(pus, ns)):
        if wire:  # flat wire format: the layers are views of one buffer (one segment per client)
            from substrafl_amd.wire import pack

            pu = pack(pu)
        p = tmp_path / f"c{k}.pkl"
        PickleSerializer().save(FedAvgSharedState(n_samples=n, parameters_update=pu), p)
        paths.append(p)
    return paths


@pytest.mark.parametrize("K,wire", [(3, False), (33, True), (40, False)])
def test_ingest_tiled_fedavg_bit_exact(torch_gpu, tmp_path, K, wire):
    """Ingest stages every client into the tile-interleaved bucket as it is loaded; the next
    FedAvg uses those tiles (prestaged, layout "tiles") and matches the reference bit for bit,
    numel==1 layers (NumPy pairwise path) included."""
    from substrafl_amd.engine import AggregationEngine
    from substrafl_amd.remote import PickleSerializer

    rng = np.random.default_rng(K)
    shapes = [(300, 41), (1,), (7,), (1, 1), (20_011,)]
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 10_000, K)]
    paths = _save_states(tmp_path, pus, ns, wire)
    eng = AggregationEngine(0)
    eng.tiled = True
    states = eng.ingest(paths, "fedavg", PickleSerializer().load)
    assert eng.last_ingest["prestaged_clients"] == K
    got = eng.fedavg([list(s.parameters_update) for s in states], [s.n_samples for s in states])
    assert eng.last_timing.get("prestaged") and eng.last_timing["layout"] == "tiles"
    _same(got, fedavg_reference_structure(pus, ns))
    # the same engine with rows: the record of a tiled ingest is not taken for rows and back
    eng.tiled = False
    states = eng.ingest(paths, "fedavg", PickleSerializer().load)
    got = eng.fedavg([list(s.parameters_update) for s in states], [s.n_samples for s in states])
    assert eng.last_timing.get("prestaged") and eng.last_timing["layout"] == "rows"
    _same(got, fedavg_reference_structure(pus, ns))


def test_ingest_tiled_invalidated_by_another_engine(torch_gpu, tmp_path):
    from substrafl_amd.engine import AggregationEngine
    from substrafl_amd.remote import PickleSerializer

    rng = np.random.default_rng(9)
    K, shapes = 6, [(4000,), (1,), (123, 5)]
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 100, K)]
    paths = _save_states(tmp_path, pus, ns)
    a, b = AggregationEngine(0), AggregationEngine(0)
    a.tiled = True
    states = a.ingest(paths, "fedavg", PickleSerializer().load)
    other = [[(x * 3 + 1).astype(np.float32) for x in pu] for pu in pus]
    _same(b.fedavg(other, ns), fedavg_reference_structure(other, ns))
    got = a.fedavg([list(s.parameters_update) for s in states], [s.n_samples for s in states])
    assert not a.last_timing.get("prestaged") and a.last_timing["layout"] == "tiles"
    _same(got, fedavg_reference_structure(pus, ns))


def test_ingest_auto_layout_follows_recommendation(torch_gpu, tmp_path):
    """auto: the ingest stages tiles exactly where the library recommends them (here a small
    bucket: rows), and the FedAvg uses what the ingest staged."""
    from substrafl_amd.engine import AggregationEngine, tiled_recommended
    from substrafl_amd.remote import PickleSerializer

    rng = np.random.default_rng(1)
    K, shapes = 40, [(10_000,), (1,)]
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 100, K)]
    eng = AggregationEngine(0)
    eng.tiled = "auto"
    states = eng.ingest(_save_states(tmp_path, pus, ns), "fedavg", PickleSerializer().load)
    got = eng.fedavg([list(s.parameters_update) for s in states], [s.n_samples for s in states])
    want = "tiles" if tiled_recommended("f32", K, 10_001) else "rows"
    assert eng.last_timing.get("prestaged") and eng.last_timing["layout"] == want
    _same(got, fedavg_reference_structure(pus, ns))
