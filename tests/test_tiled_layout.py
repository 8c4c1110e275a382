"""Tile-interleaved client buckets (``fedagg_fedavg_tiled_{f32,bf16}``, engine.TiledFedAvgPlan):
tile t of client k at tile ``t * K + k``, same kernel arithmetic as the row layout, so the
results are bit-identical to the oracle (fed_avg.py:217-222) -- partial last tiles, element
remainders, numel == 1 layers (fused patch and the separate pairwise path) and more clients than
one launch takes (K > 128) included."""

import ctypes

import numpy as np
import pytest

from oracle import fedavg_reference_structure


def _bits(a):
    a = np.asarray(a)
    return a.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize])


# ---------------------------------------------------------------------------------------------
# layout arithmetic and argument checks (CPU)
# ---------------------------------------------------------------------------------------------
TILES = [("f32", 8192), ("f32", 2048), ("bf16", 4096)]
L_OF = {"f32": 4, "bf16": 8}


@pytest.mark.parametrize("kind,tv", TILES)
@pytest.mark.parametrize("K,M", [(1, 5), (3, 70_001), (7, 300_000)])
def test_tiled_index_is_a_bijection_into_the_buffer(kind, tv, K, M):
    from substrafl_amd import engine

    n = engine.tiled_elems(kind, K, M, tv)
    e = np.arange(M)
    pos = np.concatenate([engine.tiled_index(kind, K, k, e, tv) for k in range(K)])
    assert pos.min() >= 0 and pos.max() < n
    assert np.unique(pos).size == pos.size
    # a client's elements keep their order inside a tile
    L = L_OF[kind]
    p0 = engine.tiled_index(kind, K, 0, e, tv)
    inside = (e[1:] // (tv * L)) == (e[:-1] // (tv * L))
    assert np.all(np.diff(p0)[inside] == 1)


def test_tiled_entry_rejects_a_foreign_tile():
    from substrafl_amd import _native

    lib = _native.load()
    w = (ctypes.c_float * 1)(1.0)
    idx = (ctypes.c_uint64 * 1)(0)
    assert lib.fedagg_fedavg_tiled_f32(256, w, 1, 1024, 4096, idx, 0, None, 256, None) == -1
    assert b"tile must be" in lib.fedagg_last_error()
    assert lib.fedagg_fedavg_tiled_f32(256, w, 1, 1024, 1024, idx, 0, None, 256, None) == -1
    assert lib.fedagg_fedavg_tiled_bf16(256, w, 1, 1024, 8192, idx, 0, None, 256, None) == -1
    assert lib.fedagg_fedavg_tiled_f32(None, w, 1, 1024, 8192, idx, 0, None, 256, None) == -1
    # recommended exactly where the row layout's kernel walks the same tile (>= 32 clients, large buckets)
    assert lib.fedagg_fedavg_tile_vectors_f32(64, 125_000_000) == _native.FEDAGG_TILE_VECTORS_F32
    assert lib.fedagg_fedavg_tile_vectors_bf16(128, 350_000_000) == _native.FEDAGG_TILE_VECTORS_BF16
    assert lib.fedagg_fedavg_tile_vectors_f32(64, 1_000_000) == 0  # another tile for 64 small buckets
    # below 32 clients the layout measured no faster (C2): recommended only with the tiled_few knob
    assert lib.fedagg_fedavg_tile_vectors_f32(8, 25_000_000) == 0
    assert lib.fedagg_tune(b"tiled_few", 1) == 0
    try:
        assert lib.fedagg_fedavg_tile_vectors_f32(8, 25_000_000) == _native.FEDAGG_TILE_VECTORS_F32_FEW
        assert lib.fedagg_fedavg_tile_vectors_f32(8, 1_000_000) == 0  # too few tiles
    finally:
        assert lib.fedagg_tune(b"tiled_few", 0) == 0


# ---------------------------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------------------------
def _case(rng, K, M, P, bf16):
    """K clients of M elements as layers, P of them numel == 1 (scattered), values N(0,1) x 10^U."""
    # numel == 1 layers at cuts >= 3 apart: every other layer has >= 2 elements
    cuts = np.sort(rng.choice(np.arange(2, M - 3, 3), size=P, replace=False)) if P else np.array([], int)
    shapes, pos = [], 0
    for c in cuts:
        if c > pos:
            shapes.append((int(c - pos),))
        shapes.append((1,))
        pos = c + 1
    if M > pos:
        shapes.append((int(M - pos),))
    pus = []
    for _ in range(K):
        layers = [(rng.standard_normal(s) * 10.0 ** rng.integers(-3, 3)).astype(np.float32) for s in shapes]
        if bf16:
            layers = [(a.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32) for a in layers]
        pus.append(layers)
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    return shapes, pus, ns


def _tiled_device(torch, kind, pus, M, tv):
    from substrafl_amd import engine

    K = len(pus)
    dt = torch.bfloat16 if kind == "bf16" else torch.float32
    buf = torch.zeros(engine.tiled_elems(kind, K, M, tv), dtype=dt, device="cuda")
    L = L_OF[kind]
    tiles = buf.numel() // (K * tv * L)
    for k, layers in enumerate(pus):
        row = torch.zeros(tiles * tv * L, dtype=torch.float32)
        row[:M] = torch.from_numpy(np.concatenate([a.ravel() for a in layers]))
        engine.tiled_client_view(buf, kind, K, k, tv).copy_(row.view(tiles, tv * L).to(dt).cuda())
    return buf


@pytest.mark.gpu
@pytest.mark.parametrize("kind,tv", TILES)
@pytest.mark.parametrize("K,tiles,P", [(1, 1, 0), (3, 2, 1), (9, 3, 5), (40, 2, 16), (20, 2, 17), (130, 1, 3)])
def test_tiled_fedavg_bit_exact(kind, tv, K, tiles, P):
    import torch

    from substrafl_amd import engine
    from substrafl_amd.layout import BucketLayout

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    rng = np.random.default_rng(K * 31 + tiles + P + tv)
    L = L_OF[kind]
    M = (tiles - 1) * tv * L + int(rng.integers(1, tv * L))  # a partial last tile, any remainder mod L
    shapes, pus, ns = _case(rng, K, M, P, kind == "bf16")
    lay = BucketLayout(range(len(shapes)), shapes, np.float32)
    assert lay.M == M and lay.pairwise_idx.size == P
    buf = _tiled_device(torch, kind, pus, M, tv)
    out = torch.full((lay.ld,), np.nan, dtype=torch.float32, device="cuda")
    w = engine.fedavg_weights(ns, kind)
    engine.TiledFedAvgPlan(kind, buf, K, w, M, out, lay.pairwise_idx, tv=tv).launch()
    torch.cuda.synchronize()
    got = out[:M].cpu().numpy()
    ref = np.concatenate([r.ravel() for r in fedavg_reference_structure(pus, ns)])
    assert np.array_equal(_bits(got), _bits(ref))


@pytest.mark.gpu
def test_tiled_matches_rows_at_the_recommended_shape():
    """At a recommended shape (32 fp32 clients, >= 2048 tiles) the tiled kernel and the row
    layout's kernel give the same bits (the row kernel is pinned to the oracle elsewhere)."""
    import torch

    from substrafl_amd import engine
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes

    K, M = 32, 34_000_000
    assert engine.tiled_recommended("f32", K, M)
    shapes = synthetic_state_dict_shapes(M)
    lay = BucketLayout(list(range(len(shapes))), shapes, np.float32)
    g = torch.Generator(device="cuda")
    rows = torch.empty((K, lay.ld), dtype=torch.float32, device="cuda")
    for k in range(K):
        g.manual_seed(7 + k)
        rows[k].normal_(generator=g)
    T, L = engine.tiled_tile("f32", K, lay.M), 4
    assert T == 8192
    buf = torch.zeros(engine.tiled_elems("f32", K, lay.M, T), dtype=torch.float32, device="cuda")
    tiles = buf.numel() // (K * T * L)
    for k in range(K):
        row = torch.zeros(tiles * T * L, dtype=torch.float32, device="cuda")
        row[: lay.M] = rows[k, : lay.M]
        engine.tiled_client_view(buf, "f32", K, k, T).copy_(row.view(tiles, T * L))
    ns = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    w = engine.fedavg_weights(ns, "f32")
    a = torch.empty(lay.ld, dtype=torch.float32, device="cuda")
    b = torch.empty(lay.ld, dtype=torch.float32, device="cuda")
    engine.FedAvgPlan("f32", rows, w, lay.M, a, lay.pairwise_idx).launch()
    engine.TiledFedAvgPlan("f32", buf, K, w, lay.M, b, lay.pairwise_idx, tv=T).launch()
    torch.cuda.synchronize()
    assert torch.equal(a[: lay.M].view(torch.int32), b[: lay.M].view(torch.int32))


# ---------------------------------------------------------------------------------------------
# the drop-in host path staging tile-interleaved buckets (fedagg_session_stage_tiled)
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 5, 40, 130])
@pytest.mark.parametrize("wire", [False, True])
def test_engine_stages_tiled_bit_exact(K, wire):
    from substrafl_amd.engine import AggregationEngine
    from substrafl_amd.wire import pack

    rng = np.random.default_rng(K + 1000 * wire)
    M = 2 * 32768 + 12345
    shapes, pus, ns = _case(rng, K, M, 3, False)
    eng = AggregationEngine(device=0)
    eng.tiled = True  # the layout is recommended from 32 clients over >= 2048 tiles; forced here
    got = eng.fedavg([pack(p) for p in pus] if wire else pus, ns)
    assert eng.last_timing["layout"] == "tiles"
    ref = fedavg_reference_structure(pus, ns)
    for g, r in zip(got, ref):
        assert g.shape == r.shape and np.array_equal(_bits(g), _bits(r))


@pytest.mark.gpu
def test_engine_layout_choice():
    """auto: rows below the recommended shape; fp64 / fp16 and mixed layers always rows."""
    from substrafl_amd.engine import AggregationEngine

    rng = np.random.default_rng(3)
    shapes, pus, ns = _case(rng, 4, 5000, 1, False)
    eng = AggregationEngine(device=0)
    assert eng.tiled == "auto"
    got = eng.fedavg(pus, ns)
    assert eng.last_timing["layout"] == "rows"
    for g, r in zip(got, fedavg_reference_structure(pus, ns)):
        assert np.array_equal(_bits(g), _bits(r))
    eng.tiled = True
    p64 = [[a.astype(np.float64) for a in p] for p in pus]
    got = eng.fedavg(p64, ns)
    assert eng.last_timing["layout"] == "rows"
    for g, r in zip(got, fedavg_reference_structure(p64, ns)):
        assert np.array_equal(_bits(g), _bits(r))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(24))
def test_tiled_random_sweep(seed):
    """Random client counts (1-300), bucket lengths (1-3 tiles, any remainder), numel == 1 counts
    (0-24) and tiles, against the oracle."""
    import torch

    from substrafl_amd import engine
    from substrafl_amd.layout import BucketLayout

    rng = np.random.default_rng(4242 + seed)
    kind, tv = TILES[seed % len(TILES)]
    K = int(rng.integers(1, 301))
    L = L_OF[kind]
    M = int(rng.integers(64, 3 * tv * L))
    P = int(rng.integers(0, min(25, M // 3 - 2)))
    shapes, pus, ns = _case(rng, K, M, P, kind == "bf16")
    lay = BucketLayout(range(len(shapes)), shapes, np.float32)
    buf = _tiled_device(torch, kind, pus, M, tv)
    out = torch.empty(lay.ld, dtype=torch.float32, device="cuda")
    engine.TiledFedAvgPlan(kind, buf, K, engine.fedavg_weights(ns, kind), M, out, lay.pairwise_idx, tv=tv).launch()
    torch.cuda.synchronize()
    ref = np.concatenate([r.ravel() for r in fedavg_reference_structure(pus, ns)])
    assert np.array_equal(_bits(out[:M].cpu().numpy()), _bits(ref))
