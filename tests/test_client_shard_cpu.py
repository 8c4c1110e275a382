"""Property tests of the client-sharded protocol (substrafl_amd.sharding) on CPU: G ranks as
threads over LoopbackGroup with the NumPy per-rank ops (tests/shard_cpu_ops.py, test
infrastructure) -- random client counts, rank counts, layer shapes (numel == 1 included) and
relay chunk sizes.  The relay combine must reproduce the reference oracle bit for bit; the
re-associating combines must agree to rounding and keep the numel == 1 tensors exact."""

import threading

import numpy as np
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from oracle import fedavg_reference_structure, scaffold_reference_structure
from shard_cpu_ops import CpuShardOps
from substrafl_amd.engine import fedavg_weights, scaffold_weights
from substrafl_amd.layout import BucketLayout
from substrafl_amd.sharding import (FedAvgShard, LoopbackGroup, ScaffoldShard, block_of, client_blocks,
                                    client_shard_fedavg, client_shard_scaffold)


def _rows(lists, layout, dtype):
    rows = np.zeros((max(1, len(lists)), layout.ld), dtype)
    for k, lay in enumerate(lists):
        layout.pack_row(lay, rows[k])
    return torch.from_numpy(rows)[: len(lists)]


def _run(G, fn):
    grp = LoopbackGroup(G)
    res, err = [None] * G, [None] * G

    def body(r):
        try:
            res[r] = fn(r, grp.transport(r))
        except BaseException as e:  # noqa: BLE001
            err[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
        assert not t.is_alive()
    for e in err:
        if e is not None:
            raise e
    assert all(x is None for x in res[1:])
    return res[0]


shape_st = st.lists(st.sampled_from([(1,), (1, 1), (7,), (33,), (5, 3), (200,), (2, 1, 3)]), min_size=1, max_size=5)


@settings(max_examples=40, deadline=None)
@given(st.integers(1, 12), st.integers(1, 6), shape_st, st.sampled_from([512, 1024, 4096]),
       st.sampled_from(["relay", "ordered", "rccl"]), st.integers(0, 2**31))
def test_fedavg_client_shard_property(K, G, shapes, chunk, combine, seed):
    rng = np.random.default_rng(seed)
    pus = [[(rng.standard_normal(s) * 10.0 ** rng.integers(-2, 3)).astype(np.float32) for s in shapes] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    layout = BucketLayout(range(len(shapes)), shapes, np.float32)
    w = fedavg_weights(ns, "f32")

    def rank(r, tr):
        k0, k1 = client_blocks(K, G)[block_of(r, G)]
        sh = FedAvgShard("f32", _rows(pus[k0:k1], layout, np.float32), w[k0:k1], k0, K, layout.M, layout.pairwise_idx)
        out = torch.zeros(layout.ld, dtype=torch.float32)
        if client_shard_fedavg(sh, out, tr, CpuShardOps(), combine, chunk_elems=chunk):
            return out[: layout.M].numpy().copy()
        return None

    got = [a for _, a in layout.unpack(_run(G, rank))]
    ref = fedavg_reference_structure(pus, ns)
    for g, r in zip(got, ref):
        if combine == "relay" or g.size == 1 or G == 1:
            assert np.array_equal(g.view(np.uint32), r.view(np.uint32))
        else:
            np.testing.assert_allclose(g, r, rtol=1e-5, atol=1e-4)


@settings(max_examples=25, deadline=None)
@given(st.integers(1, 9), st.integers(1, 5), shape_st, st.sampled_from(["relay", "ordered", "rccl"]),
       st.sampled_from([0.0, 0.5, 1.0, 2.0]), st.integers(0, 2**31))
def test_scaffold_client_shard_property(K, G, shapes, combine, lr, seed):
    rng = np.random.default_rng(seed)
    mk = lambda: [rng.standard_normal(s).astype(np.float32) for s in shapes]  # noqa: E731
    pus, cvs, c = [mk() for _ in range(K)], [mk() for _ in range(K)], mk()
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    layout = BucketLayout(range(len(shapes)), shapes, np.float32)
    w = scaffold_weights(ns)

    def rank(r, tr):
        k0, k1 = client_blocks(K, G)[block_of(r, G)]
        sh = ScaffoldShard("f32", _rows(pus[k0:k1], layout, np.float32), _rows(cvs[k0:k1], layout, np.float32),
                           _rows([c], layout, np.float32)[0], w[k0:k1], k0, K, layout.M, lr, layout.pairwise_idx)
        dout = torch.zeros(layout.ld, dtype=torch.float64)
        cout = torch.zeros(layout.ld, dtype=torch.float64)
        if client_shard_scaffold(sh, dout, cout, tr, CpuShardOps(), combine, chunk_elems=512):
            return dout[: layout.M].numpy().copy(), cout[: layout.M].numpy().copy()
        return None

    d, cc = _run(G, rank)
    lay64 = BucketLayout(range(len(shapes)), shapes, np.float64)
    got = [a for _, a in lay64.unpack(cc)] + [a for _, a in lay64.unpack(d)]
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, lr)
    for g, r in zip(got, rc + ra):
        if combine == "relay" or g.size == 1 or G == 1:
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64))
        else:
            np.testing.assert_allclose(g, r, rtol=1e-12, atol=1e-12)


def test_loopback_collectives():
    """The in-process transport's collectives: reduce / gather onto rank 0 in rank order,
    all_sum_int everywhere (repeatedly, so its bookkeeping is released), P2P in FIFO order."""
    G = 4
    grp = LoopbackGroup(G)
    out = [None] * G

    def body(r):
        tr = grp.transport(r)
        sums = [tr.all_sum_int(r + i) for i in range(3)]
        t = torch.full((5,), float(r + 1))
        tr.reduce_sum(t, 0)
        g = tr.gather(torch.tensor([r]), 0)
        recv = torch.zeros(2)
        works = tr.exchange([("send", torch.tensor([float(r), 1.0 * r]), (r + 1) % G),
                             ("recv", recv, (r - 1) % G)])
        for w in works:
            w.wait()
        out[r] = (sums, t.tolist() if r == 0 else None, None if g is None else [int(x) for x in g], recv.tolist())

    th = [threading.Thread(target=body, args=(r,)) for r in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    for r in range(G):
        assert out[r][0] == [6, 10, 14]
        assert out[r][3] == [float((r - 1) % G)] * 2
    assert out[0][1] == [10.0] * 5 and out[0][2] == [0, 1, 2, 3]
    assert not grp._coll  # every collective's entries consumed


def _run_striped(G, S, fn):
    """G ranks as threads; every rank gets one transport per stripe (one loopback group each)."""
    groups = [LoopbackGroup(G) for _ in range(S)]
    return _run(G, lambda r, _tr: fn(r, [g.transport(r) for g in groups]))


@settings(max_examples=30, deadline=None)
@given(st.integers(1, 12), st.integers(1, 8), st.integers(1, 4), shape_st, st.sampled_from([512, 1024]),
       st.booleans(), st.integers(0, 2**31))
def test_striped_relay_property(K, G, stripes, shapes, chunk, scaffold, seed):
    """The striped relay (S parameter stripes, stripe s's chain a_s ranks per hop) reproduces the
    reference bit for bit for FedAvg and Scaffold, empty stripes and empty blocks included."""
    from substrafl_amd.sharding import (client_shard_fedavg_striped, client_shard_scaffold_striped, stripe_layout,
                                        stripe_multipliers)

    shapes = shapes + [(700,)]  # at least two 512-element stripes' worth
    rng = np.random.default_rng(seed)
    pus = [[(rng.standard_normal(s) * 10.0 ** rng.integers(-2, 3)).astype(np.float32) for s in shapes] for _ in range(K)]
    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    layout = BucketLayout(range(len(shapes)), shapes, np.float32)
    pw = layout.pairwise_idx.astype(np.int64)
    S = len(stripe_multipliers(G, stripes))

    def rank(r, trs):
        lay = stripe_layout(layout.M, K, G, r, stripes)
        bounds = [(lo, hi, a) for lo, hi, a, *_ in lay]
        ct = _rows([c], layout, np.float32)[0]
        parts = []
        for lo, hi, a, b, k0, k1 in lay:
            loc = (pw[(pw >= lo) & (pw < hi)] - lo).astype(np.uint64)
            d = _rows(pus[k0:k1], layout, np.float32)[:, lo:hi].contiguous()
            if not scaffold:
                parts.append(FedAvgShard("f32", d, fedavg_weights(ns, "f32")[k0:k1], k0, K, hi - lo, loc))
            else:
                v = _rows(cvs[k0:k1], layout, np.float32)[:, lo:hi].contiguous()
                parts.append(ScaffoldShard("f32", d, v, ct[lo:hi], scaffold_weights(ns)[k0:k1], k0, K, hi - lo, 0.6,
                                           loc))
        if not scaffold:
            out = torch.zeros(layout.ld, dtype=torch.float32)
            if client_shard_fedavg_striped(parts, bounds, out, trs, CpuShardOps(), pw, chunk_elems=chunk):
                return out[: layout.M].numpy().copy()
            return None
        dout = torch.zeros(layout.ld, dtype=torch.float64)
        cout = torch.zeros(layout.ld, dtype=torch.float64)
        if client_shard_scaffold_striped(parts, bounds, dout, cout, trs, CpuShardOps(), pw, c=ct, chunk_elems=chunk):
            return dout[: layout.M].numpy().copy(), cout[: layout.M].numpy().copy()
        return None

    res = _run_striped(G, S, rank)
    if not scaffold:
        for g, r in zip([a for _, a in layout.unpack(res)], fedavg_reference_structure(pus, ns)):
            assert np.array_equal(g.view(np.uint32), r.view(np.uint32))
        return
    lay64 = BucketLayout(range(len(shapes)), shapes, np.float64)
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.6)
    got = [a for _, a in lay64.unpack(res[1])] + [a for _, a in lay64.unpack(res[0])]
    for g, r in zip(got, rc + ra):
        assert np.array_equal(g.view(np.uint64), r.view(np.uint64))


def test_stripe_chains_cover_disjoint_links():
    """G = 8: four stripes whose chain hops are 1, 7, 3 and 5 ranks long -- 4 x 7 distinct directed
    links, every chain ends on the root, and every rank holds exactly one block per stripe."""
    from substrafl_amd.sharding import stripe_block, stripe_multipliers, stripe_rank

    G = 8
    mult = stripe_multipliers(G)
    assert mult == [1, 7, 3, 5]
    links = set()
    for a in mult:
        order = [stripe_rank(b, G, a) for b in range(G)]
        assert sorted(order) == list(range(G)) and order[-1] == 0
        assert all(stripe_block(stripe_rank(b, G, a), G, a) == b for b in range(G))
        hops = {(order[b], order[b + 1]) for b in range(G - 1)}
        assert not hops & links
        links |= hops
    assert len(links) == 4 * (G - 1)
