"""Property tests of the client-sharded protocol (substrafl_amd.sharding) on CPU: G ranks as
threads over LoopbackGroup with the NumPy per-rank ops (tests/shard_cpu_ops.py, test
infrastructure) -- random client counts, rank counts, layer shapes (numel == 1 included) and
relay chunk sizes.  The relay combine must reproduce the reference oracle bit for bit; the
re-associating combines must agree to rounding and keep the numel == 1 tensors exact."""

import threading

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from oracle import fedavg_reference_structure, scaffold_reference_structure
from shard_cpu_ops import CpuShardOps
from substrafl_amd.engine import fedavg_weights, scaffold_weights
from substrafl_amd.layout import BucketLayout
from substrafl_amd import lockstep
from substrafl_amd.sharding import (FedAvgShard, LoopbackGroup, ScaffoldShard, block_of, client_blocks,
                                    client_shard_fedavg, client_shard_scaffold, lockstep_fedavg, lockstep_scaffold,
                                    relay_plan, striped_plan)


def _rows(lists, layout, dtype):
    rows = np.zeros((max(1, len(lists)), layout.ld), dtype)
    for k, lay in enumerate(lists):
        layout.pack_row(lay, rows[k])
    return torch.from_numpy(rows)[: len(lists)]


def _run(G, fn, wrap=None):
    grp = LoopbackGroup(G)
    res, err = [None] * G, [None] * G

    def body(r):
        try:
            tr = grp.transport(r)
            res[r] = fn(r, wrap(tr) if wrap else tr)
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


class _OneWork:
    """A whole batch's completion as ONE work (what torch's coalescing manager returns for NCCL)."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()


class _Coalescing:
    """A transport whose exchange returns a single Work per batch, like batch_isend_irecv on
    NCCL/RCCL in torch 2.10 (the relay must not slice works by op position)."""

    def __init__(self, tr):
        self.tr, self.rank, self.world = tr, tr.rank, tr.world

    def exchange(self, ops):
        works = self.tr.exchange(ops)
        return [_OneWork(works)] if works else []

    def __getattr__(self, name):
        return getattr(self.tr, name)


def _striped_rank(r, tr, G, K, layout, pus, cvs, c, ns, rings, rounds, scaffold, lr=0.6):
    """One rank of a striped run with the NumPy ops: this rank's block buffers packed as the plan says."""
    plan = striped_plan(layout.M, G, r, rings, rounds)
    full_c = _rows([c], layout, np.float32)[0]
    blocks = {}
    for b, segs in plan.blocks.items():
        k0, k1 = client_blocks(K, G)[b]

        def packed(lists):
            full = _rows(lists, layout, np.float32)
            t = torch.zeros((max(1, k1 - k0), plan.block_len[b]), dtype=torch.float32)
            for lo, hi, col in segs:
                t[: k1 - k0, col: col + hi - lo] = full[:, lo:hi]
            return t[: k1 - k0]

        if scaffold:
            blocks[b] = ScaffoldShard("f32", packed(pus[k0:k1]), packed(cvs[k0:k1]), None, scaffold_weights(ns)[k0:k1],
                                      k0, K, plan.block_len[b], lr, np.zeros(0, np.uint64))
        else:
            blocks[b] = FedAvgShard("f32", packed(pus[k0:k1]), fedavg_weights(ns, "f32")[k0:k1], k0, K,
                                    plan.block_len[b], np.zeros(0, np.uint64))
    if not scaffold:
        out = torch.zeros(layout.ld, dtype=torch.float32)
        if lockstep_fedavg(plan, blocks, out, tr, CpuShardOps(), layout.pairwise_idx):
            return out[: layout.M].numpy().copy()
        return None
    dout = torch.zeros(layout.ld, dtype=torch.float64)
    cout = torch.zeros(layout.ld, dtype=torch.float64)
    if lockstep_scaffold(plan, blocks, dout, cout, tr, CpuShardOps(), layout.pairwise_idx, full_c, lr):
        return dout[: layout.M].numpy().copy(), cout[: layout.M].numpy().copy()
    return None


def _check(res, shapes, pus, cvs, c, ns, scaffold, lr=0.6):
    layout = BucketLayout(range(len(shapes)), shapes, np.float32)
    if not scaffold:
        for g, r in zip([a for _, a in layout.unpack(res)], fedavg_reference_structure(pus, ns)):
            assert np.array_equal(g.view(np.uint32), r.view(np.uint32))
        return
    lay64 = BucketLayout(range(len(shapes)), shapes, np.float64)
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, lr)
    got = [a for _, a in lay64.unpack(res[1])] + [a for _, a in lay64.unpack(res[0])]
    for g, r in zip(got, rc + ra):
        assert np.array_equal(g.view(np.uint64), r.view(np.uint64))


@settings(max_examples=30, deadline=None)
@given(st.integers(1, 12), st.integers(1, 8), st.integers(1, 4), shape_st,
       st.sampled_from([(1.0,), (0.75, 0.25), (0.5, 0.3, 0.2)]), st.booleans(), st.integers(0, 2**31))
def test_striped_relay_property(K, G, rings, shapes, rounds, scaffold, seed):
    """The striped relay (pieces rotating over the ranks on up to four rings, every rank holding
    one client block per stripe) reproduces the reference bit for bit for FedAvg and Scaffold,
    empty pieces and empty blocks included."""
    shapes = shapes + [(700,)]
    rng = np.random.default_rng(seed)
    pus = [[(rng.standard_normal(s) * 10.0 ** rng.integers(-2, 3)).astype(np.float32) for s in shapes] for _ in range(K)]
    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    layout = BucketLayout(range(len(shapes)), shapes, np.float32)
    res = _run(G, lambda r, tr: _striped_rank(r, tr, G, K, layout, pus, cvs, c, ns, rings, rounds, scaffold))
    _check(res, shapes, pus, cvs, c, ns, scaffold)


@pytest.mark.parametrize("G,K,combine", [(3, 7, "relay"), (5, 11, "relay"), (4, 9, "striped"), (8, 17, "striped")])
@pytest.mark.parametrize("scaffold", [False, True])
def test_single_work_per_batch(G, K, combine, scaffold):
    """A transport that returns ONE work for a whole batched exchange (torch's coalescing manager on
    RCCL), with middle ranks that both receive and send: every work of a group is waited before
    the step that reads its receives, so the result stays bit-exact."""
    shapes = [(37, 29), (1,), (3000,), (1, 1), (700,)]
    rng = np.random.default_rng(G * 31 + K)
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    cvs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    c = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    layout = BucketLayout(range(len(shapes)), shapes, np.float32)

    def rank(r, tr):
        if combine == "striped":
            return _striped_rank(r, tr, G, K, layout, pus, cvs, c, ns, None, (0.75, 0.25), scaffold)
        k0, k1 = client_blocks(K, G)[block_of(r, G)]
        if not scaffold:
            sh = FedAvgShard("f32", _rows(pus[k0:k1], layout, np.float32), fedavg_weights(ns, "f32")[k0:k1], k0, K,
                             layout.M, layout.pairwise_idx)
            out = torch.zeros(layout.ld, dtype=torch.float32)
            return out[: layout.M].numpy().copy() if client_shard_fedavg(sh, out, tr, CpuShardOps(), "relay",
                                                                         chunk_elems=512) else None
        sh = ScaffoldShard("f32", _rows(pus[k0:k1], layout, np.float32), _rows(cvs[k0:k1], layout, np.float32),
                           _rows([c], layout, np.float32)[0], scaffold_weights(ns)[k0:k1], k0, K, layout.M, 0.6,
                           layout.pairwise_idx)
        dout = torch.zeros(layout.ld, dtype=torch.float64)
        cout = torch.zeros(layout.ld, dtype=torch.float64)
        if client_shard_scaffold(sh, dout, cout, tr, CpuShardOps(), "relay", chunk_elems=512):
            return dout[: layout.M].numpy().copy(), cout[: layout.M].numpy().copy()
        return None

    _check(_run(G, rank, wrap=_Coalescing), shapes, pus, cvs, c, ns, scaffold)


def test_ring_chains_cover_disjoint_links():
    """G = 8, ``rings=4``: the unit rings, hops 1, 7, 3 and 5 ranks long -- every piece of ring a
    visits every rank once, ending on its stripe's rank, and the four rings use 4 x 8 distinct
    directed links, so each rank sends on four links at every step."""
    G = 8
    mult = lockstep.ring_multipliers(G)
    assert mult == [1, 7, 3, 5]
    assert lockstep.ring_chains(G, 4) == [tuple((a * (b + 1)) % G for b in range(G)) for a in mult]
    pieces = lockstep.striped_pieces(8 * 2 * 4 * 512 * 3, G, rings=4)
    links = {}
    for p in pieces:
        assert sorted(p.ranks) == list(range(G))
        hop = (p.ranks[1] - p.ranks[0]) % G
        assert hop in mult and all((p.ranks[b + 1] - p.ranks[b]) % G == hop for b in range(G - 1))
        links.setdefault(hop, set()).update((p.ranks[b], p.ranks[b + 1]) for b in range(G - 1))
    assert all(len(v) == G for v in links.values())
    assert len(set().union(*links.values())) == 4 * G


@pytest.mark.parametrize("G", [2, 3, 4, 5, 6, 7, 8])
def test_default_chains_use_distinct_links_every_step(G):
    """The default chains (Latin at G = 6 and 8: 5 and 6 chains; the unit rings elsewhere): every
    chain visits every rank once, and at every step the chains' hops are distinct and non-zero --
    with the stripe shifts, each rank sends to (and receives from) R distinct peers per step."""
    chains = lockstep.ring_chains(G)
    assert len(chains) == {6: 5, 8: 6}.get(G, min(len(lockstep.ring_units(G)), 4))
    for c in chains:
        assert sorted(c) == list(range(G))
    pieces = lockstep.striped_pieces(G * 2 * len(chains) * 512 * 2, G)
    for t in range(1 + max(p.t0 + 2 * (G - 1) for p in pieces)):
        sends = {}
        for p in pieces:
            for b in range(G - 1):
                if p.t0 + 2 * b == t:
                    sends.setdefault(p.ranks[b], []).append(p.ranks[b + 1])
        for src, dsts in sends.items():
            assert len(set(dsts)) == len(dsts) and src not in dsts, (t, src, dsts)


@settings(max_examples=40, deadline=None)
@given(st.integers(1, 3_000_000), st.integers(1, 8), st.integers(1, 4),
       st.sampled_from([(1.0,), (0.75, 0.25), (0.6, 0.3, 0.1)]), st.sampled_from([512, 4096, 1 << 20]))
def test_lockstep_groups_pair_exactly(M, G, rings, rounds, chunk):
    """Every message of exchange group t has its partner in group t of the peer (same size, same
    order for a rank pair): the property that makes the single-thread, single-communicator
    schedule deadlock-free.  Every element is computed once per block and sent once per hop."""
    for plans in ([relay_plan(M, G, r, chunk) for r in range(G)],
                  [striped_plan(M, G, r, rings, rounds) for r in range(G)]):
        T = plans[0].n_steps
        assert all(p.n_steps == T for p in plans)
        for t in range(T + 1):
            for q in range(G):
                for r in range(G):
                    sends = [(o.n, o.key) for o in plans[q].groups[t] if o.kind == "send" and o.peer == r]
                    recvs = [(o.n, o.key) for o in plans[r].groups[t] if o.kind == "recv" and o.peer == q]
                    assert sends == recvs
        for p in plans:  # each rank computes every element once per block it holds for it
            held = sum(hi - lo for segs in p.blocks.values() for lo, hi, _c in segs)
            ran = sum(run.n for runs in p.runs for run in runs)
            assert held == ran
        assert sum(sum(hi - lo for lo, hi, _c in p.blocks.get(0, [])) for p in plans) == M


@pytest.mark.parametrize("G", [2, 3, 4, 5, 6, 8])
def test_striped_every_rank_busy_every_step(G):
    """The striped schedule has no pipeline fill: at every step every rank runs ONE launch (its
    block p of one piece per ring), and every rank holds M elements' worth of client blocks."""
    M = 2 * G * len(lockstep.ring_chains(G)) * 512 * 5
    plans = [striped_plan(M, G, r) for r in range(G)]
    for p in plans:
        assert [len(x) for x in p.runs] == [1] * p.n_steps
        assert sum(hi - lo for segs in p.blocks.values() for lo, hi, _c in segs) == M
    assert plans[0].n_steps == 2 * G


@pytest.mark.parametrize("queues", ["streams", "single"])
@pytest.mark.parametrize("G", [2, 3, 8])
def test_lockstep_deadlock_free_model(queues, G):
    """tools/lockstep_model.py plays every rank's kernels in issue order -- with the communicator
    and compute kernels on separate queues, and with ALL of a rank's kernels on one in-order
    hardware queue -- and every group completes, for the relay and the striped schedules."""
    from tools.lockstep_model import simulate

    for plans in ([relay_plan(1 << 20, G, r, 1 << 16) for r in range(G)],
                  [striped_plan(1 << 20, G, r, None, (0.75, 0.25)) for r in range(G)]):
        res = simulate(plans, queues, compute_s_per_elem=1e-9, link_s_per_elem=3e-9, latency_s=1e-5)
        assert res["makespan"] >= res["compute_max"] > 0


def test_deadlock_model_detects_a_crossed_order():
    """Negative control of the model: two ranks that each receive from the other before sending
    (NCCL's documented deadlock pattern) never complete."""
    from tools.lockstep_model import Deadlock, simulate

    def plan(rank):
        peer = 1 - rank
        groups = [[lockstep.Op("recv", peer, ("slot", 0, 0), 8, 0)], [lockstep.Op("send", peer, ("slot", 0, 0), 8, 0)]]
        return lockstep.RankPlan(rank, 2, 0, [[]], groups, {}, {}, 8)

    with pytest.raises(Deadlock):
        simulate([plan(0), plan(1)], "single")
