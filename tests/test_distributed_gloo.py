"""world_size-2 gloo tests of the multi-GPU plumbing (CPU).  The per-shard reducer is the oracle
here (test infrastructure); on the GPU box the same code runs libfedagg per rank."""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import torch

from oracle import fedavg_reference_structure, numpy_pairwise_sum, scaffold_reference_structure
from substrafl_amd.engine import fedavg_weights, scaffold_weights
from substrafl_amd.layout import BucketLayout
from substrafl_amd.sharding import (DistTransport, FedAvgShard, ScaffoldShard, block_of, chain_rank, client_blocks,
                                    client_shard_fedavg, client_shard_scaffold, pack_range, param_range_fedavg,
                                    relay_chunks, shard_bounds)
from shard_cpu_ops import CpuShardOps


def oracle_flat_reducer(rows, n_samples, pairwise_idx):
    """Flat restatement: sequential fp32 chain per element, NumPy pairwise at pairwise_idx."""
    n_all = sum(int(n) for n in n_samples)
    w = np.array([int(n) / n_all for n in n_samples], np.float64).astype(rows.dtype)
    acc = np.zeros(rows.shape[1], rows.dtype)
    for k in range(rows.shape[0]):
        acc = (acc + (rows[k] * w[k]).astype(rows.dtype)).astype(rows.dtype)
    for p in np.asarray(pairwise_idx, np.int64):
        prods = (rows[:, p] * w).astype(rows.dtype)
        acc[p] = rows.dtype.type(0.0) + numpy_pairwise_sum(prods)
    return acc


def _data(K=5, seed=0):
    rng = np.random.default_rng(seed)
    shapes = [(37, 29), (1,), (700,), (1, 1), (3, 3, 3)]
    pus = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    return pus, ns


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flat_rows(lists, layout, dtype):
    rows = np.zeros((len(lists), layout.ld), dtype)
    for k, lay in enumerate(lists):
        layout.pack_row(lay, rows[k])
    return rows


def _client_shard_cpu(rank, world, mode, K, strategy, chunk_elems):
    """This rank's block of the client-sharded FedAvg / Scaffold over gloo with the NumPy ops."""
    pus, ns = _data(K=K)
    layout = BucketLayout(range(len(pus[0])), [a.shape for a in pus[0]], np.float32)
    if mode == "striped":
        return _client_shard_striped_cpu(rank, world, K, strategy, chunk_elems, pus, ns, layout)
    k0, k1 = client_blocks(K, world)[block_of(rank, world)]
    tr = DistTransport()
    if strategy == "fedavg":
        rows = torch.from_numpy(_flat_rows(pus[k0:k1], layout, np.float32))
        sh = FedAvgShard("f32", rows, fedavg_weights(ns, "f32")[k0:k1], k0, K, layout.M, layout.pairwise_idx)
        out = torch.zeros(layout.ld, dtype=torch.float32)
        root = client_shard_fedavg(sh, out, tr, CpuShardOps(), combine=mode, chunk_elems=chunk_elems)
        return [a for _, a in layout.unpack(out[: layout.M].numpy().copy())] if root else None
    rng = np.random.default_rng(5)
    cvs = [[rng.standard_normal(a.shape).astype(np.float32) for a in pu] for pu in pus]
    c = [rng.standard_normal(a.shape).astype(np.float32) for a in pus[0]]
    delta = torch.from_numpy(_flat_rows(pus[k0:k1], layout, np.float32))
    cv = torch.from_numpy(_flat_rows(cvs[k0:k1], layout, np.float32))
    ct = torch.from_numpy(_flat_rows([c], layout, np.float32)[0])
    sh = ScaffoldShard("f32", delta, cv, ct, scaffold_weights(ns)[k0:k1], k0, K, layout.M, 0.7, layout.pairwise_idx)
    dout = torch.zeros(layout.ld, dtype=torch.float64)
    cout = torch.zeros(layout.ld, dtype=torch.float64)
    root = client_shard_scaffold(sh, dout, cout, tr, CpuShardOps(), combine=mode, chunk_elems=chunk_elems)
    if not root:
        return None
    lay64 = BucketLayout(range(len(pus[0])), [a.shape for a in pus[0]], np.float64)
    return ([a for _, a in lay64.unpack(cout[: layout.M].numpy().copy())]
            + [a for _, a in lay64.unpack(dout[: layout.M].numpy().copy())])


def _client_shard_striped_cpu(rank, world, K, strategy, chunk_elems, pus, ns, layout):
    """The striped relay over gloo: ONE process group (the default), every rank issuing its
    lockstep exchange groups from one thread, NumPy per-rank ops."""
    from substrafl_amd.sharding import ScaffoldShard as SS
    from substrafl_amd.sharding import lockstep_fedavg, lockstep_scaffold, striped_plan

    tr = DistTransport()
    plan = striped_plan(layout.M, world, rank, None, (0.75, 0.25))
    rng = np.random.default_rng(5)
    cvs = [[rng.standard_normal(a.shape).astype(np.float32) for a in pu] for pu in pus]
    c = [rng.standard_normal(a.shape).astype(np.float32) for a in pus[0]]
    ct = torch.from_numpy(_flat_rows([c], layout, np.float32)[0])
    blocks = {}
    for b, segs in plan.blocks.items():
        k0, k1 = client_blocks(K, world)[b]

        def packed(lists):
            full = _flat_rows(lists, layout, np.float32)
            t = np.zeros((k1 - k0, plan.block_len[b]), np.float32)
            for lo, hi, col in segs:
                t[:, col: col + hi - lo] = full[:, lo:hi]
            return torch.from_numpy(t)

        if strategy == "fedavg":
            blocks[b] = FedAvgShard("f32", packed(pus[k0:k1]), fedavg_weights(ns, "f32")[k0:k1], k0, K,
                                    plan.block_len[b], np.zeros(0, np.uint64))
        else:
            blocks[b] = SS("f32", packed(pus[k0:k1]), packed(cvs[k0:k1]), None, scaffold_weights(ns)[k0:k1], k0, K,
                           plan.block_len[b], 0.7, np.zeros(0, np.uint64))
    if strategy == "fedavg":
        out = torch.zeros(layout.ld, dtype=torch.float32)
        root = lockstep_fedavg(plan, blocks, out, tr, CpuShardOps(), layout.pairwise_idx)
        return [a for _, a in layout.unpack(out[: layout.M].numpy().copy())] if root else None
    dout = torch.zeros(layout.ld, dtype=torch.float64)
    cout = torch.zeros(layout.ld, dtype=torch.float64)
    if not lockstep_scaffold(plan, blocks, dout, cout, tr, CpuShardOps(), layout.pairwise_idx, ct, 0.7):
        return None
    lay64 = BucketLayout(range(len(pus[0])), [a.shape for a in pus[0]], np.float64)
    return ([a for _, a in lay64.unpack(cout[: layout.M].numpy().copy())]
            + [a for _, a in lay64.unpack(dout[: layout.M].numpy().copy())])


def _worker(rank, world, port, mode, q, on_gpu=False, K=5, strategy="fedavg", chunk_elems=512):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if mode == "param":
            pus, ns = _data()
            # on_gpu: every rank stages and reduces its slice with libfedagg on cuda:0 (the ranks
            # share the one GPU of the test box; the control plane stays gloo, as in bench.py)
            res = param_range_fedavg(pus, ns, reducer=None if on_gpu else oracle_flat_reducer)
        else:
            res = _client_shard_cpu(rank, world, mode, K, strategy, chunk_elems)
        q.put((rank, None if res is None else [np.asarray(a) for a in res]))
    finally:
        dist.destroy_process_group()


def _run(mode, world=2, on_gpu=False, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q, on_gpu), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_shard_bounds_cover_and_align():
    for M in (1, 511, 512, 513, 25_000_000, 125_000_001):
        for world in (1, 2, 3, 8):
            b = shard_bounds(M, world)
            assert b[0][0] == 0 and b[-1][1] == M
            for (lo, hi), (lo2, _) in zip(b, b[1:]):
                assert hi == lo2 and (lo % 512 == 0 or lo == M)


def test_pack_range_matches_full_row():
    pus, _ = _data()
    lay = BucketLayout(range(5), [a.shape for a in pus[0]], np.float32)
    full = np.zeros(lay.M, np.float32)
    lay.pack_row(pus[0], full)
    for lo, hi in [(0, 5), (3, 1100), (1070, lay.M), (1073, 1074)]:
        part = np.zeros(hi - lo, np.float32)
        pack_range(lay, pus[0], part, lo, hi)
        assert np.array_equal(part, full[lo:hi])


def test_param_range_world2_bit_exact():
    pus, ns = _data()
    ref = fedavg_reference_structure(pus, ns)
    out = _run("param")
    for rank in (0, 1):
        for g, r in zip(out[rank], ref):
            assert g.shape == r.shape and np.array_equal(g.view(np.uint32), r.view(np.uint32))


def test_client_blocks_and_chain():
    for K in (1, 2, 3, 5, 64, 65):
        for G in (1, 2, 3, 8):
            blocks = client_blocks(K, G)
            assert blocks[0][0] == 0 and blocks[-1][1] == K and len(blocks) == G
            assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
            sizes = [b - a for a, b in blocks]
            if K >= G:  # balanced, never empty (the native executor runs every K >= G)
                assert min(sizes) >= 1 and max(sizes) - min(sizes) <= 1
            else:
                assert sizes == [1] * K + [0] * (G - K)
            assert sorted(chain_rank(b, G) for b in range(G)) == list(range(G))
            assert chain_rank(G - 1, G) == 0  # the last block (final step) is on the root
            assert all(block_of(chain_rank(b, G), G) == b for b in range(G))
    for M in (0, 1, 511, 513, 10_000):
        ch = relay_chunks(M, 1000)
        assert ch[0][0] == 0 and ch[-1][1] == M and all(a[1] == b[0] for a, b in zip(ch, ch[1:]))


@pytest.mark.parametrize("world,K", [(2, 5), (3, 5), (3, 2), (4, 9)])
def test_client_sharded_relay_bit_exact(world, K):
    """North-star client sharding with the relay combine: the chain of blocks reproduces the
    reference's sequential client sum exactly (numel == 1 layers via the gathered pairwise
    products), also with empty blocks (K < world) and several pipelining chunks."""
    pus, ns = _data(K=K)
    ref = fedavg_reference_structure(pus, ns)
    out = _run("relay", world=world, K=K)
    assert all(out[r] is None for r in range(1, world))
    for g, r in zip(out[0], ref):
        assert g.shape == r.shape and np.array_equal(g.view(np.uint32), r.view(np.uint32))


@pytest.mark.parametrize("world,K,strategy", [(2, 5, "fedavg"), (4, 9, "fedavg"), (3, 2, "fedavg"),
                                              (4, 6, "scaffold"), (2, 3, "scaffold")])
def test_client_sharded_striped_bit_exact(world, K, strategy):
    """The striped relay over a real gloo process group (one communicator, one issuing thread per
    rank, the lockstep exchange groups): bit-identical to the reference, empty blocks included."""
    pus, ns = _data(K=K)
    out = _run("striped", world=world, K=K, strategy=strategy)
    assert all(out[r] is None for r in range(1, world))
    if strategy == "fedavg":
        ref = fedavg_reference_structure(pus, ns)
        bits = np.uint32
    else:
        rng = np.random.default_rng(5)
        cvs = [[rng.standard_normal(a.shape).astype(np.float32) for a in pu] for pu in pus]
        c = [rng.standard_normal(a.shape).astype(np.float32) for a in pus[0]]
        rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.7)
        ref, bits = rc + ra, np.uint64
    for g, r in zip(out[0], ref):
        assert g.shape == r.shape and np.array_equal(g.view(bits), r.view(bits))


@pytest.mark.parametrize("mode", ["ordered", "rccl"])
def test_client_sharded_world2_close(mode):
    """The re-associating combines: close, not bit-exact (numel == 1 layers stay exact)."""
    pus, ns = _data()
    ref = fedavg_reference_structure(pus, ns)
    out = _run(mode)
    assert out[1] is None
    for g, r in zip(out[0], ref):
        np.testing.assert_allclose(g, r, rtol=1e-5, atol=1e-6)
        if g.size == 1:
            assert np.array_equal(g.view(np.uint32), r.view(np.uint32))


@pytest.mark.parametrize("mode,world,K", [("relay", 2, 5), ("relay", 3, 2), ("ordered", 2, 5), ("rccl", 3, 7)])
def test_client_sharded_scaffold(mode, world, K):
    """Scaffold over client blocks: c added last and aggregation_lr applied on the root
    (scaffold.py:262-263, 293); relay bit-exact in fp64."""
    pus, ns = _data(K=K)
    rng = np.random.default_rng(5)
    cvs = [[rng.standard_normal(a.shape).astype(np.float32) for a in pu] for pu in pus]
    c = [rng.standard_normal(a.shape).astype(np.float32) for a in pus[0]]
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.7)
    out = _run(mode, world=world, K=K, strategy="scaffold")
    assert all(out[r] is None for r in range(1, world))
    for g, r in zip(out[0], rc + ra):
        assert g.dtype == np.float64 and g.shape == r.shape
        if mode == "relay":
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64))
        else:
            np.testing.assert_allclose(g, r, rtol=1e-12, atol=1e-14)


@pytest.mark.gpu
def test_param_range_world2_gpu_reducer_bit_exact():
    """The product reducer (libfedagg per rank) under parameter-range sharding: bit-identical to
    the reference on every rank."""
    out = _run("param", on_gpu=True)
    pus, ns = _data()
    ref = fedavg_reference_structure(pus, ns)
    for rank in (0, 1):
        for g, r in zip(out[rank], ref):
            assert g.shape == r.shape and np.array_equal(g.view(np.uint32), r.view(np.uint32))
