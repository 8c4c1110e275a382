"""world_size-2 gloo tests of the multi-GPU plumbing (CPU).  The per-shard reducer is the oracle
here (test infrastructure); on the GPU box the same code runs libfedagg per rank."""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import fedavg_reference_structure, numpy_pairwise_sum
from substrafl_amd.layout import BucketLayout
from substrafl_amd.sharding import client_sharded_fedavg, pack_range, param_range_fedavg, shard_bounds


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


def _worker(rank, world, port, mode, q, on_gpu=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pus, ns = _data()
        # on_gpu: every rank reduces its slice with libfedagg on cuda:0 (the ranks share the one
        # GPU of the test box; the control plane stays gloo, as in bench.py)
        red = None if on_gpu else oracle_flat_reducer
        if mode == "param":
            res = param_range_fedavg(pus, ns, reducer=red)
        else:
            res = client_sharded_fedavg(pus, ns, reducer=red, combine=mode)
        q.put((rank, None if res is None else [np.asarray(a) for a in res]))
    finally:
        dist.destroy_process_group()


def _run(mode, world=2, on_gpu=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q, on_gpu)) for r in range(world)]
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


@pytest.mark.parametrize("mode", ["ordered", "rccl"])
def test_client_sharded_world2_close(mode):
    """North-star mode re-associates the client sum: close, not bit-exact."""
    pus, ns = _data()
    ref = fedavg_reference_structure(pus, ns)
    out = _run(mode)
    assert out[1] is None
    for g, r in zip(out[0], ref):
        np.testing.assert_allclose(g, r, rtol=1e-5, atol=1e-6)


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
