"""GPU tests of the client-sharded (north-star) mode with the product arithmetic (libfedagg's chain
/ partial / pairwise kernels, substrafl_amd.sharding.GpuShardOps):

* G ranks as threads on the one GPU of the test box (LoopbackGroup: each rank on its own HIP
  stream, messages ordered by events) -- the relay combine bit-identical to the reference oracle
  for FedAvg fp32 / bf16 and Scaffold, also with empty client blocks; the re-associating
  combines close, their numel == 1 elements exact;
* the host entry points over a real RCCL process group of world size 1."""

import os
import socket
import threading

import numpy as np
import pytest

from oracle import fedavg_reference_structure, scaffold_reference_structure

pytestmark = pytest.mark.gpu

SHAPES = [(37, 29), (1,), (3000,), (1, 1), (3, 3, 3), (1,), (257,)]


def _data(K, seed=0, shapes=SHAPES):
    rng = np.random.default_rng(seed)
    pus = [[(rng.standard_normal(s) * 10.0 ** rng.integers(-2, 3)).astype(np.float32) for s in shapes]
           for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    return pus, ns


def _loopback(G, fn, transports=None):
    """Run ``fn(rank, transport)`` for G ranks as threads on the one GPU, each on its own stream;
    ``transports``: per-rank transports (default: one LoopbackGroup's)."""
    import torch

    from substrafl_amd.sharding import LoopbackGroup

    grp = LoopbackGroup(G)
    res, err = [None] * G, [None] * G

    def body(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                res[r] = fn(r, transports[r] if transports else grp.transport(r))
            s.synchronize()
        except BaseException as e:  # noqa: BLE001
            err[r] = e

    th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
        assert not t.is_alive(), "loopback rank hung"
    for e in err:
        if e is not None:
            raise e
    return res


def _rows(torch, lists, layout, dtype=np.float32, tdtype=None):
    rows = np.zeros((max(1, len(lists)), layout.ld), dtype)
    for k, lay in enumerate(lists):
        layout.pack_row(lay, rows[k])
    t = torch.from_numpy(rows).cuda()
    if tdtype is not None:
        t = t.to(tdtype)
    return t[: len(lists)]


def _fedavg(G, K, combine, kind="f32", chunk_elems=4096):
    import torch

    from substrafl_amd.engine import fedavg_weights
    from substrafl_amd.layout import BucketLayout
    from substrafl_amd.sharding import (FedAvgShard, GpuShardOps, block_of, client_blocks, client_shard_fedavg,
                                        out_dtype)

    pus, ns = _data(K)
    if kind == "bf16":  # bf16-representable values: the reference runs on the exact upcast
        pus = [[(a.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32) for a in c] for c in pus]
    npdt = {"f32": np.float32, "bf16": np.float32, "f64": np.float64, "f16": np.float16}[kind]
    pus = [[a.astype(npdt) for a in c] for c in pus]
    layout = BucketLayout(range(len(SHAPES)), SHAPES, npdt)
    w = fedavg_weights(ns, kind)

    def rank_fn(r, tr):
        k0, k1 = client_blocks(K, G)[block_of(r, G)]
        rows = _rows(torch, pus[k0:k1], layout, dtype=npdt, tdtype=torch.bfloat16 if kind == "bf16" else None)
        out = torch.zeros(layout.ld, dtype=out_dtype(torch, kind), device="cuda")
        sh = FedAvgShard(kind, rows, w[k0:k1], k0, K, layout.M, layout.pairwise_idx)
        if client_shard_fedavg(sh, out, tr, GpuShardOps(), combine, chunk_elems=chunk_elems):
            torch.cuda.current_stream().synchronize()
            return out[: layout.M].cpu().numpy().copy()
        return None

    res = _loopback(G, rank_fn)
    assert all(x is None for x in res[1:])
    got = [a for _, a in layout.unpack(res[0])]
    return got, fedavg_reference_structure(pus, ns)


@pytest.mark.parametrize("G,K", [(2, 7), (3, 3), (4, 2), (8, 20)])
def test_relay_fedavg_bit_exact(G, K):
    got, ref = _fedavg(G, K, "relay")
    for g, r in zip(got, ref):
        assert g.shape == r.shape and np.array_equal(g.view(np.uint32), r.view(np.uint32))


def test_relay_fedavg_bf16_bit_exact():
    got, ref = _fedavg(4, 9, "relay", kind="bf16")
    for g, r in zip(got, ref):
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32))


@pytest.mark.parametrize("kind,bits", [("f64", np.uint64), ("f16", np.uint16)])
def test_relay_fedavg_other_kinds_bit_exact(kind, bits):
    """fp64 and fp16 buckets: the accumulator travels between ranks in the product type (NumPy's
    per-op rounding for fp16), the numel == 1 tree sums fp16 products in fp32."""
    got, ref = _fedavg(3, 11, "relay", kind=kind)
    for g, r in zip(got, ref):
        assert g.dtype == r.dtype and np.array_equal(g.view(bits), r.view(bits))


@pytest.mark.parametrize("combine", ["ordered", "rccl"])
def test_reassociating_combines_close(combine):
    got, ref = _fedavg(4, 13, combine)
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r, rtol=2e-5, atol=1e-5)
        if g.size == 1:  # the numel == 1 tensors are exact in every mode (pairwise tree on the root)
            assert np.array_equal(g.view(np.uint32), r.view(np.uint32))


def _scaffold(G, K, combine, lr=0.7, chunk_elems=4096):
    import torch

    from substrafl_amd.engine import scaffold_weights
    from substrafl_amd.layout import BucketLayout
    from substrafl_amd.sharding import (GpuShardOps, ScaffoldShard, block_of, client_blocks, client_shard_scaffold)

    pus, ns = _data(K, seed=1)
    rng = np.random.default_rng(9)
    cvs = [[rng.standard_normal(a.shape).astype(np.float32) for a in pu] for pu in pus]
    c = [rng.standard_normal(a.shape).astype(np.float32) for a in pus[0]]
    layout = BucketLayout(range(len(SHAPES)), SHAPES, np.float32)
    w = scaffold_weights(ns)

    def rank_fn(r, tr):
        k0, k1 = client_blocks(K, G)[block_of(r, G)]
        d = _rows(torch, pus[k0:k1], layout)
        v = _rows(torch, cvs[k0:k1], layout)
        ct = _rows(torch, [c], layout)[0]
        dout = torch.zeros(layout.ld, dtype=torch.float64, device="cuda")
        cout = torch.zeros(layout.ld, dtype=torch.float64, device="cuda")
        sh = ScaffoldShard("f32", d, v, ct, w[k0:k1], k0, K, layout.M, lr, layout.pairwise_idx)
        if client_shard_scaffold(sh, dout, cout, tr, GpuShardOps(), combine, chunk_elems=chunk_elems):
            torch.cuda.current_stream().synchronize()
            return dout[: layout.M].cpu().numpy().copy(), cout[: layout.M].cpu().numpy().copy()
        return None

    res = _loopback(G, rank_fn)
    lay64 = BucketLayout(range(len(SHAPES)), SHAPES, np.float64)
    d, cc = res[0]
    got = [a for _, a in lay64.unpack(cc)] + [a for _, a in lay64.unpack(d)]
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, lr)
    return got, rc + ra


@pytest.mark.parametrize("G,K", [(2, 5), (3, 2), (8, 17)])
def test_relay_scaffold_bit_exact(G, K):
    """c added last and lr applied on the root, inside its last kernel (or, for an empty last
    block, by the final-step launch) -- fp64 bit-exact."""
    got, ref = _scaffold(G, K, "relay")
    for g, r in zip(got, ref):
        assert g.dtype == np.float64 and np.array_equal(g.view(np.uint64), r.view(np.uint64))


@pytest.mark.parametrize("combine", ["ordered", "rccl"])
def test_scaffold_reassociating_combines_close(combine):
    got, ref = _scaffold(3, 10, combine)
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r, rtol=1e-12, atol=1e-13)
        if g.size == 1:
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64))


# ---- host entry points over RCCL, world size 1 ----
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _nccl_world1(q, port):
    import torch
    import torch.distributed as dist

    from substrafl_amd.sharding import client_sharded_fedavg, client_sharded_scaffold

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        pus, ns = _data(6, seed=3)
        out = {"fedavg": {m: client_sharded_fedavg(pus, ns, combine=m) for m in ("relay", "ordered", "rccl", "striped")}}
        for m in ("relay", "striped"):  # client blocks re-tiled on the device (TiledBlock)
            out["fedavg"][m + "_tiled"] = client_sharded_fedavg(pus, ns, combine=m, tiled=True)
        rng = np.random.default_rng(2)
        cvs = [[rng.standard_normal(a.shape).astype(np.float32) for a in pu] for pu in pus]
        c = [rng.standard_normal(a.shape).astype(np.float32) for a in pus[0]]
        cs = [[a.copy() for a in c] for _ in pus]  # separately unpickled copies: checked on the host
        out["scaffold"] = client_sharded_scaffold(pus, cvs, cs, ns, 0.5)
        out["scaffold_striped"] = client_sharded_scaffold(pus, cvs, cs, ns, 0.5, combine="striped")
        cs[3][2][17] += 1.0
        out["scaffold_bad"] = client_sharded_scaffold(pus, cvs, cs, ns, 0.5)[0]
        # round 2+ of Scaffold: fp64 control variates and c beside fp32 deltas (widened on the device)
        cvs64 = [[a.astype(np.float64) * 1.1 for a in cv] for cv in cvs]
        c64 = [[a.astype(np.float64) / 3 for a in c] for _ in pus]
        out["scaffold_mixed"] = client_sharded_scaffold(pus, cvs64, c64, ns, 0.5)
        try:
            client_sharded_fedavg([[a.astype(np.float16) if i == 0 else a for i, a in enumerate(p)] for p in pus], ns)
            out["mixed_fedavg"] = "accepted"
        except NotImplementedError:
            out["mixed_fedavg"] = "refused"
        q.put(out)
    finally:
        dist.destroy_process_group()


def test_host_entry_points_nccl_world1():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1, args=(q, _free_port()))
    p.start()
    out = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    pus, ns = _data(6, seed=3)
    ref = fedavg_reference_structure(pus, ns)
    for mode, got in out["fedavg"].items():
        for g, r in zip(got, ref):
            assert np.array_equal(g.view(np.uint32), r.view(np.uint32)), mode
    rng = np.random.default_rng(2)
    cvs = [[rng.standard_normal(a.shape).astype(np.float32) for a in pu] for pu in pus]
    c = [rng.standard_normal(a.shape).astype(np.float32) for a in pus[0]]
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.5)
    for key in ("scaffold", "scaffold_striped"):
        mism, new_c, avg = out[key]
        assert mism == 0
        for g, r in zip(new_c + avg, rc + ra):
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64)), key
    assert out["scaffold_bad"] == 1
    cvs64 = [[a.astype(np.float64) * 1.1 for a in cv] for cv in cvs]
    c64 = [a.astype(np.float64) / 3 for a in c]
    rc, ra = scaffold_reference_structure(pus, cvs64, c64, ns, 0.5)
    mism, new_c, avg = out["scaffold_mixed"]
    assert mism == 0
    for g, r in zip(new_c + avg, rc + ra):
        assert g.dtype == r.dtype == np.float64 and np.array_equal(g.view(np.uint64), r.view(np.uint64))
    assert out["mixed_fedavg"] == "refused"


@pytest.mark.parametrize("seed", range(12))
def test_relay_random_sweep(seed):
    """Random client counts (up to 300: blocks beyond one 128-client kernel-argument chunk
    continue their own accumulator too), rank counts, layer sets, dtypes and relay chunk sizes:
    the relay is bit-identical to the reference; Scaffold over > 64-client blocks likewise."""
    import torch

    from substrafl_amd.engine import fedavg_weights, scaffold_weights
    from substrafl_amd.layout import BucketLayout
    from substrafl_amd.sharding import (FedAvgShard, GpuShardOps, ScaffoldShard, block_of, client_blocks,
                                        client_shard_fedavg, client_shard_scaffold, out_dtype)

    rng = np.random.default_rng(1000 + seed)
    G = int(rng.integers(1, 9))
    K = int(rng.choice([1, 2, 5, 17, 70, 130, 300]))
    pool = [(1,), (1, 1), (3,), (129,), (4096,), (31, 7), (2, 2, 2)]
    shapes = [pool[i] for i in rng.integers(0, len(pool), int(rng.integers(1, 6)))]
    kind = ["f32", "bf16", "f64", "f16"][seed % 4]
    npdt = {"f32": np.float32, "bf16": np.float32, "f64": np.float64, "f16": np.float16}[kind]
    pus = [[(rng.standard_normal(s) * 10.0 ** rng.integers(-2, 3)).astype(npdt) for s in shapes] for _ in range(K)]
    if kind == "bf16":
        pus = [[(a.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32) for a in c] for c in pus]
    ns = [int(v) for v in rng.integers(1, 5000, K)]
    layout = BucketLayout(range(len(shapes)), shapes, npdt)
    chunk = int(rng.choice([512, 2048, 1 << 20]))
    w = fedavg_weights(ns, kind)

    def rank_fn(r, tr):
        k0, k1 = client_blocks(K, G)[block_of(r, G)]
        rows = _rows(torch, pus[k0:k1], layout, dtype=npdt, tdtype=torch.bfloat16 if kind == "bf16" else None)
        out = torch.zeros(layout.ld, dtype=out_dtype(torch, kind), device="cuda")
        sh = FedAvgShard(kind, rows, w[k0:k1], k0, K, layout.M, layout.pairwise_idx)
        if client_shard_fedavg(sh, out, tr, GpuShardOps(), "relay", chunk_elems=chunk):
            torch.cuda.current_stream().synchronize()
            return out[: layout.M].cpu().numpy().copy()
        return None

    got = [a for _, a in layout.unpack(_loopback(G, rank_fn)[0])]
    bits = {2: np.uint16, 4: np.uint32, 8: np.uint64}
    for g, r in zip(got, fedavg_reference_structure(pus, ns)):
        assert g.dtype == r.dtype and np.array_equal(g.view(bits[g.itemsize]), r.view(bits[r.itemsize]))

    if kind in ("f32", "f64") and K <= 130:
        cvs = [[rng.standard_normal(s).astype(npdt) for s in shapes] for _ in range(K)]
        c = [rng.standard_normal(s).astype(npdt) for s in shapes]
        lr = float(rng.choice([0.0, 0.5, 1.0, 1.7]))
        ws = scaffold_weights(ns)

        def srank(r, tr):
            k0, k1 = client_blocks(K, G)[block_of(r, G)]
            sh = ScaffoldShard(kind, _rows(torch, pus[k0:k1], layout, dtype=npdt),
                               _rows(torch, cvs[k0:k1], layout, dtype=npdt), _rows(torch, [c], layout, dtype=npdt)[0],
                               ws[k0:k1], k0, K, layout.M, lr, layout.pairwise_idx)
            dout = torch.zeros(layout.ld, dtype=torch.float64, device="cuda")
            cout = torch.zeros(layout.ld, dtype=torch.float64, device="cuda")
            if client_shard_scaffold(sh, dout, cout, tr, GpuShardOps(), "relay", chunk_elems=chunk):
                torch.cuda.current_stream().synchronize()
                return dout[: layout.M].cpu().numpy().copy(), cout[: layout.M].cpu().numpy().copy()
            return None

        d, cc = _loopback(G, srank)[0]
        lay64 = BucketLayout(range(len(shapes)), shapes, np.float64)
        rc, ra = scaffold_reference_structure(pus, cvs, c, ns, lr)
        for g, r in zip([a for _, a in lay64.unpack(cc)] + [a for _, a in lay64.unpack(d)], rc + ra):
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64))


# ---- striped relay: pieces rotating over the ranks on several rings (lockstep schedule) ----
def _striped(G, K, strategy="fedavg", kind="f32", rings=None, rounds=(0.75, 0.25), shapes=SHAPES, seed=4, lr=0.9,
             tv=0, relay=False, transports=None, repeat=1):
    import torch

    from substrafl_amd.engine import fedavg_weights, scaffold_weights
    from substrafl_amd.layout import BucketLayout
    from substrafl_amd.sharding import (FedAvgShard, GpuShardOps, ScaffoldShard, TiledBlock, client_blocks,
                                        lockstep_fedavg, lockstep_scaffold, out_dtype, relay_plan, striped_plan)

    npdt = {"f32": np.float32, "bf16": np.float32, "f64": np.float64, "f16": np.float16}[kind]
    pus, ns = _data(K, seed=seed, shapes=shapes)
    pus = [[a.astype(npdt) for a in c] for c in pus]
    if kind == "bf16":  # bf16-representable values: the reference runs on the exact upcast
        pus = [[(a.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32) for a in c] for c in pus]
    layout = BucketLayout(range(len(shapes)), shapes, npdt)
    rng = np.random.default_rng(seed + 1)
    cvs = [[rng.standard_normal(a.shape).astype(npdt) for a in pu] for pu in pus]
    c = [rng.standard_normal(a.shape).astype(npdt) for a in pus[0]]

    def rank_fn(r, tr):
        plan = relay_plan(layout.M, G, r, 4096) if relay else striped_plan(layout.M, G, r, rings, rounds)
        full_c = _rows(torch, [c], layout, dtype=npdt)[0]
        blocks = {}
        for b, segs in plan.blocks.items():
            k0, k1 = client_blocks(K, G)[b]

            def packed(lists):
                full = _rows(torch, lists, layout, dtype=npdt, tdtype=torch.bfloat16 if kind == "bf16" else None)
                t = torch.zeros((max(1, k1 - k0), plan.block_len[b]), dtype=full.dtype, device="cuda")
                for lo, hi, col in segs:
                    t[: k1 - k0, col: col + hi - lo] = full[:, lo:hi]
                return t[: k1 - k0]

            if strategy == "fedavg":
                rows = packed(pus[k0:k1])
                if tv and k1 > k0:
                    rows = TiledBlock.from_rows(torch, kind, rows, tv, TiledBlock.run_extents(plan, b))
                blocks[b] = FedAvgShard(kind, rows, fedavg_weights(ns, kind)[k0:k1], k0, K,
                                        plan.block_len[b], np.zeros(0, np.uint64))
            else:
                blocks[b] = ScaffoldShard(kind, packed(pus[k0:k1]), packed(cvs[k0:k1]), None,
                                          scaffold_weights(ns)[k0:k1], k0, K, plan.block_len[b], lr,
                                          np.zeros(0, np.uint64))
        got = None
        for _ in range(repeat):  # a repeated call reuses the compiled schedule (native executor)
            if strategy == "fedavg":
                out = torch.full((layout.ld,), float("nan"), dtype=out_dtype(torch, kind), device="cuda")
                if lockstep_fedavg(plan, blocks, out, tr, GpuShardOps(), layout.pairwise_idx):
                    torch.cuda.current_stream().synchronize()
                    got = out[: layout.M].cpu().numpy().copy()
                continue
            dout = torch.full((layout.ld,), float("nan"), dtype=torch.float64, device="cuda")
            cout = torch.full((layout.ld,), float("nan"), dtype=torch.float64, device="cuda")
            if lockstep_scaffold(plan, blocks, dout, cout, tr, GpuShardOps(), layout.pairwise_idx, full_c, lr):
                torch.cuda.current_stream().synchronize()
                got = dout[: layout.M].cpu().numpy().copy(), cout[: layout.M].cpu().numpy().copy()
        return got

    res = _loopback(G, rank_fn, transports)
    assert all(x is None for x in res[1:])
    if strategy == "fedavg":
        return [a for _, a in layout.unpack(res[0])], fedavg_reference_structure(pus, ns)
    lay64 = BucketLayout(range(len(shapes)), shapes, np.float64)
    d, cc = res[0]
    rc, ra = scaffold_reference_structure(pus, cvs, c, ns, lr)
    return [a for _, a in lay64.unpack(cc)] + [a for _, a in lay64.unpack(d)], rc + ra


@pytest.mark.parametrize("G,K,kind,rings,rounds", [(8, 20, "f32", None, (1.0,)), (4, 9, "f32", 2, (0.75, 0.25)),
                                                   (3, 2, "f64", None, (1.0,)), (2, 5, "f16", None, (0.5, 0.5)),
                                                   (8, 7, "f32", 3, (0.6, 0.3, 0.1)), (1, 4, "f32", None, (1.0,))])
def test_striped_relay_fedavg_bit_exact(G, K, kind, rings, rounds):
    """Every piece's chain visits the blocks in client order, so each element keeps the
    reference's rounding sequence; K < G leaves empty blocks in every stripe."""
    shapes = SHAPES + [(5000,), (1,)]
    got, ref = _striped(G, K, kind=kind, rings=rings, rounds=rounds, shapes=shapes)
    bits = {2: np.uint16, 4: np.uint32, 8: np.uint64}
    for g, r in zip(got, ref):
        assert g.dtype == r.dtype and np.array_equal(g.view(bits[g.itemsize]), r.view(bits[r.itemsize]))


@pytest.mark.parametrize("G,K,kind", [(8, 17, "f32"), (4, 3, "f64"), (2, 6, "f32")])
def test_striped_relay_scaffold_bit_exact(G, K, kind):
    shapes = SHAPES + [(5000,), (1,)]
    got, ref = _striped(G, K, strategy="scaffold", kind=kind, shapes=shapes)
    for g, r in zip(got, ref):
        assert g.dtype == np.float64 and np.array_equal(g.view(np.uint64), r.view(np.uint64))


@pytest.mark.parametrize("G,K,kind,tv,relay", [(2, 70, "f32", 8192, False), (3, 100, "f32", 2048, False),
                                               (2, 66, "bf16", 4096, False), (4, 130, "f32", 8192, True),
                                               (2, 64, "bf16", 4096, True), (8, 9, "f32", 2048, False)])
def test_tiled_client_blocks_bit_exact(G, K, kind, tv, relay):
    """Client blocks re-tiled run by run (TiledBlock: fedagg_fedavg_chain_tiled_*, >= 32 clients per
    block, partial tiles, numel == 1 products read through the tile map) -- the striped and the
    plain relay stay bit-identical to the reference."""
    shapes = [(37, 29), (1,), (40000,), (1, 1), (3, 3, 3), (70001,), (1,)]
    got, ref = _striped(G, K, kind=kind, shapes=shapes, tv=tv, relay=relay, rounds=(0.75, 0.25))
    for g, r in zip(got, ref):
        assert g.dtype == r.dtype and np.array_equal(g.view(np.uint32), r.view(np.uint32))


# ---- the native lockstep executor (csrc/lockstep.hip) over a real RCCL communicator ----
def _native_world1(q, port):
    import torch
    import torch.distributed as dist

    from substrafl_amd import lockstep
    from substrafl_amd.engine import fedavg_weights, scaffold_weights
    from substrafl_amd.layout import BucketLayout
    from substrafl_amd.rccl import RcclTransport
    from substrafl_amd.sharding import (FedAvgShard, GpuShardOps, LoopbackGroup, ScaffoldShard, TiledBlock,
                                        lockstep_fedavg, lockstep_scaffold, out_dtype, striped_plan)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    out = {}
    try:
        tr = RcclTransport()
        shapes = [(37, 29), (1,), (40000,), (1, 1), (5000,)]
        # (1) every run kind through the native executor: one rank, the schedule's runs, the
        #     numel == 1 workspace reduce; against the Python executor and the oracle
        for kind, tv in (("f32", 0), ("f32", 8192), ("bf16", 4096), ("f64", 0), ("f16", 0)):
            npdt = {"f32": np.float32, "bf16": np.float32, "f64": np.float64, "f16": np.float16}[kind]
            K = 33
            pus, ns = _data(K, seed=7, shapes=shapes)
            pus = [[a.astype(npdt) for a in c] for c in pus]
            if kind == "bf16":
                pus = [[(a.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32) for a in c] for c in pus]
            layout = BucketLayout(range(len(shapes)), shapes, npdt)
            plan = striped_plan(layout.M, 1, 0)
            rows = _rows(torch, pus, layout, dtype=npdt, tdtype=torch.bfloat16 if kind == "bf16" else None)
            segs = plan.blocks[0]
            packed = torch.zeros((K, plan.block_len[0]), dtype=rows.dtype, device="cuda")
            for lo, hi, col in segs:
                packed[:, col: col + hi - lo] = rows[:, lo:hi]
            data = TiledBlock.from_rows(torch, kind, packed, tv, TiledBlock.run_extents(plan, 0)) if tv else packed
            blocks = {0: FedAvgShard(kind, data, fedavg_weights(ns, kind), 0, K, plan.block_len[0],
                                     np.zeros(0, np.uint64))}
            res = []
            for t in (tr, LoopbackGroup(1).transport(0)):
                o = torch.zeros(layout.ld, dtype=out_dtype(torch, kind), device="cuda")
                lockstep_fedavg(plan, blocks, o, t, GpuShardOps(), layout.pairwise_idx)
                torch.cuda.synchronize()
                res.append(o[: layout.M].cpu().numpy().copy())
            out[f"fedavg_{kind}_{tv}"] = (res[0], res[1], pus, ns, shapes, npdt)
        # Scaffold, fp32 and fp64 buckets
        for kind in ("f32", "f64"):
            npdt = np.float32 if kind == "f32" else np.float64
            K = 9
            pus, ns = _data(K, seed=8, shapes=shapes)
            pus = [[a.astype(npdt) for a in c] for c in pus]
            rng = np.random.default_rng(3)
            cvs = [[rng.standard_normal(a.shape).astype(npdt) for a in c] for c in pus]
            c = [rng.standard_normal(a.shape).astype(npdt) for a in pus[0]]
            layout = BucketLayout(range(len(shapes)), shapes, npdt)
            plan = striped_plan(layout.M, 1, 0)

            def packed(lists):
                r = _rows(torch, lists, layout, dtype=npdt)
                t = torch.zeros((len(lists), plan.block_len[0]), dtype=r.dtype, device="cuda")
                for lo, hi, col in plan.blocks[0]:
                    t[:, col: col + hi - lo] = r[:, lo:hi]
                return t

            blocks = {0: ScaffoldShard(kind, packed(pus), packed(cvs), None, scaffold_weights(ns), 0, K,
                                       plan.block_len[0], 0.6, np.zeros(0, np.uint64))}
            ct = _rows(torch, [c], layout, dtype=npdt)[0]
            res = []
            for t in (tr, LoopbackGroup(1).transport(0)):
                d = torch.zeros(layout.ld, dtype=torch.float64, device="cuda")
                cc = torch.zeros(layout.ld, dtype=torch.float64, device="cuda")
                lockstep_scaffold(plan, blocks, d, cc, t, GpuShardOps(), layout.pairwise_idx, ct, 0.6)
                torch.cuda.synchronize()
                res.append((d[: layout.M].cpu().numpy().copy(), cc[: layout.M].cpu().numpy().copy()))
            out[f"scaffold_{kind}"] = (res[0], res[1], pus, cvs, c, ns, shapes, npdt)
        # (2) the exchange path: a hand-built schedule whose relay hop goes to the rank itself
        #     (send + receive in one RCCL group): block 0 at step 0 into a slot, group 1 moves it
        #     into the output, block 1 continues it at step 2 -- the full client sum, in order
        K0, K1 = 5, 6
        pus, ns = _data(K0 + K1, seed=9, shapes=shapes)
        layout = BucketLayout(range(len(shapes)), shapes, np.float32)
        n = layout.M
        plan = lockstep.RankPlan(
            rank=0, world=1, root=0,
            runs=[[lockstep.Run(0, 0, n, 0, ("slot", 0, 0), True, False)], [],
                  [lockstep.Run(1, 0, n, 0, ("out", 0, 0), False, True)]],
            groups=[[], [lockstep.Op("recv", 0, ("out", 0, 0), n, 0), lockstep.Op("send", 0, ("slot", 0, 0), n, 0)],
                    [], []],
            blocks={0: [(0, n, 0)], 1: [(0, n, 0)]}, block_len={0: n, 1: n}, slot_elems=n)
        w = fedavg_weights(ns, "f32")
        rows = _rows(torch, pus, layout)
        blocks = {0: FedAvgShard("f32", rows[:K0], w[:K0], 0, K0 + K1, n, np.zeros(0, np.uint64)),
                  1: FedAvgShard("f32", rows[K0:], w[K0:], K0, K0 + K1, n, np.zeros(0, np.uint64))}
        res = []
        for t in (tr, LoopbackGroup(1).transport(0)):
            o = torch.zeros(layout.ld, dtype=torch.float32, device="cuda")
            lockstep_fedavg(plan, blocks, o, t, GpuShardOps(), layout.pairwise_idx)
            torch.cuda.synchronize()
            res.append(o[:n].cpu().numpy().copy())
        out["self_exchange"] = (res[0], res[1], pus, ns, shapes, np.float32)
        tr.close()
        q.put(out)
    finally:
        dist.destroy_process_group()


def test_native_lockstep_executor_world1():
    """csrc/lockstep.hip over a one-rank RCCL communicator: every run kind (fp32 rows and tiles,
    bf16 tiles, fp64, fp16, Scaffold fp32 / fp64) and the numel == 1 workspace reduce, and a
    schedule whose exchange group sends to and receives from the rank itself -- bit-identical to
    the Python executor and to the reference."""
    import torch.multiprocessing as mp

    from substrafl_amd.layout import BucketLayout

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_native_world1, args=(q, _free_port()))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    bits = {2: np.uint16, 4: np.uint32, 8: np.uint64}
    for key, val in out.items():
        if key.startswith("scaffold"):
            (nd, nc), (pd, pc), pus, cvs, c, ns, shapes, npdt = val
            assert np.array_equal(nd.view(np.uint64), pd.view(np.uint64)), key
            assert np.array_equal(nc.view(np.uint64), pc.view(np.uint64)), key
            lay = BucketLayout(range(len(shapes)), shapes, np.float64)
            rc, ra = scaffold_reference_structure(pus, cvs, c, ns, 0.6)
            for g, r in zip([a for _, a in lay.unpack(nc)] + [a for _, a in lay.unpack(nd)], rc + ra):
                assert np.array_equal(g.view(np.uint64), r.view(np.uint64)), key
            continue
        nat, py, pus, ns, shapes, npdt = val
        assert np.array_equal(nat.view(bits[nat.itemsize]), py.view(bits[py.itemsize])), key
        lay = BucketLayout(range(len(shapes)), shapes, npdt)
        for g, r in zip([a for _, a in lay.unpack(nat)], fedavg_reference_structure(pus, ns)):
            assert g.dtype == r.dtype and np.array_equal(g.view(bits[g.itemsize]), r.view(bits[r.itemsize])), key


# ---- the native executor with G ranks: threads on one GPU over tests/native/libthread_rccl.so ----
THREAD_RCCL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libthread_rccl.so")

# (G, K, strategy, kind, rings, rounds, tv, relay); client_blocks(K, G) decides native or Python
NATIVE_THREAD_CASES = [
    (8, 70, "fedavg", "f32", None, (0.5, 0.3, 0.2), 0, False),   # the bench's schedule at G = 8
    (8, 20, "fedavg", "f32", 3, (1.0,), 0, False),             # ragged split (blocks of 2 and 3)
    (4, 9, "fedavg", "f32", 2, (0.75, 0.25), 0, True),          # relay
    (3, 100, "fedavg", "f32", None, (0.5, 0.3, 0.2), 2048, False),  # tiled blocks (>= 32 clients each)
    (2, 66, "fedavg", "bf16", None, (0.5, 0.3, 0.2), 4096, False),
    (3, 5, "fedavg", "f64", None, (0.6, 0.4), 0, False),
    (2, 5, "fedavg", "f16", None, (1.0,), 0, False),
    (8, 17, "scaffold", "f32", None, (0.5, 0.3, 0.2), 0, False),
    (4, 6, "scaffold", "f64", None, (1.0,), 0, False),
    (8, 5, "fedavg", "f32", None, (0.5, 0.3, 0.2), 0, False),    # K < G: empty blocks, the Python fallback
]


def _native_threads(q, cases):
    import ctypes
    import faulthandler
    import sys

    import torch

    faulthandler.dump_traceback_later(110, exit=True)  # a hang names its threads' stacks, then ends

    from substrafl_amd import _native, rccl
    from substrafl_amd.sharding import LoopbackGroup

    class ThreadTransport(rccl.RcclTransport):
        """RcclTransport over the thread-ranks stand-in (no torch process group): the native
        executor unchanged, its RCCL calls served by tests/native/thread_rccl.hip."""

        def __init__(self, uid, rank, world, py):
            self.lib, self.rank, self.world, self.device, self.group = _native.load(), rank, world, 0, None
            self._programs, self._py = [], py
            h = ctypes.c_void_p()
            rccl._check(self.lib.fedagg_comm_create(THREAD_RCCL.encode(), world, rank, uid, 0, ctypes.byref(h)),
                        "fedagg_comm_create")
            self._h = h

        def all_sum_int(self, v):
            return self._py.all_sum_int(v)

    torch.cuda.set_device(0)
    lib = _native.load()
    res = {}
    for i, (G, K, strategy, kind, rings, rounds, tv, relay) in enumerate(cases):
        print(f"[native threads] case {i}: {cases[i]}", file=sys.stderr, flush=True)
        uid = (ctypes.c_char * 128)()
        rccl._check(lib.fedagg_comm_unique_id(THREAD_RCCL.encode(), uid), "fedagg_comm_unique_id")
        py = LoopbackGroup(G)
        trs = [ThreadTransport(uid, r, G, py.transport(r)) for r in range(G)]
        shapes = SHAPES + [(5000,), (1,)] if not tv else [(37, 29), (1,), (40000,), (1, 1), (3, 3, 3), (70001,), (1,)]
        got, ref = _striped(G, K, strategy=strategy, kind=kind, rings=rings, rounds=rounds, shapes=shapes, tv=tv,
                            relay=relay, transports=trs, repeat=2, seed=11 + i)
        bits = {2: np.uint16, 4: np.uint32, 8: np.uint64}
        bad = sum(int(np.count_nonzero(g.view(bits[g.itemsize]) != r.view(bits[r.itemsize])))
                  + int(g.dtype != r.dtype or g.shape != r.shape) for g, r in zip(got, ref))
        programs = sum(len(t._programs) for t in trs)
        for t in trs:
            t.close()
        res[i] = (bad, programs)
    q.put(res)


@pytest.mark.skipif(not os.path.exists(THREAD_RCCL), reason="tests/native/libthread_rccl.so not built")
def test_native_executor_multi_rank_threads():
    """csrc/lockstep.hip with 2-8 ranks: each rank a thread with its own stream and communicator on
    the one GPU, RCCL's P2P / reduce served by the thread stand-in (real RCCL refuses two ranks on
    one GPU).  Every rank's compiled run / message tables, the cross-stream event order, slot reuse
    over 48 steps and the numel == 1 workspace reduce -- relay, striped (1-3 rounds), tiled blocks,
    every kind, Scaffold, called twice through the cached program -- bit-identical to the
    reference; K < G takes the Python fallback through the same transport."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_native_threads, args=(q, NATIVE_THREAD_CASES))
    p.start()
    try:
        res = q.get(timeout=130)
    finally:
        p.join(timeout=20)
        if p.is_alive():
            p.kill()  # our own child, by handle
    assert p.exitcode == 0
    from substrafl_amd.sharding import client_blocks

    for i, case in enumerate(NATIVE_THREAD_CASES):
        bad, programs = res[i]
        assert bad == 0, (case, bad)
        native = all(k1 > k0 for k0, k1 in client_blocks(case[1], case[0]))  # the same choice on every rank
        assert (programs > 0) == native, (case, programs)
