"""Client-side bucket producer / consumer (substrafl_amd.algorithms.weight_manager) against the
reference's torch semantics (weight_manager.py:53-265, restated inline with the same torch ops)."""

import numpy as np
import pytest
import torch

from substrafl_amd import wire
from substrafl_amd.algorithms import weight_manager as wm


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = torch.nn.Conv2d(3, 8, 3)
        self.bn = torch.nn.BatchNorm2d(8)
        self.fc = torch.nn.Linear(8 * 6 * 6, 10)
        self.head = torch.nn.Linear(10, 1)

    def forward(self, x):
        return self.head(self.fc(torch.relu(self.bn(self.conv(x))).flatten(1)))


def ref_wsum(lists, coeffs):  # weight_manager.py:205-210
    return [sum(p * c for p, c in zip(ps, coeffs)) for ps in zip(*lists)]


def _same(a, b):
    return a.shape == b.shape and torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))


def _model(device, seed=0):
    torch.manual_seed(seed)
    m = Net().to(device)
    with torch.no_grad():
        m.bn.running_mean.normal_()
        m.bn.running_var.uniform_(0.5, 2.0)
        m.head.bias.fill_(-0.0)  # signed zero through the weighted sum
    return m


def test_layer_order_and_cpu_semantics():
    m = _model("cpu")
    names = [p.shape for p in wm.model_parameters(m, True)()]
    assert names[-2:] == [torch.Size([8]), torch.Size([8])] and len(names) == 10
    a = wm.get_parameters(m, True)
    b = [t * 3 for t in a]
    for got, ref in zip(wm.subtract_parameters(b, a), ref_wsum([b, a], [1, -1])):
        assert _same(got, ref)


def test_host_flat_detects_engine_style_views():
    flat = np.arange(20, dtype=np.float32)
    views = [flat[0:6].reshape(2, 3), flat[6:7], flat[7:20].reshape(13)]
    got = wm._host_flat(views)
    assert got is not None and got.size == 20 and np.shares_memory(got, flat)
    assert wm._host_flat([flat[0:6].reshape(2, 3), flat[8:9]]) is None


@pytest.fixture(params=[1, 0], ids=["vec16", "scalar"])
def flat_path(request):
    """Run a client-op test on the 16-B fp32 kernel and on the generic scalar kernel."""
    from substrafl_amd import _native

    _native.tune(flat_vec=request.param)
    yield request.param
    _native.tune(flat_vec=1)


@pytest.mark.gpu
def test_flat_ops_bit_exact_vs_torch_semantics(flat_path):
    assert torch.cuda.is_available()
    m = _model("cuda")
    old = wm.get_parameters(m, True)
    ref_old = [p.detach().clone() for p in wm.model_parameters(m, True)()]
    assert all(_same(a, b) for a, b in zip(old, ref_old))
    assert wm.flat_bucket(old) is not None  # one bucket

    # a "training step" changes the weights
    with torch.no_grad():
        for p in wm.model_parameters(m, True)():
            p.add_(torch.randn_like(p) * 1e-2)
    new = wm.get_parameters(m, True)
    delta = wm.subtract_parameters(new, old)  # torch_fed_avg_algo.py:212-218
    for got, ref in zip(delta, ref_wsum([new, old], [1, -1])):
        assert _same(got, ref)

    # Scaffold control-variate update (torch_scaffold_algo.py:451-458): {-1, -1/(lr*n)}
    c = [torch.randn_like(t) for t in new]
    rm = -1.0 / (0.05 * 100)
    got = wm.weighted_sum_parameters([c, delta], [-1.0, rm])
    for g, r in zip(got, ref_wsum([c, delta], [-1.0, rm])):
        assert _same(g, r)

    # increment with a multiplier, from device tensors and from host arrays (aggregator output)
    m2 = _model("cuda", seed=1)
    m3 = _model("cuda", seed=1)
    wm.increment_parameters(m2, delta, with_batch_norm_parameters=True, updates_multiplier=0.3)
    with torch.no_grad():
        for w, u in zip(wm.model_parameters(m3, True)(), delta):
            w.data += 0.3 * u.data  # weight_manager.py:137
    for a, b in zip(wm.model_parameters(m2, True)(), wm.model_parameters(m3, True)()):
        assert _same(a.data, b.data)
    host = wm.export_numpy(delta)
    assert all(isinstance(h, np.ndarray) for h in host) and wire.flat_of(host) is not None
    wm.increment_parameters(m2, host, with_batch_norm_parameters=True)
    with torch.no_grad():
        for w, u in zip(wm.model_parameters(m3, True)(), host):
            w.data += 1.0 * torch.from_numpy(u).cuda()
    for a, b in zip(wm.model_parameters(m2, True)(), wm.model_parameters(m3, True)()):
        assert _same(a.data, b.data)


@pytest.mark.gpu
def test_flat_ops_many_layers(flat_path):
    """> 32 layers (several launches of the segmented kernel) and layers > 8192 elements."""
    torch.manual_seed(3)
    a = [torch.randn(int(n), device="cuda") for n in np.random.default_rng(0).integers(1, 40000, 75)]
    b = [torch.randn_like(t) for t in a]
    for g, r in zip(wm.subtract_parameters(a, b), ref_wsum([a, b], [1, -1])):
        assert _same(g, r)
    flat = wm._gather_flat(a)
    assert torch.equal(flat, torch.cat(a))
    # signed zeros: Python sum() starts from int 0, so -0.0 - (+0.0) is +0.0 (p - q would be -0.0)
    z = [torch.full((5,), -0.0, device="cuda")]
    o = [torch.zeros(5, device="cuda")]
    got = wm.subtract_parameters(z, o)[0]
    assert _same(got, ref_wsum([z, o], [1, -1])[0]) and not torch.signbit(got).any()


@pytest.mark.gpu
def test_scaffold_client_round_mixed_fp64_vs_torch():
    """A Scaffold client round (torch_scaffold_algo.py:405-481) after the first aggregation: the
    server control variate arrives as fp64 (scaffold.py outputs fp64), so the client's torch ops
    promote -- the flat kernels follow that promotion bit for bit."""
    assert torch.cuda.is_available()
    lr, num_updates = 0.05, 7
    m_ref, m = _model("cuda", seed=4), _model("cuda", seed=4)
    shapes = [p.shape for p in wm.model_parameters(m, True)()]
    g = torch.Generator(device="cuda").manual_seed(11)
    server_c = [torch.randn(s, device="cuda", dtype=torch.float64, generator=g) * 1e-2 for s in shapes]
    client_c = [torch.randn(s, device="cuda", dtype=torch.float32, generator=g) * 1e-2 for s in shapes]

    def params(model):
        return list(wm.model_parameters(model, True)())

    # reference semantics, spelled with the reference's own torch expressions
    orig_ref = [p.detach().clone() for p in params(m_ref)]
    delta_v_ref = ref_wsum([client_c, server_c], [1, -1])
    # ours
    orig = wm.get_parameters(m, True)
    delta_v = wm.subtract_parameters(client_c, server_c)
    assert all(d.dtype == torch.float64 for d in delta_v)
    assert all(_same64(a, b) for a, b in zip(delta_v, delta_v_ref))
    for step in range(num_updates):
        noise = [torch.randn(s, device="cuda", generator=g) * 1e-3 for s in shapes]
        with torch.no_grad():
            for p, p2, n in zip(params(m_ref), params(m), noise):  # the optimizer step
                p.add_(n)
                p2.add_(n)
            for w, u in zip(params(m_ref), delta_v_ref):  # weight_manager.py:137
                w.data += lr * u.data
        wm.increment_parameters(m, delta_v, with_batch_norm_parameters=True, updates_multiplier=lr)
        assert all(_same(a.data, b.data) for a, b in zip(params(m), params(m_ref))), step
    pu_ref = ref_wsum([[p.detach().clone() for p in params(m_ref)], orig_ref], [1, -1])
    pu = wm.subtract_parameters(wm.get_parameters(m, True), orig)
    assert all(_same(a, b) for a, b in zip(pu, pu_ref))
    rm = -1.0 / (lr * num_updates)
    cvu_ref = ref_wsum([server_c, pu_ref], [-1.0, rm])
    cvu = wm.weighted_sum_parameters([server_c, pu], [-1.0, rm])
    assert all(a.dtype == torch.float64 and _same64(a, b) for a, b in zip(cvu, cvu_ref))
    new_c_ref = ref_wsum([client_c, cvu_ref], [1, 1])
    new_c = wm.add_parameters(client_c, cvu)
    assert all(_same64(a, b) for a, b in zip(new_c, new_c_ref))
    # fp64 host arrays (the aggregator's Scaffold output) applied to an fp32 model
    host = wm.export_numpy(new_c)
    assert all(h.dtype == np.float64 for h in host)
    wm.increment_parameters(m, host, with_batch_norm_parameters=True)
    with torch.no_grad():
        for w, u in zip(params(m_ref), host):
            w.data += 1.0 * torch.from_numpy(np.asarray(u)).cuda().data
    assert all(_same(a.data, b.data) for a, b in zip(params(m), params(m_ref)))


def _same64(a, b):
    return a.shape == b.shape and a.dtype == b.dtype and torch.equal(a.contiguous().view(torch.int64),
                                                                      b.contiguous().view(torch.int64))


def test_host_result_buffer_reused_only_when_released():
    """D2H result buffers (export_numpy, the engine's outputs) are recycled across calls (no 100 MB
    of fresh page faults per call) only when no array handed out from them is alive."""
    from substrafl_amd.runtime import reusable_host_array
    from substrafl_amd.wire import bucket_views

    a = reusable_host_array(100, np.float32, "t")
    held = bucket_views(a, [(10, 10)])
    del a
    b = reusable_host_array(100, np.float32, "t")
    assert not np.shares_memory(b, held[0])
    ptr = b.__array_interface__["data"][0]
    del b
    c = reusable_host_array(64, np.float32, "t")  # smaller request: a prefix of the released buffer
    assert c.__array_interface__["data"][0] == ptr
    assert not np.shares_memory(reusable_host_array(8, np.float32, "other"), c)  # per call site
    assert not np.shares_memory(reusable_host_array(8, np.float64, "t"), c)  # per dtype
    views = [c[:10].reshape(2, 5), c[10:20]]  # plain views (the engine's per-layer outputs) hold it too
    del c
    d = reusable_host_array(64, np.float32, "t")
    assert not any(np.shares_memory(d, v) for v in views)


def test_host_result_buffers_pooled_across_held_rounds():
    """Simulation mode holds round r's results while round r+1's are made (the strategy keeps its
    last train states and last average until the new ones return): two buffers per call site then
    alternate instead of one fresh allocation per call; the pool is bounded."""
    from substrafl_amd import runtime

    ptrs = []
    held = runtime.reusable_host_array(1000, np.float32, "pool_t")
    ptrs.append(held.__array_interface__["data"][0])
    for _ in range(6):
        nxt = runtime.reusable_host_array(1000, np.float32, "pool_t")  # made while the last is held
        assert not np.shares_memory(nxt, held)
        ptrs.append(nxt.__array_interface__["data"][0])
        held = nxt  # the previous round's result is released here
    assert len(set(ptrs)) == 2, ptrs
    keep = [runtime.reusable_host_array(10, np.float64, "pool_cap") for _ in range(runtime.HOST_POOL_DEPTH + 3)]
    assert len(runtime._host_cache[("pool_cap", np.dtype(np.float64))]["pool"]) == runtime.HOST_POOL_DEPTH
    assert len({a.__array_interface__["data"][0] for a in keep}) == len(keep)  # every live one distinct


def test_host_result_pool_byte_cap(monkeypatch):
    """Past ``HOST_POOL_BYTES`` per site the least recently used buffers are forgotten."""
    from substrafl_amd import runtime

    monkeypatch.setattr(runtime, "HOST_POOL_BYTES", 10_000)
    keep = [runtime.reusable_host_array(1000, np.float32, "pool_bytes") for _ in range(5)]  # 4000 B each
    pool = runtime._host_cache[("pool_bytes", np.dtype(np.float32))]["pool"]
    assert len(pool) == 2 and pool[-1][0] is keep[-1]  # a fresh buffer is handed out itself


def test_host_result_pool_follows_a_shrinking_working_set():
    """the pool is sized by the working set it sees -- six results held at once grow it
    to six buffers; once only one is held at a time, the five that stay free past HOST_POOL_IDLE
    turns of the pool are released (not kept for the life of the process)."""
    from substrafl_amd import runtime

    key = ("pool_shrink", np.dtype(np.float32))
    held = [runtime.reusable_host_array(1000, np.float32, "pool_shrink") for _ in range(6)]
    assert len(runtime._host_cache[key]["pool"]) == 6
    del held
    for _ in range(runtime.HOST_POOL_IDLE * 6 + 4):
        a = runtime.reusable_host_array(1000, np.float32, "pool_shrink")
        del a
    assert len(runtime._host_cache[key]["pool"]) == 1
    runtime.drop_host_pools()
    assert key not in runtime._host_cache
