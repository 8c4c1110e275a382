"""The reference's own weight-manager tests (tests/algorithms/pytorch/test_weight_manager.py:9-205)
restated against substrafl_amd.algorithms.weight_manager, on the CPU (the reference's torch loop)
and on the GPU (the flat-bucket kernels: gather, wsum, increment), so the client-side bucket
producer / consumer is checked with the reference's own expectations."""

from collections import OrderedDict

import pytest
import torch

from substrafl_amd.algorithms import weight_manager

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(device):
    if device == "cuda":
        assert torch.cuda.is_available(), "GPU tests need an MI355X"
        from substrafl_amd import _native

        _native.load()  # the flat path must be the one that runs
    return torch.device(device)


class _BatchNormNetwork(torch.nn.Module):  # test_weight_manager.py:9-19
    def __init__(self):
        super().__init__()
        self.bn1 = torch.nn.BatchNorm1d(num_features=1)

    def forward(self, x):
        return x


class _Perceptron(torch.nn.Module):  # tests/conftest.py:323-341 (LINEAR_N_COL = 3, one target)
    def __init__(self):
        super().__init__()
        self.linear1 = torch.nn.Linear(3, 1)

    def forward(self, x):
        return self.linear1(x)


MODELS = {"torch_linear_model": _Perceptron, "batch_norm_network": _BatchNormNetwork}


def _bn_state():
    return OrderedDict([("bn1.weight", torch.tensor([5.0])), ("bn1.bias", torch.tensor([3.0])),
                        ("bn1.running_mean", torch.tensor([0.0])), ("bn1.running_var", torch.tensor([1.0])),
                        ("bn1.num_batches_tracked", torch.tensor(0))])


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("make, num_parameters, init_shape", [
    (lambda: torch.nn.Linear(1, 1), 2, (10, 1)),
    (lambda: torch.nn.Conv1d(in_channels=1, out_channels=1, kernel_size=1), 2, (1, 1)),
    (lambda: torch.nn.BatchNorm1d(num_features=1), 4, (2, 1, 1)),
    (lambda: torch.nn.BatchNorm2d(num_features=1), 4, (2, 1, 1, 1)),
    (lambda: torch.nn.BatchNorm3d(num_features=1), 4, (2, 1, 1, 1, 1)),
    (lambda: torch.nn.LazyBatchNorm1d(), 4, (1, 2, 3)),
    (lambda: torch.nn.LazyBatchNorm2d(), 4, (1, 2, 3, 4)),
    (lambda: torch.nn.LazyBatchNorm3d(), 4, (1, 2, 3, 4, 5)),
])
def test_get_parameters(device, make, num_parameters, init_shape):
    dev = _dev(device)
    model = make().to(dev)
    model(torch.ones(init_shape, device=dev))  # lazy layers materialise here
    params = list(weight_manager.get_parameters(model=model, with_batch_norm_parameters=True))
    assert len(params) == num_parameters
    ref = [p.detach() for p in model.parameters()]
    if num_parameters == 4:
        ref += [model.running_mean, model.running_var]
    for got, want in zip(params, ref):
        assert torch.equal(got, want) and got.data_ptr() != want.data_ptr()  # copies, not the live tensors


@pytest.mark.parametrize("device", DEVICES)
def test_get_parameters_no_batch_norm(device):
    dev = _dev(device)
    model = _BatchNormNetwork()
    model.load_state_dict(_bn_state())
    model.to(dev)
    params = list(weight_manager.get_parameters(model=model, with_batch_norm_parameters=False))
    assert len(params) == 2
    assert torch.equal(params[0].cpu(), torch.tensor([5.0]))
    assert torch.equal(params[1].cpu(), torch.tensor([3.0]))


@pytest.mark.parametrize("device", DEVICES)
def test_get_batch_norm_layer(device):
    dev = _dev(device)
    model = _BatchNormNetwork()
    model.load_state_dict(_bn_state())
    model.to(dev)
    params = list(weight_manager.get_parameters(model=model, with_batch_norm_parameters=True))
    assert len(params) == 4
    assert torch.equal(params[-2].cpu(), torch.Tensor([0.0]))  # running mean
    assert torch.equal(params[-1].cpu(), torch.Tensor([1.0]))  # running var


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("model", list(MODELS))
@pytest.mark.parametrize("with_bn", [True, False])
def test_set_parameters(device, model, with_bn):
    dev = _dev(device)
    torch.manual_seed(42)
    m = MODELS[model]().to(dev)
    new = [torch.randn_like(p) for p in weight_manager.get_parameters(model=m, with_batch_norm_parameters=with_bn)]
    weight_manager.set_parameters(model=m, parameters=new, with_batch_norm_parameters=with_bn)
    for a, b in zip(new, weight_manager.get_parameters(model=m, with_batch_norm_parameters=with_bn)):
        assert torch.equal(a, b)


def _twins(model, dev):
    torch.manual_seed(42)
    m1 = MODELS[model]().to(dev)
    torch.manual_seed(42)
    m2 = MODELS[model]().to(dev)
    return m1, m2


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("model", list(MODELS))
@pytest.mark.parametrize("with_bn", [True, False])
def test_subtract_parameters(device, model, with_bn):
    m1, m2 = _twins(model, _dev(device))
    diff = weight_manager.subtract_parameters(
        weight_manager.get_parameters(m1, with_batch_norm_parameters=with_bn),
        weight_manager.get_parameters(m2, with_batch_norm_parameters=with_bn))
    for p in diff:
        assert torch.equal(p, torch.zeros_like(p))


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("model", list(MODELS))
@pytest.mark.parametrize("with_bn", [True, False])
def test_increment_parameters(device, model, with_bn):
    # running mean stays 0 (0 + 0) and running var becomes 2 (1 + 1) on the batch-norm network
    m1, m2 = _twins(model, _dev(device))
    weight_manager.increment_parameters(model=m1, updates=weight_manager.get_parameters(
        m2, with_batch_norm_parameters=with_bn), with_batch_norm_parameters=with_bn)
    p1 = weight_manager.get_parameters(m1, with_batch_norm_parameters=with_bn)
    p2 = weight_manager.get_parameters(m2, with_batch_norm_parameters=with_bn)
    for a, b in zip(p1, p2):
        assert torch.equal(a, 2 * b)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("model", list(MODELS))
@pytest.mark.parametrize("with_bn", [True, False])
def test_add_parameters(device, model, with_bn):
    m1, m2 = _twins(model, _dev(device))
    added = weight_manager.add_parameters(
        weight_manager.get_parameters(m1, with_batch_norm_parameters=with_bn),
        weight_manager.get_parameters(m2, with_batch_norm_parameters=with_bn))
    for a, b in zip(added, weight_manager.get_parameters(m1, with_batch_norm_parameters=with_bn)):
        assert torch.equal(a, 2 * b)


@pytest.mark.parametrize("device", DEVICES)
def test_weighted_sum_parameters(device):
    dev = _dev(device)
    params = [torch.tensor([1.0, 2.0, 3.0], device=dev), torch.tensor([1.0, 2.0, 3.0], device=dev)]
    out = weight_manager.weighted_sum_parameters(parameters_list=[params, params], coefficient_list=[-1.0, 2.0])
    for a, b in zip(out, params):
        assert torch.equal(a, b)


@pytest.mark.parametrize("device", DEVICES)
def test_zeros_like_parameters(device):
    dev = _dev(device)
    torch.manual_seed(0)
    m = _BatchNormNetwork().to(dev)
    z = weight_manager.zeros_like_parameters(m, with_batch_norm_parameters=True, device=dev)
    ref = list(weight_manager.get_parameters(m, with_batch_norm_parameters=True))
    assert len(z) == len(ref)
    for a, b in zip(z, ref):
        assert a.shape == b.shape and a.dtype == b.dtype and a.device == b.device and not a.any()


def test_length_mismatches_raise():
    m = _Perceptron()
    params = weight_manager.get_parameters(m, with_batch_norm_parameters=False)
    with pytest.raises(AssertionError):
        weight_manager.set_parameters(m, params[:1], with_batch_norm_parameters=False)
    with pytest.raises(AssertionError):
        weight_manager.increment_parameters(m, params[:1], with_batch_norm_parameters=False)
    with pytest.raises(AssertionError):
        weight_manager.weighted_sum_parameters([params, params[:1]], [1.0, 1.0])
    with pytest.raises(AssertionError):
        weight_manager.weighted_sum_parameters([params, params], [1.0])
