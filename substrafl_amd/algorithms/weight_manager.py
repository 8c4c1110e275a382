"""Client-side bucket producer / consumer with flat-bucket HIP paths.

Same functions, signatures and results as the reference's
``substrafl/algorithms/pytorch/weight_manager.py`` (``model_parameters`` :53-76, ``get_parameters``
:79-100, ``increment_parameters`` :103-137, ``subtract_parameters`` :140-158, ``add_parameters``
:161-179, ``weighted_sum_parameters`` :182-212, ``set_parameters`` :215-238,
``zeros_like_parameters`` :241-265), so an algorithm can switch its import.  When every tensor is
fp32 on a ROCm device the per-layer torch loops become single launches of libfedagg's flat-bucket
kernels, and the tensors they return are views of ONE flat device bucket -- which
:func:`export_numpy` brings home with a single D2H copy (the wire format the aggregator stages
with one contiguous segment per client).  Other dtypes and CPU tensors keep the reference's torch
semantics (they are the client's own device choice, not the aggregation hot path).

Bit-exact with the reference's torch ops: ``weighted_sum_parameters`` is Python ``sum()`` from int 0
over ``param * coeff`` (so ``-0.0`` becomes ``+0.0``, and ``coeff`` is rounded to fp32 as torch does
for a Python scalar); ``increment_parameters`` is ``w += fl32(multiplier) * u``.
"""

from __future__ import annotations

import ctypes
from typing import Generator, List, Optional, Sequence

import numpy as np
import torch
from torch._utils import _unflatten_dense_tensors

from .. import _native
from ..wire import bucket_views, flat_of

_BN = (
    torch.nn.BatchNorm1d,
    torch.nn.BatchNorm2d,
    torch.nn.BatchNorm3d,
    torch.nn.LazyBatchNorm1d,
    torch.nn.LazyBatchNorm2d,
    torch.nn.LazyBatchNorm3d,
)


def is_batchnorm_layer(layer: torch.nn.Module) -> bool:
    return isinstance(layer, _BN)


def batch_norm_param(model: torch.nn.Module) -> Generator[torch.Tensor, None, None]:
    for _, module in model.named_modules():
        if is_batchnorm_layer(module):
            yield module.running_mean
            yield module.running_var


def model_parameters(model: torch.nn.Module, with_batch_norm_parameters: bool):
    """Generator factory: ``model.parameters()`` then (optionally) every BatchNorm layer's running
    mean and variance -- the bucket layer order (weight_manager.py:53-76)."""

    def my_iterator():
        for p in model.parameters():
            yield p
        if with_batch_norm_parameters:
            for p in batch_norm_param(model):
                yield p

    return my_iterator


# ----------------------------------------------------------------------------------------
# flat-bucket helpers
# ----------------------------------------------------------------------------------------
_KIND = {torch.float32: _native.FEDAGG_F32, torch.float64: _native.FEDAGG_F64}


def _kind(tensors: Sequence[torch.Tensor], device=None) -> Optional[int]:
    """The libfedagg kind when ``tensors`` are contiguous ROCm tensors of ONE dtype (fp32 or fp64)
    on one device (``device`` if given); else None (the op keeps the reference's torch loop)."""
    if not tensors:
        return None
    t0 = tensors[0]
    if not (t0.is_cuda and t0.dtype in _KIND):
        return None
    if device is None:
        idx = t0.get_device()
    else:
        d = torch.device(device)
        if d.type != "cuda":
            return None
        idx = d.index if d.index is not None else torch.cuda.current_device()
    dt = t0.dtype
    for t in tensors:  # get_device() is -1 on the CPU: one int compare covers device and placement
        if t.dtype != dt or t.get_device() != idx or not t.is_contiguous():
            return None
    return _KIND[dt]


def _fast(tensors: Sequence[torch.Tensor]) -> bool:
    return _kind(tensors) == _native.FEDAGG_F32


def _numel_array(tensors):
    return (ctypes.c_uint64 * max(1, len(tensors)))(*[t.numel() for t in tensors])


def _views(flat: torch.Tensor, like: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    """Per-layer views of ``flat`` shaped like ``like`` (one C++ call: per-layer ``narrow().view()``
    from Python cost ≈10 µs a layer, more than the flat kernels themselves on a 300-layer model)."""
    return list(_unflatten_dense_tensors(flat, list(like)))


def _stream(device) -> int:
    return int(torch.cuda.current_stream(device).cuda_stream)


def flat_bucket(tensors: Sequence[torch.Tensor]) -> Optional[torch.Tensor]:
    """The flat 1-D tensor the given tensors are consecutive views of, else None."""
    if not tensors:
        return None
    base = tensors[0]
    if not base.is_contiguous():
        return None
    storage = base.untyped_storage().data_ptr()
    start = base.storage_offset()
    off = start
    for t in tensors:
        if (t.untyped_storage().data_ptr() != storage or t.storage_offset() != off or not t.is_contiguous()
                or t.dtype != base.dtype):
            return None
        off += t.numel()
    total = off - start
    return torch.as_strided(base, (total,), (1,), start)


def _gather_flat(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    kind = _kind(tensors)
    flat = torch.empty(sum(t.numel() for t in tensors), dtype=tensors[0].dtype, device=tensors[0].device)
    lib = _native.load()
    _native.check(lib.fedagg_flat_gather(_native.ptr_array([t.data_ptr() for t in tensors]), kind,
                                         _numel_array(tensors), len(tensors), flat.data_ptr(),
                                         _stream(flat.device)), "flat_gather")
    return flat


# ----------------------------------------------------------------------------------------
# reference API
# ----------------------------------------------------------------------------------------
def get_parameters(model: torch.nn.Module, with_batch_norm_parameters: bool) -> List[torch.Tensor]:
    """Copies of the model parameters (weight_manager.py:79-100); on a ROCm device one gather
    launch into one flat bucket, returned as per-layer views."""
    with torch.no_grad():
        params = list(model_parameters(model, with_batch_norm_parameters=with_batch_norm_parameters)())
        if _kind(params) is not None:
            return _views(_gather_flat(params), params)
        return [p.clone() for p in params]


def increment_parameters(
    model: torch.nn.Module,
    updates: List,
    *,
    with_batch_norm_parameters: bool,
    updates_multiplier: float = 1.0,
):
    """``w += updates_multiplier * u`` for every model parameter (weight_manager.py:103-137)."""
    with torch.no_grad():
        params = list(model_parameters(model=model, with_batch_norm_parameters=with_batch_norm_parameters)())
        assert len(params) == len(updates), "Length of model parameters and updates are unequal."
        for w, u in zip(params, updates):
            assert tuple(u.shape) == tuple(w.data.shape), (
                f"The shape of the model weights ({w.data.shape}) and of the update ({u.shape}) "
                "passed in the updates argument are unequal."
            )
        if _fast([p.data for p in params]):
            flat = _device_flat(updates, params[0].device)
            if flat is not None:
                lib = _native.load()
                _native.check(lib.fedagg_flat_increment(_native.ptr_array([p.data.data_ptr() for p in params]),
                                                        _numel_array(params), len(params), flat.data_ptr(),
                                                        _KIND[flat.dtype], float(updates_multiplier),
                                                        _stream(flat.device)), "flat_increment")
                return
        for w, u in zip(params, updates):
            u = torch.from_numpy(u).to(w.device) if isinstance(u, np.ndarray) else u
            w.data += updates_multiplier * u.data


def _device_flat(updates, device) -> Optional[torch.Tensor]:
    """One device bucket (fp32 or fp64) holding ``updates`` back to back, None if they are not all
    of one of those dtypes."""
    if all(isinstance(u, torch.Tensor) for u in updates):
        if _kind(updates, device) is None:
            return None
        flat = flat_bucket(updates)
        return flat if flat is not None else _gather_flat(updates)
    if all(isinstance(u, np.ndarray) for u in updates) and updates[0].dtype in (np.float32, np.float64) and all(
            u.dtype == updates[0].dtype for u in updates):
        return _stage_host_layers(updates, torch.device(device))
    return None


def _stage_host_layers(arrays: Sequence[np.ndarray], device) -> torch.Tensor:
    """Host layers (one dtype) -> ONE flat device bucket through the native session's pinned ring:
    the layers are packed chunk by chunk into pinned memory by its workers while earlier chunks
    are on the PCIe link (``fedagg_session_stage``, one row of L segments) -- no host-side
    concatenation, no pageable copy.  Wherever the layers live: one unpickled array each (the
    subprocess / docker task inputs), or views of one aggregator output (simulation)."""
    from .. import runtime

    from .. import handoff

    idx = device.index if device.index is not None else torch.cuda.current_device()
    layers = [np.ascontiguousarray(a) for a in arrays]
    n = sum(int(a.size) for a in layers)
    dt = torch.float64 if layers[0].dtype == np.float64 else torch.float32  # the caller checked: one of the two
    flat = torch.empty(n, dtype=dt, device=torch.device("cuda", idx))
    if n:
        # the bucket may reuse memory torch's stream still reads: the copy starts after that stream
        torch.cuda.current_stream(flat.device).synchronize()
        with runtime.device_lock(idx):  # the session's ring is shared with the aggregation engine
            s = runtime.session(idx)
            # simulation mode: an aggregator output (or another client's export) still on this GPU
            # is copied device to device (handoff.py); otherwise staged through the pinned ring
            hit = handoff.lookup(list(arrays), idx)
            if hit is not None and hit[1] == n * flat.element_size():
                s.copy_d2d(flat.data_ptr(), hit[0], hit[1])
            else:
                s.stage(flat.data_ptr(), n * flat.element_size(), [layers])
            s.sync()
    return flat


def _host_flat(arrays: Sequence[np.ndarray]) -> Optional[np.ndarray]:
    """The 1-D array the given arrays are consecutive views of (the aggregator returns exactly
    that: per-layer views of one owned array), else None."""
    base = arrays[0].base if arrays[0].base is not None else arrays[0]
    if not isinstance(base, np.ndarray) or base.ndim != 1 or not base.flags.c_contiguous:
        return None
    start = arrays[0].__array_interface__["data"][0]
    b0 = base.__array_interface__["data"][0]
    off = start
    for a in arrays:
        if (a.base is not base and a is not base) or a.__array_interface__["data"][0] != off or not a.flags.c_contiguous:
            return None
        off += a.nbytes
    first = (start - b0) // base.itemsize
    return base[first : first + (off - start) // base.itemsize]


def weighted_sum_parameters(parameters_list: List[List[torch.Tensor]], coefficient_list: List[float]) -> List[torch.Tensor]:
    """``sum(param * coeff ...)`` per layer (weight_manager.py:182-212); fused into one launch."""
    assert all(
        len(parameters_list[0]) == len(parameters) for parameters in parameters_list
    ), "The number of parameters in each List is not the same"
    assert len(parameters_list) == len(coefficient_list), "There must be a coefficient for each List of parameters"
    for parameters_to_sum in zip(*parameters_list):
        assert all(
            parameters_to_sum[0].data.shape == parameter.data.shape for parameter in parameters_to_sum
        ), "The shape of the parameters are unequal."
    kinds = [_kind(lst, parameters_list[0][0].device if parameters_list[0] else None) for lst in parameters_list]
    if 1 <= len(parameters_list) <= _native.FEDAGG_FLAT_MAX_LISTS and all(k is not None for k in kinds):
        like = parameters_list[0]
        out_dtype = torch.float64 if _native.FEDAGG_F64 in kinds else torch.float32
        with torch.no_grad():
            out = torch.empty(sum(t.numel() for t in like), dtype=out_dtype, device=like[0].device)
            lib = _native.load()
            coeffs = (ctypes.c_double * len(coefficient_list))(*[float(c) for c in coefficient_list])
            _native.check(lib.fedagg_flat_wsum(_native.ptr_array([t.data_ptr() for lst in parameters_list for t in lst]),
                                               (ctypes.c_int * len(kinds))(*kinds), len(parameters_list), coeffs,
                                               _numel_array(like), len(like), out.data_ptr(), _KIND[out_dtype],
                                               _stream(out.device)), "flat_wsum")
        return _views(out, like)
    weighted_sum = []
    for parameters_to_sum in zip(*parameters_list):
        with torch.no_grad():
            weighted_sum.append(sum(param * coeff for param, coeff in zip(parameters_to_sum, coefficient_list)))
    return weighted_sum


def subtract_parameters(parameters: List[torch.Tensor], parameters_to_subtract: List[torch.Tensor]) -> List[torch.Tensor]:
    return weighted_sum_parameters(parameters_list=[parameters, parameters_to_subtract], coefficient_list=[1, -1])


def add_parameters(parameters: List[torch.Tensor], parameters_to_add: List[torch.Tensor]) -> List[torch.Tensor]:
    return weighted_sum_parameters(parameters_list=[parameters, parameters_to_add], coefficient_list=[1, 1])


def set_parameters(model: torch.nn.Module, parameters: List[torch.Tensor], with_batch_norm_parameters: bool):
    """Rebind every model parameter's data to the given tensors (weight_manager.py:215-238)."""
    with torch.no_grad():
        iter_params = model_parameters(model, with_batch_norm_parameters=with_batch_norm_parameters)
        n_parameters = len(list(iter_params()))
        assert n_parameters == len(parameters), "Length of model parameters and provided parameters are unequal."
        for p, w in zip(iter_params(), parameters):
            p.data = w.data


def zeros_like_parameters(model: torch.nn.Module, with_batch_norm_parameters: bool, device: torch.device):
    with torch.no_grad():
        params = list(model_parameters(model, with_batch_norm_parameters=with_batch_norm_parameters)())
        if params and torch.device(device).type == "cuda" and all(p.dtype == torch.float32 for p in params):
            flat = torch.zeros(sum(p.numel() for p in params), dtype=torch.float32, device=device)
            return _views(flat, params)
        return [torch.zeros_like(p).to(device) for p in params]


def export_numpy(tensors: Sequence[torch.Tensor], wire: bool = True, tag: str = "export") -> List[np.ndarray]:
    """``[p.cpu().detach().numpy() for p in ...]`` (torch_fed_avg_algo.py:227-230) with ONE D2H copy
    when the tensors are views of one flat bucket.  With ``wire`` the arrays returned are
    :class:`wire.BucketArray` layers of one host buffer -- they pickle as that one buffer, and the
    aggregator stages the client as a single segment; without it they are plain ``np.ndarray``
    views of that buffer, which any process unpickles (no ``substrafl_amd`` import needed).
    ``tag`` names the host buffer recycled across calls (``runtime.reusable_host_array``): exports
    that are alive together (Scaffold's three lists) need one tag each, or every round after the
    first re-faults a fresh buffer for all but one of them."""
    flat = flat_bucket(list(tensors))
    if flat is None or not flat.is_cuda:
        return [t.cpu().detach().numpy() for t in tensors]
    from .. import handoff, runtime

    # one D2H through the native session's pinned ring (chunked, copied out by its worker pool)
    host = runtime.reusable_host_array(flat.numel(), torch.empty(0, dtype=flat.dtype).numpy().dtype,
                                       tag)  # bf16 raises, as .numpy()
    torch.cuda.current_stream(flat.device).synchronize()  # the bucket was written on torch's stream
    with runtime.device_lock(flat.device.index):  # the session's ring is shared with the engine
        runtime.session(flat.device.index).fetch(flat.data_ptr(), host)
    handoff.record_tensor(host, flat)  # simulation mode (opt-in): freezes host, keeps flat for the aggregator
    shapes = [tuple(t.shape) for t in tensors]
    if wire:
        return bucket_views(host, shapes)
    out, off = [], 0
    for shp in shapes:
        n = int(np.prod(shp, dtype=np.int64)) if len(shp) else 1
        out.append(host[off : off + n].reshape(shp))
        off += n
    return out


def to_device(arrays: Sequence[np.ndarray], device) -> List[torch.Tensor]:
    """``[torch.from_numpy(x).to(device) for x in arrays]`` (torch_scaffold_algo.py:397,404-406):
    on a ROCm device, when the arrays share one fp32 or fp64 dtype, ONE host->device copy into a
    flat bucket, returned as per-layer views (so the flat kernels take the bucket as is)."""
    arrays = list(arrays)
    d = torch.device(device)
    if d.type == "cuda" and arrays and all(isinstance(a, np.ndarray) for a in arrays):
        flat = _device_flat(arrays, d)
        if flat is not None:
            shapes = [a.shape for a in arrays]
            return [v.view(s) for v, s in zip(torch.split(flat, [int(np.prod(s, dtype=np.int64)) for s in shapes]),
                                               shapes)]
    return [torch.from_numpy(x).to(d) for x in arrays]

