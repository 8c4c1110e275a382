"""Per-layer torch weight moves with the semantics the reference's ``weight_manager`` pins
(layer order = ``model.parameters()`` then every BatchNorm layer's running mean / var; a weighted
sum is Python ``sum()`` from int 0 over ``tensor * coefficient``; an increment is
``w += multiplier * u``), written for this stand-in as plain torch -- the semantics the
accelerated client kernels must reproduce bit for bit."""

import torch

_BN = (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d, torch.nn.BatchNorm3d)


def layers(model, bn: bool):
    out = list(model.parameters())
    if bn:
        for m in model.modules():
            if isinstance(m, _BN):
                out += [m.running_mean, m.running_var]
    return out


def snapshot(model, bn: bool):
    with torch.no_grad():
        return [t.clone() for t in layers(model, bn)]


def add_into(model, updates, bn: bool, multiplier: float = 1.0):
    with torch.no_grad():
        ws = layers(model, bn)
        assert len(ws) == len(updates)
        for w, u in zip(ws, updates):
            w.data += multiplier * u.data


def combine(lists, coeffs):
    with torch.no_grad():
        return [sum(t * c for t, c in zip(group, coeffs)) for group in zip(*lists)]


def rebind(model, tensors, bn: bool):
    with torch.no_grad():
        ws = layers(model, bn)
        assert len(ws) == len(tensors)
        for w, t in zip(ws, tensors):
            w.data = t.data


def zeros(model, bn: bool, device):
    with torch.no_grad():
        return [torch.zeros_like(t).to(device) for t in layers(model, bn)]
