"""CPU restatement of the reference aggregation arithmetic (TEST INFRASTRUCTURE ONLY).

Two restatements of each strategy live here:

* ``*_reference_structure`` keeps the reference's call structure exactly -- per
  layer a Python list of ``x_k * w_k`` temporaries, then ``np.sum(list, axis=0)``
  -- so that timing it on the GPU box's host cores is a faithful stand-in for the
  reference CPU path (the reference itself never travels there).  It is the
  ``cpu_baseline`` ("port") leg of ``bench.py``.
* ``*_explicit`` spells out the bit-level order those NumPy calls perform
  (SURVEY.md §8.0 N1/N2/N6): per element a sequential fp32 (or fp64) chain over
  clients in list order, except for ``numel == 1`` tensors where NumPy reduces
  along the contiguous axis with its 8-accumulator pairwise sum.  The HIP
  kernels implement this order; the explicit form documents it and is checked
  against the structure form and against the golden vectors.

Reference anchors:
  FedAvg.avg_shared_states      substrafl/strategies/fed_avg.py:176-224 (arith 217-222)
  Scaffold.avg_shared_states    substrafl/strategies/scaffold.py:297-337
  Scaffold._weight_arrays       substrafl/strategies/scaffold.py:204-231
  Scaffold._update_server_control_variate  scaffold.py:233-265 (c appended last, 262-263)
  Scaffold._avg_weight_update   substrafl/strategies/scaffold.py:267-295 (lr * sum, 293)
  NewtonRaphson.compute_averaged_states  substrafl/strategies/newton_raphson.py:151-216
                                (explicit in-place += chain from client 0's product, 195-211)
  NumPy pairwise summation      numpy/_core/src/umath/loops_utils.h.src (pairwise_sum,
                                PW_BLOCKSIZE 128), numpy 2.x -- third-party, restated below.
"""

from __future__ import annotations

from typing import List, Sequence

import numpy as np

PW_BLOCKSIZE = 128


# --------------------------------------------------------------------------------------
# weights
# --------------------------------------------------------------------------------------
def fedavg_weights_f32(n_samples: Sequence[int]) -> np.ndarray:
    """``fl32(n_k / n)`` with ``n = sum(n_k)`` a Python int and ``/`` a double division.

    fed_avg.py:217 (``n_all_samples = sum(...)``) and :221 (``state.n_samples / n_all_samples``
    is a Python float; multiplying an fp32 array by it casts it to fp32 first, NEP 50).
    """
    n_all = sum(int(n) for n in n_samples)
    return np.array([float(int(n) / n_all) for n in n_samples], dtype=np.float64).astype(np.float32)


def scaffold_weights_f64(n_samples: Sequence[int]) -> np.ndarray:
    """``int64_array / np.sum(int64_array)`` -> float64 (scaffold.py:319-320)."""
    arr = np.array([int(n) for n in n_samples])
    return arr / np.sum(arr)


# --------------------------------------------------------------------------------------
# NumPy pairwise sum restated (used for numel == 1 tensors)
# --------------------------------------------------------------------------------------
def _pairwise(vals: np.ndarray, lo: int, n: int, dtype) -> np.generic:
    """NumPy ``@TYPE@_pairwise_sum`` on ``vals[lo:lo+n]`` in ``dtype`` arithmetic."""
    t = dtype.type
    if n < 8:
        res = t(-0.0)
        for i in range(n):
            res = t(res + vals[lo + i])
        return res
    if n <= PW_BLOCKSIZE:
        r = [t(vals[lo + j]) for j in range(8)]
        i = 8
        stop = n - (n % 8)
        while i < stop:
            for j in range(8):
                r[j] = t(r[j] + vals[lo + i + j])
            i += 8
        res = t(t(t(r[0] + r[1]) + t(r[2] + r[3])) + t(t(r[4] + r[5]) + t(r[6] + r[7])))
        while i < n:
            res = t(res + vals[lo + i])
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return t(_pairwise(vals, lo, n2, dtype) + _pairwise(vals, lo + n2, n - n2, dtype))


def numpy_pairwise_sum(vals: np.ndarray) -> np.generic:
    """``np.add.reduce`` over a contiguous 1-D axis of ``n`` elements: all ``n`` go through
    ``pairwise_sum`` (seeded with ``-0.0`` below 8 elements).  Checked against ``np.sum`` in
    ``tests/test_oracle.py`` (3000 random cases, K in 1..400, 0 mismatches)."""
    vals = np.ascontiguousarray(vals)
    dtype = vals.dtype
    return _pairwise(vals, 0, vals.size, dtype)


# --------------------------------------------------------------------------------------
# FedAvg
# --------------------------------------------------------------------------------------
def fedavg_reference_structure(parameters_updates: List[List[np.ndarray]], n_samples: Sequence[int]):
    """Same calls as fed_avg.py:217-222 (list of products, ``np.sum(axis=0)``)."""
    n_all_samples = sum(n_samples)
    averaged = []
    for idx in range(len(parameters_updates[0])):
        states = [pu[idx] * (n / n_all_samples) for pu, n in zip(parameters_updates, n_samples)]
        averaged.append(np.sum(states, axis=0))
    return averaged


def fedavg_explicit(parameters_updates: List[List[np.ndarray]], n_samples: Sequence[int]):
    """Explicit-order restatement for same-dtype fp32/fp64 layers.

    ``p_k = fl(x_k * fl(w_k))``; numel >= 2: ``acc = +0.0; acc = fl(acc + p_k)`` in list order
    (NumPy seeds the reduction with the +0.0 identity: an all ``-0.0`` column sums to ``+0.0``);
    numel == 1: ``+0.0 + pairwise(p_0..p_{K-1})``.
    """
    n_all = sum(int(n) for n in n_samples)
    out = []
    for idx in range(len(parameters_updates[0])):
        dtype = parameters_updates[0][idx].dtype
        w = np.array([int(n) / n_all for n in n_samples], dtype=np.float64).astype(dtype)
        prods = [np.multiply(pu[idx], w[k], dtype=dtype) for k, pu in enumerate(parameters_updates)]
        if prods[0].size == 1:
            vals = np.array([p.reshape(-1)[0] for p in prods], dtype=dtype)
            out.append(np.full(prods[0].shape, dtype.type(0.0) + numpy_pairwise_sum(vals), dtype=dtype))
        else:
            acc = np.zeros(prods[0].shape, dtype=dtype)
            for p in prods:
                np.add(acc, p, out=acc)
            out.append(acc)
    return out


# --------------------------------------------------------------------------------------
# Scaffold
# --------------------------------------------------------------------------------------
def scaffold_reference_structure(
    parameters_updates: List[List[np.ndarray]],
    control_variate_updates: List[List[np.ndarray]],
    server_control_variate: List[np.ndarray],
    n_samples: Sequence[int],
    aggregation_lr,
):
    """Same calls as scaffold.py:204-337 (returns ``(server_control_variate, avg_parameters_update)``)."""
    n_samples_per_client = np.array([n for n in n_samples])
    client_weight = n_samples_per_client / np.sum(n_samples_per_client)
    new_c = []
    for layer_idx in range(len(control_variate_updates[0])):
        weighted = [client_weight[k] * control_variate_updates[k][layer_idx] for k in range(len(n_samples))]
        weighted.append(server_control_variate[layer_idx])
        new_c.append(np.sum(weighted, axis=0))
    avg = []
    for layer_idx in range(len(parameters_updates[0])):
        weighted = [client_weight[k] * parameters_updates[k][layer_idx] for k in range(len(n_samples))]
        avg.append(aggregation_lr * np.sum(weighted, axis=0))
    return new_c, avg


def scaffold_explicit(
    parameters_updates: List[List[np.ndarray]],
    control_variate_updates: List[List[np.ndarray]],
    server_control_variate: List[np.ndarray],
    n_samples: Sequence[int],
    aggregation_lr,
):
    """Explicit-order restatement: everything in fp64, ``c`` added last,
    ``lr`` applied after the sum; numel == 1 tensors use the pairwise order over K (delta)
    or K + 1 (control variate, c is the last element)."""
    w = scaffold_weights_f64(n_samples)
    lr = np.float64(aggregation_lr)
    K = len(n_samples)

    def reduce(terms):
        if terms[0].size == 1:
            vals = np.array([t.reshape(-1)[0] for t in terms], dtype=np.float64)
            return np.full(terms[0].shape, np.float64(0.0) + numpy_pairwise_sum(vals), dtype=np.float64)
        acc = np.zeros(terms[0].shape, dtype=np.float64)
        for t in terms:
            np.add(acc, t, out=acc)
        return acc

    new_c = []
    for li in range(len(control_variate_updates[0])):
        terms = [np.multiply(w[k], control_variate_updates[k][li].astype(np.float64)) for k in range(K)]
        terms.append(server_control_variate[li].astype(np.float64))
        new_c.append(reduce(terms))
    avg = []
    for li in range(len(parameters_updates[0])):
        terms = [np.multiply(w[k], parameters_updates[k][li].astype(np.float64)) for k in range(K)]
        avg.append(np.multiply(lr, reduce(terms)))
    return new_c, avg


# --------------------------------------------------------------------------------------
# Newton-Raphson
# --------------------------------------------------------------------------------------
def newton_raphson_sums(gradients: List[List[np.ndarray]], hessians: List[np.ndarray], n_samples: Sequence[int]):
    """The weighted sums of newton_raphson.py:195-211, same calls: ``total = x_0 * c_0`` then
    ``total += x_k * c_k`` (``c_k = n_k / n``, a Python float), the gradients concatenated per
    client first.  Returns ``(total_hessians, total_gradient_one_d)``."""
    n_all = sum(n_samples)
    total_h = total_g = None
    for idx, (g, h, n) in enumerate(zip(gradients, hessians, n_samples)):
        c = n / n_all
        gc = np.concatenate([x.reshape(-1) for x in g])
        if idx == 0:
            total_h = h * c
            total_g = gc * c
        else:
            total_h += h * c
            total_g += gc * c
    return total_h, total_g


def newton_raphson_reference_structure(gradients: List[List[np.ndarray]], hessians: List[np.ndarray],
                                       n_samples: Sequence[int], damping_factor):
    """newton_raphson.py:195-216: the sums, ``-damping * solve(H, G)``, unflattened like the last
    client's gradients (``_unflatten_array``, :218-244)."""
    total_h, total_g = newton_raphson_sums(gradients, hessians, n_samples)
    upd = -damping_factor * np.linalg.solve(total_h, total_g)
    out, i = [], 0
    for a in gradients[-1]:
        n = len(a.ravel())
        out.append(np.array(upd[i: i + n].reshape(a.shape)))
        i += n
    return out
