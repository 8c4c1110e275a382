"""Flat-bucket wire format for shared states.

The reference ships a client's update as ``List[np.ndarray]`` -- one pickled array per layer
(``torch_fed_avg_algo.py:227-230``, ``remote/serializers/pickle_serializer.py:10-18``).  Here the
layers of one update are :class:`BucketArray` views of ONE contiguous host buffer (the flat
bucket that ``weight_manager.export_numpy`` brings home with a single D2H copy, or that the
aggregation engine fetches), and they pickle as that buffer plus ``(offset, shape, dtype)``
records, so that

* the loaded update is again L views of one buffer: the aggregator stages a client with one
  host→device segment and the client applies an averaged update with one H2D copy;
* a pickle stays a pickle: plain ``pickle.load`` (the reference's ``PickleSerializer``) reads it,
  any protocol; protocol 5 writes the buffer as an in-band ``bytearray`` or, with a
  ``buffer_callback``, out of band;
* every element stays an ``np.ndarray`` of the layer's shape and dtype (the schemas check
  ``isinstance(np.ndarray)``, ``strategies/schemas.py:29``), and arithmetic on one returns a
  plain ``np.ndarray``.

Nothing here is specific to the GPU; :func:`flat_of` is how the engine and the client ops
recognise a flat row.
"""

from __future__ import annotations

import pickle
from typing import List, Optional, Sequence, Tuple

import numpy as np

_SMALL = 4096  # below this a payload is copied on load (never alias a possibly shared bytes object)


class _Bucket:
    """Owner of one flat byte buffer (1-D uint8, C-contiguous, writable)."""

    __slots__ = ("flat", "__weakref__")

    def __init__(self, flat: np.ndarray):
        if flat.dtype != np.uint8 or flat.ndim != 1 or not flat.flags.c_contiguous:
            raise ValueError("a bucket is a 1-D contiguous uint8 buffer")
        self.flat = flat

    def __reduce_ex__(self, protocol):
        if protocol >= 5 and self.flat.flags.writeable:
            return _bucket_from_buffer, (pickle.PickleBuffer(self.flat),)
        return _bucket_from_buffer, (self.flat.tobytes(),)


def _bucket_from_buffer(buf) -> _Bucket:
    """Unpickle: a writable uint8 array over ``buf`` without a copy where that is safe."""
    if isinstance(buf, bytes):
        if len(buf) < _SMALL:
            return _Bucket(np.frombuffer(bytearray(buf), dtype=np.uint8))
        # NumPy's own protocol-4 path: a writable array owning the unpickled bytes object.
        a = np.ndarray.__new__(np.ndarray, (0,), np.uint8)
        a.__setstate__((1, (len(buf),), np.dtype(np.uint8), False, buf))
        return _Bucket(a)
    a = np.frombuffer(buf, dtype=np.uint8)
    if not a.flags.writeable:
        a = a.copy()
    return _Bucket(a)


class BucketArray(np.ndarray):
    """One layer of a flat bucket: a plain ``np.ndarray`` view that pickles by reference to the
    bucket.  Slices and arithmetic results are ordinary arrays (``__array_finalize__`` and
    ``__array_ufunc__`` drop the bucket link)."""

    _bucket: Optional[_Bucket] = None
    _offset: int = 0

    def __array_finalize__(self, obj):
        self._bucket = None
        self._offset = 0

    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        inputs = tuple(x.view(np.ndarray) if isinstance(x, BucketArray) else x for x in inputs)
        out = kwargs.get("out")
        if out:
            kwargs["out"] = tuple(x.view(np.ndarray) if isinstance(x, BucketArray) else x for x in out)
        return getattr(ufunc, method)(*inputs, **kwargs)

    def __reduce_ex__(self, protocol):
        if self._bucket is None:
            return self.view(np.ndarray).__reduce_ex__(protocol)
        return _layer, (self._bucket, self._offset, self.shape, self.dtype.str)

    def __reduce__(self):
        return self.__reduce_ex__(2)


def _layer(bucket: _Bucket, offset: int, shape: Tuple[int, ...], dtype: str) -> BucketArray:
    dt = np.dtype(dtype)
    n = int(np.prod(shape, dtype=np.int64)) if len(shape) else 1
    return _member(bucket, offset, dt, n, tuple(shape))


def _member(bucket: _Bucket, offset: int, dt: np.dtype, n: int, shape) -> BucketArray:
    raw = bucket.flat[offset : offset + n * dt.itemsize]
    v = raw.view(dt).reshape(shape).view(BucketArray)
    v._bucket = bucket
    v._offset = offset
    return v


def bucket_views(flat: np.ndarray, shapes: Sequence[Tuple[int, ...]], dtypes=None) -> List[BucketArray]:
    """Per-layer :class:`BucketArray` views of ``flat`` (layers back to back, in order)."""
    flat = np.ascontiguousarray(flat).reshape(-1)
    base_dt = flat.dtype
    bucket = _Bucket(flat.view(np.uint8))
    out, off = [], 0
    for i, shp in enumerate(shapes):
        dt = np.dtype(dtypes[i]) if dtypes is not None else base_dt
        n = int(np.prod(shp, dtype=np.int64)) if len(shp) else 1
        if off % dt.itemsize:
            raise ValueError("layer offsets must be aligned to the layer's item size")
        out.append(_member(bucket, off, dt, n, tuple(shp)))
        off += n * dt.itemsize
    if off > bucket.flat.nbytes:
        raise ValueError("the layers do not fit in the buffer")
    return out


def pack(arrays: Sequence[np.ndarray]) -> List[BucketArray]:
    """Copy ``arrays`` (any dtypes) into one new flat bucket, each layer aligned to its item size
    (layers of one dtype are therefore back to back, like an engine bucket row)."""
    shapes = [np.shape(a) for a in arrays]
    dtypes = [np.asarray(a).dtype for a in arrays]
    offs, off = [], 0
    for a, dt in zip(arrays, dtypes):
        off = -(-off // dt.itemsize) * dt.itemsize
        offs.append(off)
        off += np.asarray(a).nbytes
    flat = np.empty(off, dtype=np.uint8)  # NumPy allocations are at least 16-B aligned
    bucket = _Bucket(flat)
    out = []
    for a, shp, dt, o in zip(arrays, shapes, dtypes, offs):
        n = int(np.prod(shp, dtype=np.int64)) if len(shp) else 1
        v = _member(bucket, o, dt, n, tuple(shp))
        np.copyto(v.view(np.ndarray), np.asarray(a), casting="no")
        out.append(v)
    return out


def flat_of(arrays: Sequence[np.ndarray]) -> Optional[np.ndarray]:
    """If ``arrays`` are consecutive layers of one bucket, all of one dtype, with no gaps, the 1-D
    array of that dtype spanning exactly them; else None."""
    if not arrays or not all(isinstance(a, BucketArray) and a._bucket is not None for a in arrays):
        return None
    b = arrays[0]._bucket
    dt = arrays[0].dtype
    off = arrays[0]._offset
    start = off
    for a in arrays:
        if a._bucket is not b or a.dtype != dt or a._offset != off:
            return None
        off += a.nbytes
    if start % dt.itemsize:
        return None
    return b.flat[start:off].view(dt)
