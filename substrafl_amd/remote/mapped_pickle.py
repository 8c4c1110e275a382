"""Zero-copy loading of shared-state pickles for the aggregate task.

An aggregate task unpickles K shared-state files (substratools_methods.py:54-66) and then only
reads the arrays in them.  ``pickle.load`` copies every array payload into freshly allocated
memory, and in a fresh process that memory is first-touched page by page: ≈8 ms per 100 MB of
page faults on the GPU box (profiles/r01_d2h_probe.log), most of the task's load time.

:func:`load_mapped` maps the file instead (``MAP_PRIVATE``: the page cache's pages,
copy-on-write) and builds each NumPy array as a view of its payload inside the mapping:
no copy, no zeroed pages.  Everything else in the pickle is unpickled as usual, by the standard
library's own unpickler (``pickle._Unpickler``) with two hooks:

* the file object hands out payloads of >= 1 MiB as ``memoryview`` slices of the mapping;
* ``BUILD`` of a plain ``ndarray`` whose raw data is such a slice (NumPy's protocol 3-4
  reduction ``_reconstruct`` + ``__setstate__``) becomes ``np.frombuffer(slice).reshape(...)``,
  replacing the placeholder on the stack and in the memo;
* protocol 5 in-band buffers (``BYTEARRAY8``: NumPy's ``PickleBuffer`` reduction, the flat wire
  bucket) of >= 1 MiB are handed to their reduction as writable views of the mapping.

The arrays are writable (copy-on-write), C- or F-ordered as pickled, and equal to what
``pickle.load`` returns.  If any large payload is consumed by something else (a ``bytes`` field,
an object array, an unknown reduction), the file is loaded again with ``pickle.load``, so the
result never differs in type from the reference's.  Task inputs are read-only by contract;
deleting a mapped file is harmless (the mapping keeps it), truncating it while the task runs
is not supported.
"""

from __future__ import annotations

import mmap
import pickle
import struct
from pathlib import Path
from typing import Any, List

import numpy as np

BIG = 1 << 20  # payloads handed out as views of the mapping
# callables a pickle may hand such a payload to, that build an array viewing it (protocol 5 arrays,
# the flat wire format)
_VIEW_CONSUMERS = {("numpy._core.numeric", "_frombuffer"), ("numpy.core.numeric", "_frombuffer"),
                   ("substrafl_amd.wire", "_bucket_from_buffer")}


class _MappedFile:
    """Read-only file object over a mapping for ``pickle._Unpickler``."""

    def __init__(self, mm: mmap.mmap):
        self.mm = mm
        self.view = memoryview(mm)
        self.pos = 0
        self.size = len(mm)
        self.views: List[memoryview] = []

    def read(self, n: int = -1):
        a = self.pos
        b = self.size if n is None or n < 0 else min(self.size, a + n)
        self.pos = b
        if b - a >= BIG:
            v = self.view[a:b]
            self.views.append(v)
            return v
        return self.mm[a:b]

    def readinto(self, buf) -> int:
        n = min(len(buf), self.size - self.pos)
        memoryview(buf).cast("B")[:n] = self.view[self.pos : self.pos + n]
        self.pos += n
        return n

    def readline(self) -> bytes:
        i = self.mm.find(b"\n", self.pos)
        b = self.size if i < 0 else i + 1
        out = self.mm[self.pos : b]
        self.pos = b
        return out


class _MappedUnpickler(pickle._Unpickler):  # the pure-Python unpickler: its dispatch table is overridable
    dispatch = dict(pickle._Unpickler.dispatch)

    def __init__(self, f: _MappedFile):
        super().__init__(f)
        self._mapped = f
        self.consumed = 0

    def find_class(self, module, name):
        obj = super().find_class(module, name)
        if (module, name) in _VIEW_CONSUMERS:  # reductions that take a buffer and keep a view of it

            def consume(buf, *args, _f=obj):
                if isinstance(buf, memoryview):
                    self.consumed += 1  # a writable view of the mapping: np.frombuffer keeps it
                return _f(buf, *args)

            return consume
        return obj

    def load_bytearray8(self):
        # protocol 5 in-band buffers (NumPy's PickleBuffer reduction, the wire bucket): a view of
        # the mapping instead of a fresh bytearray, for payloads written outside a frame
        n, = struct.unpack("<Q", self.read(8))
        f = self._mapped
        if n >= BIG and not self._unframer.current_frame and f.pos + n <= f.size:
            v = f.view[f.pos : f.pos + n]
            f.pos += n
            f.views.append(v)
            self.append(v)
            return
        b = bytearray(n)
        self.readinto(b)
        self.append(b)

    dispatch[pickle.BYTEARRAY8[0]] = load_bytearray8

    def load_build(self):
        stack = self.stack
        state = stack[-1]
        inst = stack[-2]
        if (type(inst) is np.ndarray and isinstance(state, tuple) and len(state) == 5
                and isinstance(state[4], memoryview)):
            _, shape, dtype, fortran, raw = state
            dtype = np.dtype(dtype)
            if not dtype.hasobject:
                n = int(np.prod(shape, dtype=np.int64)) if len(shape) else 1
                arr = np.frombuffer(raw, dtype=dtype, count=n).reshape(shape, order="F" if fortran else "C")
                stack.pop()
                stack[-1] = arr
                for k, v in list(self.memo.items()):
                    if v is inst:
                        self.memo[k] = arr
                self.consumed += 1
                return
        pickle._Unpickler.load_build(self)

    dispatch[pickle.BUILD[0]] = load_build


POPULATE = False  # MAP_POPULATE on a private WRITABLE mapping breaks copy-on-write of every page


def load_mapped(path) -> Any:
    """``pickle.load`` of ``path`` with NumPy array payloads left in a private mapping of the
    file (see the module docstring); falls back to ``pickle.load`` for anything else."""
    path = Path(path)
    with path.open("rb") as fh:
        try:
            flags = mmap.MAP_PRIVATE | (getattr(mmap, "MAP_POPULATE", 0) if POPULATE else 0)
            mm = mmap.mmap(fh.fileno(), 0, flags=flags, prot=mmap.PROT_READ | mmap.PROT_WRITE)
        except (ValueError, OSError):  # empty file, special file, ...: the plain path decides
            fh.seek(0)
            return pickle.load(fh)
    f = _MappedFile(mm)
    try:
        up = _MappedUnpickler(f)
        obj = up.load()
    except Exception:  # noqa: BLE001 - the reference's loader raises the reference's error
        obj, up = None, None
    if up is None or up.consumed != len(f.views):
        with path.open("rb") as fh:  # a payload went somewhere else: keep pickle.load's exact objects
            return pickle.load(fh)
    return obj
