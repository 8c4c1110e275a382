"""Flat-bucket layout of a client's list of update tensors.

The reference ships each client's update as ``List[np.ndarray]`` in the layer order defined by
``weight_manager.model_parameters`` (substrafl/algorithms/pytorch/weight_manager.py:53-76:
``model.parameters()`` then BatchNorm ``running_mean``/``running_var``) and reduces it layer by
layer (fed_avg.py:219-222).  The engine instead lays every layer of one dtype back to back in
one contiguous row per client ("bucket"), so one kernel launch streams the whole model:

    row k = [ layer_0 | layer_1 | ... | layer_{L-1} | pad to a 256-B multiple ]

Rows are ``ld`` elements apart in one ``[K, ld]`` HBM allocation, so every client stream starts
256-B aligned (16-B vector loads, no split cache lines).  ``numel == 1`` layers (and 0-d
layers) are listed in ``pairwise_idx``: NumPy reduces those along the contiguous axis with its
pairwise tree and the engine patches them with the pairwise kernel.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

from .wire import bucket_views

ROW_ALIGN_BYTES = 256


@dataclass(frozen=True)
class Segment:
    layer: int  # index in the client's parameters_update list
    shape: Tuple[int, ...]
    offset: int  # element offset inside the bucket row
    numel: int


class BucketLayout:
    """Layout of the layers ``layer_ids`` (all of storage dtype ``dtype``) inside one bucket row."""

    def __init__(self, layer_ids: Sequence[int], shapes: Sequence[Tuple[int, ...]], dtype):
        self.dtype = np.dtype(dtype)
        segs = []
        off = 0
        for li, shp in zip(layer_ids, shapes):
            n = int(np.prod(shp, dtype=np.int64)) if len(shp) else 1
            segs.append(Segment(int(li), tuple(int(s) for s in shp), off, n))
            off += n
        self.segments: List[Segment] = segs
        self.M = off
        per_row = max(1, ROW_ALIGN_BYTES // self.dtype.itemsize)
        self.ld = ((off + per_row - 1) // per_row) * per_row if off else per_row
        self.pairwise_idx = np.array([s.offset for s in segs if s.numel == 1], dtype=np.uint64)

    @property
    def n_layers(self) -> int:
        return len(self.segments)

    def pack_row(self, layers: Sequence[np.ndarray], dst: np.ndarray) -> None:
        """Copy one client's layers into ``dst`` (a 1-D view of length >= M, this bucket's dtype)."""
        for s in self.segments:
            src = np.asarray(layers[s.layer])
            np.copyto(dst[s.offset : s.offset + s.numel], src.reshape(-1), casting="unsafe")

    def unpack(self, flat: np.ndarray, wire: bool = False) -> List[Tuple[int, np.ndarray]]:
        """Views of ``flat`` shaped like each layer; with ``wire`` they are :class:`wire.BucketArray`
        layers of one bucket, so the result pickles as one flat buffer.  0-d layers come back as
        NumPy scalars, which is what ``np.sum`` of 0-d arrays returns in the reference."""
        if wire:
            views = bucket_views(flat[: self.M], [s.shape for s in self.segments])
        else:
            views = [flat[s.offset : s.offset + s.numel].reshape(s.shape) for s in self.segments]
        out = []
        for s, v in zip(self.segments, views):
            out.append((s.layer, flat[s.offset] if len(s.shape) == 0 else v))
        return out

    def __repr__(self) -> str:  # pragma: no cover
        return f"BucketLayout(dtype={self.dtype}, layers={self.n_layers}, M={self.M}, ld={self.ld})"


def synthetic_state_dict_shapes(M: int) -> List[Tuple[int, ...]]:
    """Layer shapes of the synthetic state_dict used by bench.py: one embedding
    ``(M // 8 // 1024, 1024)``, then repeated ``[(1024, 1024), (1024,)]`` blocks, a 1-D remainder
    and one ``(1,)`` tensor (exercises the numel == 1 pairwise order)."""
    shapes: List[Tuple[int, ...]] = []
    rem = M - 1
    emb_rows = M // 8 // 1024
    if emb_rows > 0:
        shapes.append((emb_rows, 1024))
        rem -= emb_rows * 1024
    block = 1024 * 1024 + 1024
    while rem >= block:
        shapes.append((1024, 1024))
        shapes.append((1024,))
        rem -= block
    if rem > 0:
        shapes.append((rem,))
    shapes.append((1,))
    return shapes
