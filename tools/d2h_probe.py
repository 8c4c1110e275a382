#!/usr/bin/env python3
"""D2H paths for one 100 MB device bucket on the GPU box: the native session's pinned-ring fetch
(into a fresh or a reused host array), torch's single pageable .cpu(), and torch's per-layer .cpu()
loop (the reference's Δ export).  Wall time per call, median of 7."""

import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch

    from substrafl_amd import runtime
    from substrafl_amd.layout import synthetic_state_dict_shapes

    n = 25_000_000
    flat = torch.randn(n, device="cuda")
    shapes = synthetic_state_dict_shapes(n)
    views, off = [], 0
    for s in shapes:
        k = int(np.prod(s))
        views.append(flat[off:off + k].view(s))
        off += k
    sess = runtime.session(0)
    reuse = np.empty(n, np.float32)

    def t(fn, reps=7):
        fn()
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return round(float(np.median(ts)) * 1e3, 3)

    res = {
        "session_fetch_fresh_ms": t(lambda: sess.fetch(flat.data_ptr(), np.empty(n, np.float32))),
        "session_fetch_reused_ms": t(lambda: sess.fetch(flat.data_ptr(), reuse)),
        "np_empty_and_touch_ms": t(lambda: np.empty(n, np.float32).fill(0)),
        "torch_cpu_flat_ms": t(lambda: flat.cpu()),
        "torch_cpu_per_layer_ms": t(lambda: [v.cpu() for v in views]),
        "session_threads": int(sess.lib.fedagg_session_set(sess._h, b"threads", 16) == 0) and 16,
    }
    for th in (4, 8, 32):
        sess.set("threads", th)
        res[f"session_fetch_fresh_threads{th}_ms"] = t(lambda: sess.fetch(flat.data_ptr(), np.empty(n, np.float32)))
    sess.set("threads", 16)
    for cb in (1 << 20, 16 << 20):
        sess.set("chunk_bytes", cb)
        res[f"session_fetch_fresh_chunk{cb >> 20}M_ms"] = t(lambda: sess.fetch(flat.data_ptr(), np.empty(n, np.float32)))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
