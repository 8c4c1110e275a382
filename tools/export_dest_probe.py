"""Where should an export's D2H land?  100 MB / 400 MB fp32 from HBM into (a) a recycled pageable
NumPy buffer through the native session's pinned ring (``fedagg_session_fetch``: what
``export_numpy`` does), (b) a pinned host tensor (torch ``pin_memory``, one direct DMA), (c) (b)
followed by nothing else -- the ceiling.  Best / median of --reps, one JSON line per size.

    python3 tools/export_dest_probe.py --mb 100,400 --reps 10
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", default="100,400")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()

    import torch

    from substrafl_amd import runtime

    for mb in [int(v) for v in args.mb.split(",")]:
        n = mb * 1_000_000 // 4
        d = torch.randn(n, device="cuda")
        torch.cuda.synchronize()
        s = runtime.session(0)
        host = np.empty(n, np.float32)
        host[:] = 0  # touched: the recycled buffer of a later round
        ring = []
        for _ in range(args.reps):
            t = time.perf_counter()
            s.fetch(d.data_ptr(), host)
            ring.append(time.perf_counter() - t)
        pinned = torch.empty(n, dtype=torch.float32, pin_memory=True)
        direct = []
        for _ in range(args.reps):
            t = time.perf_counter()
            pinned.copy_(d)
            torch.cuda.synchronize()
            direct.append(time.perf_counter() - t)
        ok = np.array_equal(host.view(np.uint32), pinned.numpy().view(np.uint32))
        gb = mb / 1e3
        print(json.dumps({"mb": mb, "ring_fetch_ms": [round(1e3 * min(ring), 3), round(1e3 * float(np.median(ring)), 3)],
                          "ring_fetch_GBps": round(gb / float(np.median(ring)), 1),
                          "pinned_direct_ms": [round(1e3 * min(direct), 3), round(1e3 * float(np.median(direct)), 3)],
                          "pinned_direct_GBps": round(gb / float(np.median(direct)), 1), "same_bytes": ok}), flush=True)
        del d, pinned


if __name__ == "__main__":
    main()
