"""Per-client staging as ingest does it (one client per call) into the row layout vs the
tile-interleaved layout (Session.stage vs Session.stage_tiled_row: one 2-D H2D copy per pinned
chunk), 32 fp32 clients x 34M: seconds per client and GB/s, plus a FedAvg on each staged bucket."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

from substrafl_amd.engine import tiled_elems, tiled_tile  # noqa: E402
from substrafl_amd.runtime import Session  # noqa: E402

K, M = 32, 34_000_000
rng = np.random.default_rng(1)
base = rng.standard_normal(M, dtype=np.float32)
rows = [[base * np.float32(1 + 0.01 * k)] for k in range(K)]
tv = tiled_tile("f32", K, M)
ld = (M + 127) // 128 * 128
s = Session(0)
if len(sys.argv) > 1:  # pinned-chunk size in MiB (session knob chunk_bytes)
    s.set("chunk_bytes", int(sys.argv[1]) << 20)
d_rows = s.buffer(0, K * ld * 4)
d_t = s.buffer(1, tiled_elems("f32", K, M, tv) * 4)
res = {"K": K, "M": M, "tv": tv, "chunk_MiB": int(sys.argv[1]) if len(sys.argv) > 1 else "default"}
for rep in range(3):
    for name in ("rows", "tiles"):
        s.sync()
        t0 = time.perf_counter()
        for k in range(K):
            if name == "rows":
                s.stage(d_rows + k * ld * 4, ld * 4, [rows[k]])
            else:
                s.stage_tiled_row(d_t, tv * 16, K, k, rows[k])
        s.sync()
        t = time.perf_counter() - t0
        res.setdefault(name, []).append({"s_per_client": round(t / K, 5), "GB_s": round(K * M * 4 / t / 1e9, 2)})
print(json.dumps(res))
s.close()
