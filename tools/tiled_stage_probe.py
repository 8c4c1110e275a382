"""Host path with the row vs the tile-interleaved staging (AggregationEngine.tiled) at a recommended shape
(32 fp32 clients x 34M): stage / kernel+fetch time per call and bit-identity of the two."""
import sys, time, json
sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
import numpy as np
from substrafl_amd.engine import AggregationEngine
from substrafl_amd.layout import synthetic_state_dict_shapes
K, M = 32, 34_000_000
shapes = synthetic_state_dict_shapes(M)
rng = np.random.default_rng(1)
base = [rng.standard_normal(int(np.prod(s)), dtype=np.float32).reshape(s) for s in shapes]
pus = [[(a * np.float32(1 + 0.01 * k)).astype(np.float32) for a in base] for k in range(K)]
ns = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
eng = AggregationEngine(device=0)
res = {}
for mode in [False, True, False, True]:
    eng.tiled = mode
    outs = None
    for rep in range(3):
        t0 = time.perf_counter(); o = eng.fedavg(pus, ns); t = time.perf_counter() - t0
    tm = eng.last_timing
    res.setdefault(str(mode), []).append({"total_s": round(t, 4), "stage_s": round(tm["stage_s"], 4),
                                          "kernel_fetch_s": round(tm["kernel_fetch_s"], 4), "layout": tm["layout"]})
    if outs is None:
        outs = np.concatenate([x.ravel() for x in o]).copy()
eng.tiled = False; a = np.concatenate([x.ravel() for x in eng.fedavg(pus, ns)]).copy()
eng.tiled = True; b = np.concatenate([x.ravel() for x in eng.fedavg(pus, ns)]).copy()
res["bit_identical"] = bool(np.array_equal(a.view(np.uint32), b.view(np.uint32)))
print(json.dumps(res))
