#!/usr/bin/env python3
"""Numerical drift and on-GPU cost of the north-star client-sharded mode.

Client sharding splits the K clients into G contiguous blocks, sums each block on its own GPU
with the global weights fl32(n_k / n), and combines the G partial sums on the root (RCCL reduce,
or a gather + rank-order sum).  That re-associates the reference's sequential client sum
(fed_avg.py:222), so the result drifts from the reference.  This tool measures the drift in ulp
against the single-pass kernel result -- bit-identical to the reference (tests/test_gpu_parity.py)
-- on N(0,1) data (SURVEY.md §8(e) setup: K = 64, M = 1M, n_k ~ U{100..10000}) and on
cancellation-heavy data (G2-style: alternating +-1e4 plus N(0,1)), for G in {2, 4, 8}, and times
the per-block partial kernels and the rank-order combine on one GPU.  The xGMI reduce itself
needs several GPUs and is not timed here.

Prints one JSON line per (data, G)."""

import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def ulp_distance(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """|a - b| in units in the last place (fp32, through the ordered integer representation)."""
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, np.int64(-(2**31)) - ia, ia)
    ib = np.where(ib < 0, np.int64(-(2**31)) - ib, ib)
    return np.abs(ia - ib)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--M", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    from substrafl_amd.engine import FedAvgPlan, fedavg_weights

    K, M = args.K, args.M
    dev = torch.device("cuda", 0)
    ns = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    w = fedavg_weights(ns, "f32")  # global weights fl32(n_k / n)
    g = torch.Generator(device=dev)
    g.manual_seed(20241016)
    data = {"normal": torch.randn((K, M), generator=g, device=dev)}
    sign = torch.tensor([1.0 if k % 2 == 0 else -1.0 for k in range(K)], device=dev)[:, None]
    data["cancellation"] = sign * 1e4 + torch.randn((K, M), generator=g, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, x in data.items():
        ref = torch.empty(M, device=dev)
        FedAvgPlan("f32", x, w, M, ref).launch()
        ref_h = ref.cpu().numpy()
        for G in (2, 4, 8):
            per = -(-K // G)
            blocks = [list(range(r * per, min(K, (r + 1) * per))) for r in range(G)]
            parts = torch.empty((G, M), device=dev)
            plans = [FedAvgPlan("f32", [x[k].data_ptr() for k in b], w[b], M, parts[r]) for r, b in enumerate(blocks)]

            def run():
                for p in plans:
                    p.launch()
                tot = parts[0].clone()
                for r in range(1, G):
                    tot.add_(parts[r])  # rank-order combine on the root, fp32
                return tot

            tot = run()
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(args.iters):
                run()
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / args.iters
            d = ulp_distance(tot.cpu().numpy(), ref_h)
            print(json.dumps({
                "data": name, "K": K, "M": M, "G": G,
                "median_ulp": float(np.median(d)), "p99_ulp": float(np.percentile(d, 99)), "max_ulp": int(d.max()),
                "frac_gt_2ulp": round(float(np.mean(d > 2)), 4), "frac_exact": round(float(np.mean(d == 0)), 4),
                "one_gpu_partials_plus_combine_ms": round(ms, 4),
                "single_pass_equivalent_GBps": round((K * M * 4 + M * 4) / (ms / 1e3) / 1e9, 1),
            }), flush=True)


if __name__ == "__main__":
    main()
