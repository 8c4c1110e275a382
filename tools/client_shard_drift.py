#!/usr/bin/env python3
"""Numerical drift of the client-sharded (north-star) combines, computed by the product code
(substrafl_amd.sharding.client_shard_fedavg with GpuShardOps) with G ranks as threads on one GPU
(LoopbackGroup: the same per-rank kernels and the same exchange steps as over RCCL).

For each combine (relay / ordered / rccl-style sum) and G in {2, 4, 8}, the root's result is
compared with the single-pass kernel result -- bit-identical to the reference
(tests/test_gpu_parity.py) -- in ulp, on N(0,1) data (SURVEY.md §8(e) setup: K = 64, M = 1M,
n_k ~ U{100..10000}) and on cancellation-heavy data (alternating +-1e4 plus N(0,1)).  The
loopback's reduce sums the partials in rank order (RCCL's order over xGMI is its own choice:
same drift class).  Prints one JSON line per (data, combine, G)."""

import argparse
import json
import sys
import threading
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
    args = ap.parse_args()
    import torch

    from substrafl_amd.engine import FedAvgPlan, fedavg_weights
    from substrafl_amd.sharding import (FedAvgShard, GpuShardOps, LoopbackGroup, block_of, client_blocks,
                                        client_shard_fedavg)

    K, M = args.K, args.M
    dev = torch.device("cuda", 0)
    ns = [int(v) for v in np.random.default_rng(7).integers(100, 10000, K)]
    w = fedavg_weights(ns, "f32")  # global weights fl32(n_k / n)
    g = torch.Generator(device=dev)
    g.manual_seed(20241016)
    data = {"normal": torch.randn((K, M), generator=g, device=dev)}
    sign = torch.tensor([1.0 if k % 2 == 0 else -1.0 for k in range(K)], device=dev)[:, None]
    data["cancellation"] = sign * 1e4 + torch.randn((K, M), generator=g, device=dev)
    pw = np.zeros(0, np.uint64)
    for name, x in data.items():
        ref = torch.empty(M, device=dev)
        FedAvgPlan("f32", x, w, M, ref).launch()
        ref_h = ref.cpu().numpy()
        for combine in ("relay", "ordered", "rccl"):
            for G in (2, 4, 8):
                grp = LoopbackGroup(G)
                res = [None] * G
                err = [None] * G

                def body(r):
                    try:
                        s = torch.cuda.Stream(device=dev)
                        with torch.cuda.stream(s):
                            k0, k1 = client_blocks(K, G)[block_of(r, G)]
                            out = torch.empty(M, device=dev)
                            sh = FedAvgShard("f32", x[k0:k1], w[k0:k1], k0, K, M, pw)
                            if client_shard_fedavg(sh, out, grp.transport(r), GpuShardOps(), combine):
                                s.synchronize()
                                res[r] = out.cpu().numpy()
                        s.synchronize()
                    except BaseException as e:  # noqa: BLE001
                        err[r] = e

                th = [threading.Thread(target=body, args=(r,)) for r in range(G)]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
                for e in err:
                    if e is not None:
                        raise e
                d = ulp_distance(res[0], ref_h)
                print(json.dumps({
                    "data": name, "combine": combine, "K": K, "M": M, "G": G,
                    "median_ulp": float(np.median(d)), "p99_ulp": float(np.percentile(d, 99)), "max_ulp": int(d.max()),
                    "frac_gt_2ulp": round(float(np.mean(d > 2)), 4), "frac_exact": round(float(np.mean(d == 0)), 4),
                }), flush=True)


if __name__ == "__main__":
    main()
