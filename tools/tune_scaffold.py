#!/usr/bin/env python3
"""Launch-shape sweep of the Scaffold two-bucket kernel (interleaved rounds, one process)."""

import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=16)
    ap.add_argument("--M", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only-new", action="store_true", help="only the c-prefetch / occupancy / 512-thread variants")
    ap.add_argument("--two-launch", action="store_true", help="one launch per bucket (sc_2l) shapes")
    ap.add_argument("--kind", default="f32", choices=["f32", "f64"], help="client bucket dtype")
    ap.add_argument("--sc1", action="store_true", help="write-through (sc1) output stores on the 4 x 4 tiles")
    args = ap.parse_args()
    import torch

    from substrafl_amd import _native
    from substrafl_amd.engine import ScaffoldPlan, scaffold_weights
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes

    shapes = synthetic_state_dict_shapes(args.M)
    ndt, tdt = (np.float32, torch.float32) if args.kind == "f32" else (np.float64, torch.float64)
    lay = BucketLayout(range(len(shapes)), shapes, ndt)
    d = torch.randn((args.K, lay.ld), device="cuda", dtype=tdt)
    cv = torch.randn((args.K, lay.ld), device="cuda", dtype=tdt)
    c = torch.randn(lay.ld, device="cuda", dtype=tdt)
    dout = torch.empty(lay.ld, dtype=torch.float64, device="cuda")
    cout = torch.empty(lay.ld, dtype=torch.float64, device="cuda")
    ns = [int(v) for v in np.random.default_rng(7).integers(100, 10000, args.K)]
    plan = ScaffoldPlan(args.kind, d, cv, c, scaffold_weights(ns), args.M, 1.0, dout, cout, lay.pairwise_idx)
    nbytes = plan.bytes_alg()
    variants = [dict(sc_split=0, sc_pipe=0, sc_vpt=v, sc_unroll=u, nt_store=1, grid_cap=0, xcd=0)
                for v, u in ((0, 4), (2, 4), (2, 8), (1, 8), (4, 2), (4, 4), (8, 1), (8, 2))]  # sc_vpt 0: auto
    variants += [dict(sc_split=0, sc_pipe=1, sc_vpt=v, sc_unroll=u, nt_store=1, grid_cap=0, xcd=0)
                 for v, u in ((4, 2), (2, 4))]
    variants += [dict(sc_split=1, sc_pipe=0, sc_vpt=v, sc_unroll=u, nt_store=1, grid_cap=0, xcd=0)
                 for v, u in ((4, 4), (8, 2))]
    variants += [dict(sc_split=0, sc_pipe=0, sc_vpt=0, sc_unroll=4, nt_store=1, grid_cap=0, xcd=0, tpb=t)
                 for t in (2, 4, 8)]
    variants += [dict(sc_split=0, sc_pipe=0, sc_bsplit=1, sc_vpt=v, sc_unroll=u, nt_store=1, grid_cap=0, xcd=0)
                 for v, u in ((8, 4), (8, 2), (4, 4), (4, 8), (2, 8))]
    variants += [dict(sc_split=0, sc_pipe=0, sc_buf=1, sc_vpt=v, sc_unroll=u, nt_store=1, grid_cap=0, xcd=0)
                 for v, u in ((4, 4), (4, 2), (8, 2), (8, 4))]
    variants += [dict(sc_split=0, sc_pipe=0, sc_vpt=4, sc_unroll=4, nt_store=1, grid_cap=0, xcd=0, sc_cpf=cpf,
                      sc_occ=occ, sc_blk=blk)
                 for cpf in (0, 1) for occ in (0, 4) for blk in (256, 512) if (cpf, occ, blk) != (0, 0, 256)
                 if not (occ == 4 and blk == 512)]
    variants += [dict(sc_split=0, sc_pipe=0, sc_vpt=v, sc_unroll=u, nt_store=0, grid_cap=0, xcd=0)
                 for v, u in ((4, 4), (4, 2), (8, 1))]
    if args.sc1:
        variants = [dict(sc_split=0, sc_pipe=0, sc_vpt=0, sc_unroll=4, nt_store=1, grid_cap=0, xcd=0),
                    dict(sc_split=0, sc_pipe=0, sc_vpt=4, sc_unroll=4, nt_store=1, grid_cap=0, xcd=0, sc_sc1=1),
                    dict(sc_split=0, sc_pipe=0, sc_buf=1, sc_vpt=4, sc_unroll=4, nt_store=1, grid_cap=0, xcd=0),
                    dict(sc_split=0, sc_pipe=0, sc_buf=1, sc_vpt=4, sc_unroll=4, nt_store=1, grid_cap=0, xcd=0,
                         sc_sc1=1)]
    elif args.two_launch:
        variants = [dict(sc_split=0, sc_pipe=0, sc_vpt=0, sc_unroll=4, nt_store=1, grid_cap=0, xcd=0),
                    dict(sc_split=0, sc_pipe=0, sc_vpt=0, sc_unroll=4, nt_store=1, grid_cap=0, xcd=0, sc_2l=-1)]
        variants += [dict(sc_split=0, sc_pipe=0, sc_2l=1, sc_vpt=v, sc_unroll=u, nt_store=1, grid_cap=0, xcd=0,
                          sc_sc1=s1) for v, u in ((4, 4), (8, 4), (8, 2), (16, 2), (4, 8), (16, 1))
                     for s1 in (0, 1)]
        variants += [dict(sc_split=0, sc_pipe=0, sc_2l=2, sc_vpt=v, sc_unroll=u, nt_store=1, grid_cap=0, xcd=0)
                     for v, u in ((8, 4), (4, 8))]
        variants += [dict(sc_split=0, sc_pipe=1, sc_2l=1, sc_vpt=v, sc_unroll=u, nt_store=1, grid_cap=0, xcd=0)
                     for v, u in ((8, 2), (4, 4), (4, 2))]
    elif args.only_new:
        variants = [v for v in variants if "sc_cpf" in v or v.get("nt_store") == 0] + [dict(sc_split=0, sc_pipe=0, sc_vpt=0, sc_unroll=4,
                                                                  nt_store=1, grid_cap=0, xcd=0)]
    variants = [dict(dict(tpb=1, sc_bsplit=0, sc_buf=0, sc_cpf=0, sc_occ=0, sc_blk=256, sc_sc1=0, sc_2l=0), **v) for v in variants]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = {i: [] for i in range(len(variants))}
    for _ in range(args.rounds):
        for i, kn in enumerate(variants):
            _native.tune(**kn)
            plan.launch()
            ev[0].record()
            for _ in range(args.iters):
                plan.launch()
            ev[1].record()
            torch.cuda.synchronize()
            times[i].append(ev[0].elapsed_time(ev[1]) / args.iters)
    # the c-equality check of the same call (scaffold.py:193-196): K copies of c, scalar vs 16-B
    from substrafl_amd.engine import equal_count

    cc = c.repeat(args.K, 1)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for vec in (0, 1):
        _native.tune(eq_vec=vec)
        tt = []
        for _ in range(args.rounds):
            equal_count("f32", cc, lay.M, cnt)
            ev[0].record()
            for _ in range(args.iters):
                equal_count("f32", cc, lay.M, cnt)
            ev[1].record()
            torch.cuda.synchronize()
            tt.append(ev[0].elapsed_time(ev[1]) / args.iters)
        nb = args.K * lay.M * 4
        print(json.dumps(dict(equal_count=True, eq_vec=vec, K=args.K, M=args.M, median_us=round(float(np.median(tt)) * 1e3, 2),
                              GBps=round(nb / (np.median(tt) / 1e3) / 1e9, 1))))
    _native.tune(eq_vec=1)
    res = []
    for i, kn in enumerate(variants):
        t = np.array(times[i])
        res.append(dict(kn, K=args.K, M=args.M, median_us=round(float(np.median(t)) * 1e3, 2),
                        GBps=round(nbytes / (np.median(t) / 1e3) / 1e9, 1)))
    for r in sorted(res, key=lambda d: d["median_us"]):
        print(json.dumps(r))


if __name__ == "__main__":
    main()
