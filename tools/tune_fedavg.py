#!/usr/bin/env python3
"""Launch-shape sweep of the FedAvg bucket kernel on one MI355X (interleaved rounds in ONE
process, cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per variant with the
median / min kernel time and GB/s of algorithmic bytes."""

import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def x_isz(dt):
    import torch

    return torch.empty(0, dtype=dt).element_size()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=8)
    ap.add_argument("--M", type=int, default=25_000_000)
    ap.add_argument("--kind", default="f32")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--full", action="store_true", help="the whole shape family (nt_store 0/1, grid-strided)")
    ap.add_argument("--xcd", action="store_true", help="each shape also with the XCD-contiguous tile order")
    ap.add_argument("--tpb", type=int, nargs="*", default=[2, 4, 8], help="auto shape with N consecutive tiles per block")
    ap.add_argument("--pads", type=int, nargs="*", default=[],
                    help="row-pitch paddings (elements) to time the auto shape with instead of the shape sweep")
    ap.add_argument("--occ", action="store_true",
                    help="register-capped occupancy variants (fa_occ 2-4) of the 8/16-KiB shapes beside the uncapped ones")
    ap.add_argument("--buf", action="store_true", help="buffer-descriptor client loads (buf 1) beside global loads")
    ap.add_argument("--sc1", action="store_true", help="write-through (sc1) output stores beside nt / plain")
    ap.add_argument("--blk", action="store_true", help="512-thread workgroups (fa_blk 512) beside the auto shape")
    ap.add_argument("--gridstride", action="store_true",
                    help="grid-strided and tile shapes under grid caps (the read probe's walk), next to the auto shape")
    args = ap.parse_args()

    import torch

    from substrafl_amd import _native
    from substrafl_amd.engine import FedAvgPlan, fedavg_weights
    from substrafl_amd.layout import BucketLayout, synthetic_state_dict_shapes

    shapes = synthetic_state_dict_shapes(args.M)
    lay = BucketLayout(range(len(shapes)), shapes, np.float32)
    dt = {"bf16": torch.bfloat16, "f32": torch.float32, "f64": torch.float64, "f16": torch.float16}[args.kind]
    out_dt = {"bf16": torch.float32, "f32": torch.float32, "f64": torch.float64, "f16": torch.float16}[args.kind]
    x = torch.empty((args.K, lay.ld), device="cuda", dtype=dt)
    for k in range(args.K):  # row by row: a full fp32 temporary of C5 would not fit
        x[k].copy_(torch.randn(lay.ld, device="cuda"))
    out = torch.empty(lay.ld, device="cuda", dtype=out_dt)
    ns = [int(v) for v in np.random.default_rng(7).integers(100, 10000, args.K)]
    plan = FedAvgPlan(args.kind, x, fedavg_weights(ns, args.kind), args.M, out, lay.pairwise_idx)
    nbytes = plan.bytes_alg()
    if args.pads:  # client rows at pitch ld + pad: do the clients' same offsets collide in the HBM channels?
        del x
        plans = []
        for pad in args.pads:
            xp = torch.empty((args.K, lay.ld + pad), device="cuda", dtype=dt)
            xp.normal_()
            plans.append((pad, FedAvgPlan(args.kind, xp[:, :lay.ld], fedavg_weights(ns, args.kind), args.M, out,
                                          lay.pairwise_idx), xp))
        _native.tune(vpt=0, tile=1, nt_store=1, grid_cap=0, xcd=0, tpb=1, pipe=0)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        tt = {pad: [] for pad, _, _ in plans}
        for r in range(args.rounds):
            for pad, pl, _ in plans:
                for _ in range(3):
                    pl.launch()
                ev[0].record()
                for _ in range(args.iters):
                    pl.launch()
                ev[1].record()
                torch.cuda.synchronize()
                tt[pad].append(ev[0].elapsed_time(ev[1]) / args.iters)
        for pad in tt:
            m = float(np.median(tt[pad]))
            print(json.dumps(dict(pad_elems=pad, pad_bytes=pad * x_isz(dt), kind=args.kind, K=args.K, M=args.M,
                                  median_us=round(m * 1e3, 2), GBps=round(nbytes / (m / 1e3) / 1e9, 1))))
        return

    base = dict(grid_cap=0, vpt=1, nt_load=1, nt_store=0, unroll=8, pipe=0, tile=0, xcd=0, tpb=1, fa_occ=0, buf=0,
                fa_blk=0, st_sc1=-1)
    if args.sc1:
        variants = [dict(base, vpt=0, tile=1, nt_store=n, st_sc1=c) for n, c in ((1, 0), (1, 1), (0, 0))]
        variants += [dict(base, vpt=v, unroll=u, tile=1, nt_store=1, st_sc1=1) for v, u in ((8, 4), (4, 4), (16, 2))]
    elif args.blk:
        variants = [dict(base, vpt=0, tile=1, nt_store=1)]
        variants += [dict(base, vpt=v, unroll=u, tile=1, nt_store=1, fa_blk=512)
                     for v, u in ((16, 2), (8, 2), (8, 4), (4, 4))]
        if args.kind == "f32":
            variants += [dict(base, vpt=v, unroll=u, tile=1, nt_store=1, fa_blk=1024) for v, u in ((8, 2), (4, 4))]
    elif args.buf:
        variants = [dict(base, vpt=0, tile=1, nt_store=1, buf=b) for b in (0, 1)]
        variants += [dict(base, vpt=v, unroll=u, tile=1, nt_store=1, fa_occ=o, buf=b)
                     for v, u, o, b in ((8, 4, 0, 0), (8, 4, 0, 1), (8, 4, 3, 1), (16, 2, 2, 0), (16, 2, 0, 1),
                                        (16, 2, 2, 1), (16, 1, 0, 0), (16, 1, 0, 1))]
    elif args.occ:
        variants = [dict(base, vpt=v, unroll=u, tile=1, nt_store=1, fa_occ=o)
                    for v, u, occs in ((8, 4, (0, 3, 4)), (16, 2, (0, 2)), (16, 1, (0, 3))) for o in occs]
        variants.insert(0, dict(base, vpt=0, tile=1, nt_store=1))
    elif args.gridstride:
        shapes = [dict(vpt=1, unroll=8), dict(vpt=1, unroll=4), dict(vpt=2, unroll=8), dict(vpt=1, unroll=8, pipe=1),
                  dict(vpt=1, unroll=16)]
        variants = [dict(base, vpt=0, tile=1, nt_store=1)]
        variants += [dict(base, **sh, tile=0, nt_store=1, grid_cap=g) for sh in shapes
                     for g in (0, 2048, 4096, 8192, 16384)]
        variants += [dict(base, vpt=v, unroll=u, tile=1, nt_store=1, grid_cap=g) for v, u in ((8, 4), (4, 4))
                     for g in (1024, 2048, 4096)]
    elif args.full:
        shapes = [dict(), dict(unroll=16), dict(vpt=2, tile=1), dict(vpt=4, tile=1), dict(vpt=4, tile=1, unroll=4),
                  dict(vpt=8, tile=1, unroll=4), dict(vpt=8, tile=1, unroll=2), dict(vpt=4, tile=1, grid_cap=8192),
                  dict(vpt=4, tile=1, grid_cap=2048)]
        variants = [dict(base, **sh, nt_store=nts) for sh in shapes for nts in (0, 1)]
    else:  # contiguous-tile shapes with nt stores (--xcd: also the XCD-contiguous tile order)
        shapes = [dict(vpt=0), dict(vpt=8, unroll=4), dict(vpt=8, unroll=2), dict(vpt=16, unroll=2), dict(vpt=16, unroll=1),
                  dict(vpt=4, unroll=4), dict(vpt=4, unroll=8), dict(vpt=2, unroll=8),
                  dict(vpt=4, unroll=4, pipe=1), dict(vpt=8, unroll=2, pipe=1), dict(vpt=1, unroll=8, tile=0, pipe=1)]
        variants = [dict(base, **dict(dict(tile=1), **sh), nt_store=1, xcd=x, tpb=1) for sh in shapes
                    for x in ((0, 1) if args.xcd else (0,))]
        variants += [dict(base, vpt=0, tile=1, nt_store=1, xcd=0, tpb=t) for t in args.tpb]
    times = {i: [] for i in range(len(variants))}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for r in range(args.rounds):
        for i, kn in enumerate(variants):
            _native.tune(**kn)
            for _ in range(3):
                plan.launch()
            ev[0].record()
            for _ in range(args.iters):
                plan.launch()
            ev[1].record()
            torch.cuda.synchronize()
            times[i].append(ev[0].elapsed_time(ev[1]) / args.iters)
    # read-stream probe ceiling at several grid sizes (same process, same buffer)
    sink = torch.empty(1 << 20, device="cuda")
    nfl = x.numel() * x.element_size() // 4 // 4 * 4
    for g in (2048, 4096, 8192, 16384, 65536, int(min(nfl // 4 // 256, 1 << 20))):
        tt = []
        for _ in range(args.rounds):
            ev[0].record()
            for _ in range(args.iters):
                _native.check(_native.load().fedagg_read_probe_f32(x.data_ptr(), nfl, sink.data_ptr(), g,
                                                                   torch.cuda.current_stream().cuda_stream), "probe")
            ev[1].record()
            torch.cuda.synchronize()
            tt.append(ev[0].elapsed_time(ev[1]) / args.iters)
        print(json.dumps(dict(probe_grid=g, bytes=nfl * 4, median_us=round(float(np.median(tt)) * 1e3, 2),
                              GBps=round(nfl * 4 / (np.median(tt) / 1e3) / 1e9, 1))))
    res = []
    for i, kn in enumerate(variants):
        t = np.array(times[i])
        res.append(dict(kn, kind=args.kind, K=args.K, M=args.M, median_us=round(float(np.median(t)) * 1e3, 2),
                        min_us=round(float(t.min()) * 1e3, 2), GBps=round(nbytes / (np.median(t) / 1e3) / 1e9, 1)))
    for r in sorted(res, key=lambda d: d["median_us"]):
        print(json.dumps(r))


if __name__ == "__main__":
    main()
