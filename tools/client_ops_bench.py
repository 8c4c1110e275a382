#!/usr/bin/env python3
"""Client-side bucket ops on one MI355X: the reference's per-layer
torch loops (substrafl/algorithms/pytorch/weight_manager.py:79-212, the Δ export of
torch_fed_avg_algo.py:227-230) against substrafl_amd.algorithms.weight_manager's flat-bucket
launches, on the same ROCm tensors.  Device time per call (HIP events, median of --iters), the
algorithmic bytes moved, and a bit-equality check of the two results.

One round of a FedAvg client does: get_parameters (copy of the weights, :79-100), train,
subtract_parameters (Δ = after - before, :140-158 -> weighted_sum :182-212), export of Δ to host
(.cpu().numpy() per layer), then on the next round increment_parameters (w += 1.0 * avg, :103-137).
Prints one JSON line per (model, op)."""

import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=25_000_000)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    from substrafl_amd.algorithms import weight_manager as wm
    from substrafl_amd.layout import synthetic_state_dict_shapes

    dev = torch.device("cuda", 0)
    models = {
        f"synthetic_{args.M // 1_000_000}M_{len(synthetic_state_dict_shapes(args.M))}layers":
            synthetic_state_dict_shapes(args.M),
        # MNIST-CNN-like: many small layers (launch-bound in the per-layer loop)
        "cnn_small_10layers": [(32, 1, 5, 5), (32,), (64, 32, 5, 5), (64,), (1024, 1600), (1024,), (10, 1024),
                               (10,), (64,), (64,)],
    }

    class Net(torch.nn.Module):
        def __init__(self, shapes):
            super().__init__()
            self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(s)) for s in shapes])

    def timed(fn, iters):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(iters):
            ev[0].record()
            fn()
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        return float(np.median(ts))

    for name, shapes in models.items():
        torch.manual_seed(0)
        model = Net(shapes).to(dev)
        params = list(model.parameters())
        M = sum(p.numel() for p in params)
        before = [p.detach().clone() for p in params]
        after = [p + 0.01 * torch.randn_like(p) for p in params]
        upd = [0.001 * torch.randn_like(p) for p in params]

        # reference loops (weight_manager.py), restated inline
        def ref_get():
            with torch.no_grad():
                return [p.clone() for p in params]

        def ref_sub():
            with torch.no_grad():
                return [sum(a * c for a, c in zip(pair, [1, -1])) for pair in zip(after, before)]

        def ref_inc():
            with torch.no_grad():
                for w, u in zip(params, upd):
                    w.data += 1.0 * u.data

        def ref_export(delta):
            return [p.cpu().detach().numpy() for p in delta]

        ops = {
            "get_parameters": (ref_get, lambda: wm.get_parameters(model, False), 2 * M * 4),
            "subtract_parameters": (ref_sub, lambda: wm.subtract_parameters(after, before), 3 * M * 4),
            "increment_parameters": (ref_inc, lambda: wm.increment_parameters(model, upd,
                                                                              with_batch_norm_parameters=False),
                                     3 * M * 4),
        }
        for op, (ref_fn, our_fn, nbytes) in ops.items():
            if op == "increment_parameters":  # same start point for the equality check
                snap = [p.detach().clone() for p in params]
                ref_fn()
                r = [p.detach().clone() for p in params]
                with torch.no_grad():
                    for p, s in zip(params, snap):
                        p.copy_(s)
                our_fn()
                o = [p.detach().clone() for p in params]
                with torch.no_grad():
                    for p, s in zip(params, snap):
                        p.copy_(s)
            else:
                r, o = ref_fn(), our_fn()
            same = all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(r, o))
            t_ref = timed(ref_fn, args.iters)
            t_our = timed(our_fn, args.iters)
            print(json.dumps({"model": name, "layers": len(shapes), "params": M, "op": op,
                              "reference_loop_ms": round(t_ref, 4), "flat_bucket_ms": round(t_our, 4),
                              "speedup": round(t_ref / t_our, 2), "flat_GBps": round(nbytes / (t_our / 1e3) / 1e9, 1),
                              "bit_equal": bool(same)}), flush=True)
        # export of Δ to host: per-layer D2H vs one D2H of the flat bucket (wall time, host included)
        import time

        d_ref = ref_sub()
        d_our = wm.subtract_parameters(after, before)
        for tag, fn in (("reference_loop", lambda: ref_export(d_ref)), ("flat_bucket", lambda: wm.export_numpy(d_our))):
            fn()
            ts = []
            for _ in range(max(3, args.iters // 4)):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            print(json.dumps({"model": name, "op": "export_numpy", "path": tag,
                              "ms": round(float(np.median(ts)) * 1e3, 3),
                              "GBps": round(M * 4 / float(np.median(ts)) / 1e9, 2)}), flush=True)
        same = all(np.array_equal(a.view(np.uint32), b.view(np.uint32))
                   for a, b in zip(ref_export(d_ref), wm.export_numpy(d_our)))
        print(json.dumps({"model": name, "op": "export_numpy", "bit_equal": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
