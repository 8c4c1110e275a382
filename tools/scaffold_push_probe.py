"""Cost of the Scaffold push runs on one GPU (local memory): one client block's two sums as the
push executor issues them -- ``fedagg_scaffold_chain_push_f32`` phase 0 (delta rows) and phase 1
(control-variate rows), each continuing its fp64 input accumulator into a separate output with
system-scope write-through stores -- against ``fedagg_scaffold_chain_f32`` continuing the same two
accumulators in place (the RCCL executor's runs).  Same bytes either way (K x n fp32 per bucket
in, an fp64 accumulator in and out per bucket); results compared bit for bit.

  python tools/scaffold_push_probe.py [--trials 20]   (one JSON line per shape)
"""

from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=20)
    a = ap.parse_args()

    import torch

    from substrafl_amd import _native

    torch.cuda.set_device(0)
    lib = _native.load()
    s = torch.cuda.current_stream().cuda_stream
    # (clients in the block, elements of the run): C4 over 8 GPUs (2 clients x M / 8), a 64-client
    # Scaffold over 8 GPUs, and a whole C4 block on one GPU
    for K, n in ((2, 3_125_248), (8, 3_125_248), (16, 25_000_000)):
        torch.manual_seed(K)
        d = torch.randn((K, n), device="cuda")
        v = torch.randn((K, n), device="cuda")
        c = torch.randn(n, device="cuda")
        w = (ctypes.c_double * K)(*[1.0 / (k + 3) for k in range(K)])
        dp = _native.ptr_array([d[k].data_ptr() for k in range(K)])
        vp = _native.ptr_array([v[k].data_ptr() for k in range(K)])
        ins = [torch.randn(n, dtype=torch.float64, device="cuda") for _ in range(2)]
        outs = [torch.empty(n, dtype=torch.float64, device="cuda") for _ in range(2)]
        inplace = [x.clone() for x in ins]

        def chain():
            for x, y in zip(inplace, ins):
                x.copy_(y)  # (outside the timed launch: each timed call continues the same input)
            ev0.record()
            _native.check(lib.fedagg_scaffold_chain_f32(dp, vp, c.data_ptr(), w, K, n, 0, 1, 0.5,
                                                        inplace[0].data_ptr(), inplace[1].data_ptr(), s), "chain")
            ev1.record()

        def push():
            ev0.record()
            for ph, rows in enumerate((dp, vp)):
                _native.check(lib.fedagg_scaffold_chain_push_f32(rows, w, K, n, ph, c.data_ptr(), 0.5, 1,
                                                                 ins[ph].data_ptr(), outs[ph].data_ptr(), s), "push")
            ev1.record()

        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = {}
        for name, fn in (("chain_inplace", chain), ("push_two_launches", push)):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.trials):
                fn()
                torch.cuda.synchronize()
                ts.append(ev0.elapsed_time(ev1))
            res[name] = sorted(ts)[len(ts) // 2]
        same = all(torch.equal(x.view(torch.int64), y.view(torch.int64)) for x, y in zip(inplace, outs))
        nbytes = 2 * K * n * 4 + n * 4 + 4 * n * 8
        print(json.dumps({"clients": K, "elements": n, "bytes": nbytes, "bit_identical": same,
                          **{f"{k}_us": round(t * 1e3, 1) for k, t in res.items()},
                          **{f"{k}_GBps": round(nbytes / (t / 1e3) / 1e9, 1) for k, t in res.items()},
                          "push_over_chain": round(res["push_two_launches"] / res["chain_inplace"], 4)}), flush=True)


if __name__ == "__main__":
    main()
