"""Per-step cost of the push executor's order kernels (fedagg_push_execute, csrc/lockstep.hip) on
one GPU: S steps with no runs, each with a one-lane wait kernel whose counters -- and landing
tags (ABI 13) -- are already there (``--waits`` producers per step, each a counter and a tag) and
the step's signal kernel writing ``--waits`` tags; and the same S steps around the chain runs of a
64-client x n-element block (runs alone, through the executor's own run table, against runs +
waits + signals).  Also the cost of the push runs' per-wave system-scope release
(``fedagg_fedavg_chain_push_f32`` against ``fedagg_fedavg_chain_f32``, back to back).  The counters
live in a page-locked host page, as in substrafl_amd/push.py.

  python tools/push_overhead_probe.py [--steps 48] [--n 2600000] [--waits 6] [--push-runs]
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
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--n", type=int, default=2_600_000)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--waits", type=int, default=6)
    ap.add_argument("--trials", type=int, default=9)
    ap.add_argument("--push-runs", action="store_true", help="the executor's runs as FEDAGG_RUN_FEDAVG_PUSH")
    a = ap.parse_args()

    import numpy as np
    import torch

    from substrafl_amd import _native, push, rccl

    torch.cuda.set_device(0)
    lib = _native.load()
    G = max(2, a.waits + 1)
    page = np.zeros(512, np.uint64)
    dev = ctypes.c_void_p()
    push._check(lib.fedagg_host_map(page.ctypes.data, page.nbytes, ctypes.byref(dev)), "fedagg_host_map")
    page[1:G] = 1 << 40  # the other "ranks" are far ahead: every wait is satisfied at once
    K, n, S = a.clients, a.n, a.steps
    rows = torch.randn((K, n), dtype=torch.float32, device="cuda")
    acc = torch.zeros(n, dtype=torch.float32, device="cuda")
    ptrs = _native.ptr_array([rows[k].data_ptr() for k in range(K)])
    w = (ctypes.c_float * K)(*[1.0 / K] * K)
    runs = []
    for t in range(S):
        r = rccl._Run()
        op = _native.FEDAGG_RUN_FEDAVG_PUSH if a.push_runs else _native.FEDAGG_RUN_FEDAVG
        r.step, r.op, r.kind, r.K, r.seed, r.finish, r.n = t, op, _native.FEDAGG_F32, K, 1, 0, n
        r.x, r.w, r.acc = ctypes.addressof(ptrs), ctypes.addressof(w), acc.data_ptr()
        runs.append(r)
    R = (rccl._Run * S)(*runs)
    landed = torch.full((1,), 1 << 40, dtype=torch.int64, device="cuda")  # every tag already there
    sink = torch.zeros(max(1, a.waits), dtype=torch.int64, device="cuda")  # where the signals' tags go
    waits = [push._Wait(t, 1 + i, 1, landed.data_ptr()) for t in range(S) for i in range(a.waits)]
    W = (push._Wait * max(1, len(waits)))(*waits)
    tags = [push._Tag(t, 0, sink.data_ptr() + 8 * i) for t in range(S) for i in range(a.waits)]
    T = (push._Tag * max(1, len(tags)))(*tags)
    stream = torch.cuda.current_stream()
    base = [0]

    def call(with_runs, with_order):
        push._check(lib.fedagg_push_execute(ctypes.byref(R) if with_runs else None, S if with_runs else 0,
                                            ctypes.byref(W) if with_order and waits else None,
                                            len(waits) if with_order else 0,
                                            ctypes.byref(T) if with_order and tags else None,
                                            len(tags) if with_order else 0, S, dev.value, 0, G, base[0],
                                            1 << 40, None, None, 0, _native.FEDAGG_F32, None, None, 0, None, 0,
                                            stream.cuda_stream), "fedagg_push_execute")
        base[0] += S + 1

    def timed(*cfg):
        v = []
        for i in range(a.trials + 1):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            call(*cfg)
            e1.record(stream)
            torch.cuda.synchronize()
            if i:
                v.append(e0.elapsed_time(e1))
        return float(np.median(v))

    def plain_runs(fn):
        for _ in range(S):
            seed = None if fn is lib.fedagg_fedavg_chain_push_f32 else 1  # push: d_in NULL = seed
            _native.check(fn(ptrs, w, K, n, seed, acc.data_ptr(), stream.cuda_stream), "chain")

    def timed_plain(fn):
        v = []
        for i in range(a.trials + 1):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            plain_runs(fn)
            e1.record(stream)
            torch.cuda.synchronize()
            if i:
                v.append(e0.elapsed_time(e1))
        return float(np.median(v))

    chain_plain = timed_plain(lib.fedagg_fedavg_chain_f32)
    chain_release = timed_plain(lib.fedagg_fedavg_chain_push_f32)
    chain_plain2 = timed_plain(lib.fedagg_fedavg_chain_f32)
    runs_only = chain_release if a.push_runs else min(chain_plain, chain_plain2)
    order = timed(False, True)
    runs_sig = timed(True, False)  # runs + the step signals (no waits)
    both = timed(True, True)
    nbytes = (K * n + n) * 4
    print(json.dumps({"steps": S, "waits_per_step": a.waits, "tags_per_step": a.waits, "push_runs": a.push_runs,
                      "clients": K, "elements_per_run": n,
                      "chain_plain_us": round(min(chain_plain, chain_plain2) / S * 1e3, 2),
                      "chain_release_us": round(chain_release / S * 1e3, 2),
                      "chain_release_cost_pct": round((chain_release / min(chain_plain, chain_plain2) - 1) * 100, 2),
                      "chain_plain_TBps": round(nbytes / (min(chain_plain, chain_plain2) / S * 1e-3) / 1e12, 3),
                      "runs_only_ms": round(runs_only, 4), "order_only_ms": round(order, 4), "order_us_per_step": round(order / S * 1e3, 2),
                      "runs_and_signals_ms": round(runs_sig, 4), "runs_signals_waits_ms": round(both, 4),
                      "added_us_per_step": round((both - runs_only) / S * 1e3, 2)}), flush=True)
    lib.fedagg_host_unmap(page.ctypes.data)


if __name__ == "__main__":
    main()
