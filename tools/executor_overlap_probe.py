"""Overlap of the native lockstep executor's RCCL exchange with its chain kernels, on ONE GPU.

``fedagg_lockstep_execute`` (csrc/lockstep.hip) over a one-rank RCCL communicator: S steps, each
one FedAvg chain run of 64 clients x n fp32 elements (the striped schedule's run at 8 GPUs is
1.6-3.9M elements), and exchange groups of ``msgs`` self sends + receives of ``mib`` MiB each (the
striped schedule at 8 GPUs: six messages per step whose sizes sum to the run's accumulator bytes).
The RCCL P2P kernels here copy HBM to HBM on the one GPU instead of crossing xGMI, so this probes
only whether RCCL's kernels make progress beside a chain kernel that saturates HBM (dispatch and
memory arbitration), not the link rate.  Printed: runs only, exchange only, both (median of the
trials, HIP events on the compute stream) and overlap = (runs + exchange - both) / min(runs, exchange).

  python tools/executor_overlap_probe.py [--n 3900000] [--mib 2.6] [--msgs 6] [--steps 32]
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
    ap.add_argument("--n", type=int, default=3_900_000)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--mib", type=float, default=2.6)
    ap.add_argument("--msgs", type=int, default=6)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--trials", type=int, default=7)
    ap.add_argument("--grid-cap", type=int, default=0)
    ap.add_argument("--sdma-mib", type=float, default=0.0,
                    help="instead of RCCL: a pinned-host -> device copy of this many MiB per step on a side stream "
                         "(hipMemcpyAsync: an SDMA engine, like RCCL's copy-engine P2P path), beside the chain runs")
    ap.add_argument("--d2d", action="store_true", help="with --sdma-mib: a device -> device copy instead of "
                    "host -> device (HIP picks the engine: blit kernel or SDMA)")
    ap.add_argument("--nocu", action="store_true", help="with --d2d: hipMemcpyDeviceToDeviceNoCU (an SDMA "
                    "engine instead of a blit kernel)")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="run the chain kernels on a CU-masked stream that leaves this many CUs (spread evenly "
                         "over the mask) to the communicator's RCCL kernels")
    a = ap.parse_args()

    import numpy as np
    import torch

    from substrafl_amd import _native, rccl

    torch.cuda.set_device(0)
    lib = _native.load()
    if a.grid_cap:
        _native.tune(grid_cap=a.grid_cap)
    path = rccl.rccl_path().encode()
    uid = (ctypes.c_char * 128)()
    rccl._check(lib.fedagg_comm_unique_id(path, uid), "unique_id")
    h = ctypes.c_void_p()
    rccl._check(lib.fedagg_comm_create(path, 1, 0, uid, 0, ctypes.byref(h)), "comm_create")

    K, n, S = a.clients, a.n, a.steps
    rows = torch.randn((K, n), dtype=torch.float32, device="cuda")
    acc = torch.zeros(n, dtype=torch.float32, device="cuda")
    cnt = max(1, int(a.mib * (1 << 20) / 4))
    sbuf = torch.ones((a.msgs, cnt), dtype=torch.float32, device="cuda")
    rbuf = torch.empty((a.msgs, cnt), dtype=torch.float32, device="cuda")
    ptrs = _native.ptr_array([rows[k].data_ptr() for k in range(K)])
    w = (ctypes.c_float * K)(*[1.0 / K] * K)

    runs = []
    for t in range(S):
        r = rccl._Run()
        r.step, r.op, r.kind, r.K, r.seed, r.finish, r.n = t, _native.FEDAGG_RUN_FEDAVG, _native.FEDAGG_F32, K, 1, 0, n
        r.x, r.w, r.acc = ctypes.addressof(ptrs), ctypes.addressof(w), acc.data_ptr()
        runs.append(r)
    msgs = []
    for g in range(1, S + 1):  # group t exchanges what step t - 1 computed, beside step t
        for send in (1, 0):
            for i in range(a.msgs):
                m = rccl._Msg()
                m.group, m.send, m.peer, m.kind = g, send, 0, _native.FEDAGG_F32
                m.buf, m.count = (sbuf if send else rbuf)[i].data_ptr(), cnt
                msgs.append(m)
    R = (rccl._Run * len(runs))(*runs)
    M = (rccl._Msg * len(msgs))(*msgs)
    stream = torch.cuda.current_stream()
    if a.reserve_cus:
        ncu = torch.cuda.get_device_properties(0).multi_processor_count
        words = (ncu + 31) // 32
        mask = (ctypes.c_uint32 * words)()
        stride = ncu // a.reserve_cus
        for i in range(ncu):
            if not (i % stride == 0 and i // stride < a.reserve_cus):
                mask[i // 32] |= 1 << (i % 32)
        hip = ctypes.CDLL("libamdhip64.so")
        hs = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(hs), ctypes.c_uint32(words), mask)
        if rc:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
        stream = torch.cuda.ExternalStream(hs.value)

    def execute(with_runs, with_msgs):
        rccl._check(lib.fedagg_lockstep_execute(h, ctypes.byref(R) if with_runs else None, len(runs) if with_runs else 0,
                                                ctypes.byref(M) if with_msgs else None, len(msgs) if with_msgs else 0, S + 1,
                                                None, 0, _native.FEDAGG_F32, 0, stream.cuda_stream), "execute")

    def timed(*cfg):
        v = []
        for i in range(a.trials + 1):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            execute(*cfg)
            e1.record(stream)
            torch.cuda.synchronize()
            if i:
                v.append(e0.elapsed_time(e1))
        return float(np.median(v))

    if a.sdma_mib:
        side = torch.cuda.Stream()
        hip = ctypes.CDLL("libamdhip64.so")
        nb = int(a.sdma_mib * (1 << 20))
        host = torch.empty(nb, dtype=torch.uint8, device="cuda") if a.d2d else \
            torch.empty(nb, dtype=torch.uint8).pin_memory()
        dev = torch.empty(nb, dtype=torch.uint8, device="cuda")

        def execute(with_runs, with_copies):  # noqa: F811 -- the SDMA variant of the step loop
            evs = [torch.cuda.Event() for _ in range(S + 1)]
            for t in range(S):
                if with_copies:
                    evs[t].record(stream)
                    side.wait_event(evs[t])
                    if a.nocu:
                        rc = hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(host.data_ptr()),
                                                ctypes.c_size_t(nb), 1024, ctypes.c_void_p(side.cuda_stream))
                        if rc:
                            raise RuntimeError(f"hipMemcpyAsync(NoCU): {rc}")
                    else:
                        with torch.cuda.stream(side):
                            dev.copy_(host, non_blocking=True)
                if with_runs:
                    rccl._check(lib.fedagg_lockstep_execute(h, ctypes.byref(R, t * ctypes.sizeof(rccl._Run)), 1,
                                                            None, 0, 1, None, 0, _native.FEDAGG_F32, 0,
                                                            stream.cuda_stream), "execute")
            if with_copies:
                evs[S].record(side)
                stream.wait_event(evs[S])
        for r in runs:
            r.step = 0
        R = (rccl._Run * len(runs))(*runs)
    tr, tx, tb = timed(True, False), timed(False, True), timed(True, True)
    print(json.dumps({"clients": K, "elements_per_run": n, "steps": S, "msgs_per_group": 2 * a.msgs,
                      "MiB_per_msg": a.mib, "sdma_MiB_per_step": a.sdma_mib, "copy": ("d2d-nocu" if a.nocu else "d2d") if a.d2d else "h2d", "grid_cap": a.grid_cap, "reserved_cus": a.reserve_cus, "runs_only_ms": round(tr, 4),
                      "exchange_only_ms": round(tx, 4), "both_ms": round(tb, 4),
                      "overlap": round((tr + tx - tb) / min(tr, tx), 3),
                      "exchange_GBps_alone": round((S * a.sdma_mib * (1 << 20) if a.sdma_mib else S * a.msgs * cnt * 4)
                                                   / (tx / 1e3) / 1e9, 1)}), flush=True)
    lib.fedagg_comm_destroy(h)


if __name__ == "__main__":
    main()
