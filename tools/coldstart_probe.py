#!/usr/bin/env python3
"""Cold start of a one-shot aggregate task process: time to the first usable GPU buffer through
libfedagg's native session (--mode native) vs through PyTorch (--mode torch).  One JSON line."""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["native", "torch", "breakdown"], default="native")
    ap.add_argument("--slots", type=int, default=0)
    ap.add_argument("--chunk-mib", type=int, default=0)
    a = ap.parse_args()
    t0 = time.perf_counter()
    res = {"mode": a.mode}
    if a.mode == "breakdown":
        # every step of a one-shot task's first aggregation, in order, through the C ABI
        import ctypes

        import numpy as np

        from substrafl_amd import _native

        t = [time.perf_counter()]
        lib = _native.load()
        t.append(time.perf_counter())
        h = ctypes.c_void_p(lib.fedagg_session_create(0))
        t.append(time.perf_counter())
        if a.slots:
            lib.fedagg_session_set(h, b"slots", a.slots)
        if a.chunk_mib:
            lib.fedagg_session_set(h, b"chunk_bytes", a.chunk_mib << 20)
        lib.fedagg_session_set(h, b"threads", 16)
        n = _native.FEDAGG_SESSION_BUFFERS
        sizes = (ctypes.c_uint64 * n)(*([0] * n))
        _native.check(lib.fedagg_session_warm(h, sizes, n), "warm-ring-only")  # ring + pool + code object
        t.append(time.perf_counter())
        nbytes = 8 * 25_000_000 * 4
        d = ctypes.c_void_p()
        _native.check(lib.fedagg_session_buffer(h, 0, nbytes, ctypes.byref(d)), "buf")
        o = ctypes.c_void_p()
        _native.check(lib.fedagg_session_buffer(h, 1, nbytes // 8, ctypes.byref(o)), "buf")
        t.append(time.perf_counter())
        host = np.ones(nbytes // 4, np.float32)  # already faulted, like unpickled inputs
        t.append(time.perf_counter())
        ptrs = (ctypes.c_void_p * 1)(host.ctypes.data)
        szs = (ctypes.c_uint64 * 1)(nbytes)
        _native.check(lib.fedagg_session_stage(h, d, nbytes, 1, 1, ptrs, szs), "stage")
        _native.check(lib.fedagg_session_sync(h), "sync")
        t.append(time.perf_counter())
        _native.check(lib.fedagg_session_stage(h, d, nbytes, 1, 1, ptrs, szs), "stage")
        _native.check(lib.fedagg_session_sync(h), "sync")
        t.append(time.perf_counter())
        out = np.empty(nbytes // 8 // 4, np.float32)
        _native.check(lib.fedagg_session_fetch(h, o, ctypes.c_void_p(out.ctypes.data), out.nbytes), "fetch")
        t.append(time.perf_counter())
        _native.check(lib.fedagg_session_fetch(h, o, ctypes.c_void_p(out.ctypes.data), out.nbytes), "fetch")
        t.append(time.perf_counter())
        names = ["dlopen_lib", "session_create", "ring_pool_codeobj", "hipMalloc_900MB", "host_fault_800MB",
                 "stage_800MB_first", "stage_800MB_second", "fetch_100MB_fresh_host", "fetch_100MB_again"]
        res.update({k: round(t[i + 1] - t[i], 4) for i, k in enumerate(names)})
        res.update(slots=a.slots or "default", chunk_mib=a.chunk_mib or 16)
    elif a.mode == "native":
        from substrafl_amd import runtime

        t1 = time.perf_counter()
        s = runtime.Session(0)
        t2 = time.perf_counter()
        s.buffer(0, 800 << 20)
        s.sync()
        t3 = time.perf_counter()
        res.update(import_s=round(t1 - t0, 4), session_create_s=round(t2 - t1, 4), first_800MB_buffer_s=round(t3 - t2, 4))
    else:
        import torch

        t1 = time.perf_counter()
        x = torch.empty(800 << 20, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        y = torch.empty(800 << 20, dtype=torch.uint8, pin_memory=True)
        t3 = time.perf_counter()
        res.update(import_s=round(t1 - t0, 4), cuda_init_and_800MB_s=round(t2 - t1, 4),
                   pinned_800MB_s=round(t3 - t2, 4))
        del x, y
    res["total_s"] = round(time.perf_counter() - t0, 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
