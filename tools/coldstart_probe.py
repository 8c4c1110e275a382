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
    ap.add_argument("--mode", choices=["native", "torch"], default="native")
    a = ap.parse_args()
    t0 = time.perf_counter()
    res = {"mode": a.mode}
    if a.mode == "native":
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
