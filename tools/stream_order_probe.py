"""Is work issued by torch and work issued by libfedagg on the same stream handle ordered?

The client-shard paths mix them on "torch's current stream" (sharding.GpuShardOps launches
libfedagg kernels on ``torch.cuda.current_stream().cuda_stream``; the buffers around them are
zeroed / summed / copied by torch ops).  tools/push_tail_probe.py found the root's numel == 1
workspace read by a libfedagg kernel BEFORE a torch copy into it had landed, although a libfedagg
snapshot kernel issued in between saw the copy.  This probe isolates the question on one process:

    1. a long libfedagg kernel writes A := B (B = 2.0, 1 GiB: milliseconds)     [libfedagg, handle h]
    2. a torch op on the same stream: A += 1                                      [torch]
    3. a libfedagg kernel copies A -> C                                           [libfedagg, handle h]
    4. synchronize; in stream order A == C == 3 everywhere.

for h = torch's current (default) stream, an explicit torch.cuda.Stream, and the default stream
entered through torch.cuda.stream(ExternalStream(h)) (the round-3 tail's idiom); with the torch op
a kernel (add_) and a runtime copy (copy_ from a 3.0 tensor); each case repeated.  One JSON line
per case: the handles seen, and how many elements of A / C are out of order.
"""

from __future__ import annotations

import contextlib
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from substrafl_amd import _native

    lib = _native.load()
    dev = torch.device("cuda", 0)
    n = 1 << 28  # 1 GiB of fp32
    B = torch.full((n,), 2.0, device=dev)
    A = torch.zeros(n, device=dev)
    C = torch.zeros(n, device=dev)
    three = torch.full((n,), 3.0, device=dev)
    cnt = (ctypes.c_uint64 * 1)(n)

    def fed_copy(dst, src, h):
        _native.check(lib.fedagg_flat_gather_f32(_native.ptr_array([src.data_ptr()]), cnt, 1, dst.data_ptr(), h),
                      "flat_gather")

    side = torch.cuda.Stream(device=dev)
    cases = []
    for stream_name in ("current", "side", "external_current"):
        for op in ("add_", "copy_"):
            cases.append((stream_name, op))
    for rep in range(3):
        for stream_name, op in cases:
            A.zero_()
            C.zero_()
            torch.cuda.synchronize()
            if stream_name == "side":
                ctxm = torch.cuda.stream(side)
            else:
                ctxm = contextlib.nullcontext()
            with ctxm:
                h = int(torch.cuda.current_stream().cuda_stream)
                fed_copy(A, B, h)                                   # 1: A := 2 (long)
                inner = torch.cuda.stream(torch.cuda.ExternalStream(h)) if stream_name == "external_current" \
                    else contextlib.nullcontext()
                with inner:
                    h_in = int(torch.cuda.current_stream().cuda_stream)
                    if op == "add_":
                        A.add_(1.0)                                 # 2: A += 1 (torch kernel)
                    else:
                        A.copy_(three)                              # 2: A := 3 (torch copy_)
                fed_copy(C, A, h)                                   # 3: C := A
            torch.cuda.synchronize()
            bad_a = int((A != 3.0).sum().item())
            bad_c = int((C != 3.0).sum().item())
            print(json.dumps({"rep": rep, "stream": stream_name, "torch_op": op, "handle": h, "handle_in_ctx": h_in,
                              "A_not_3": bad_a, "C_not_3": bad_c}), flush=True)


def small(reps: int = 300):
    """The tail's shape at its size: a 36-float buffer W written by a one-workgroup libfedagg
    kernel (zeros, then the pattern P1), then overwritten by a torch op (P2 = P1 + 1: add_, or
    copy_ from a P2 tensor), then read by a one-workgroup libfedagg kernel into C; `reps` times
    back to back on one stream.  C must be P2 every time.  Control: the overwrite as a libfedagg
    kernel too."""
    import torch

    from substrafl_amd import _native

    lib = _native.load()
    dev = torch.device("cuda", 0)
    m = 36
    p1 = torch.arange(m, dtype=torch.float32, device=dev) + 1.0
    p2 = p1 + 1.0
    zero = torch.zeros(m, device=dev)
    W = torch.zeros(m, device=dev)
    Cs = torch.zeros((reps, m), device=dev)
    cnt = (ctypes.c_uint64 * 1)(m)
    h = int(torch.cuda.current_stream().cuda_stream)

    def fed_copy(dst_ptr, src):
        _native.check(lib.fedagg_flat_gather_f32(_native.ptr_array([src.data_ptr()]), cnt, 1, dst_ptr, h), "gather")

    for op in ("fedagg_control", "torch_add_", "torch_copy_", "torch_add_ext"):
        Cs.zero_()
        torch.cuda.synchronize()
        for i in range(reps):
            fed_copy(W.data_ptr(), zero)
            fed_copy(W.data_ptr(), p1)
            if op == "fedagg_control":
                fed_copy(W.data_ptr(), p2)
            elif op == "torch_add_":
                W.add_(1.0)
            elif op == "torch_copy_":
                W.copy_(p2)
            else:
                with torch.cuda.stream(torch.cuda.ExternalStream(h)):
                    W.add_(1.0)
            fed_copy(Cs[i].data_ptr(), W)
        torch.cuda.synchronize()
        bad = (Cs != p2[None, :]).any(dim=1)
        stale_p1 = (Cs == p1[None, :]).all(dim=1)
        print(json.dumps({"case": "small", "op": op, "reps": reps, "handle": h, "wrong_reads": int(bad.sum().item()),
                          "reads_equal_to_P1": int(stale_p1.sum().item()),
                          "first_wrong": [int(x) for x in torch.nonzero(bad).view(-1)[:8].tolist()]}), flush=True)


if __name__ == "__main__":
    small()
    main()
