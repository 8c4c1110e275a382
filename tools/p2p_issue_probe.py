#!/usr/bin/env python3
"""Host cost of issuing one batched point-to-point exchange through torch.distributed
(batch_isend_irecv) with 1, 4 and 8 sends + receives per batch -- the per-step issue cost of the
Python lockstep executor.  Two gloo ranks on the CPU, 16-element tensors."""
import os, sys, time, torch, torch.distributed as dist
import torch.multiprocessing as mp
def w(r, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=r, world_size=2)
    peer = 1 - r
    bufs = [torch.zeros(16) for _ in range(8)]
    rb = [torch.zeros(16) for _ in range(8)]
    for n in (1, 4, 8):
        ts = []
        for it in range(200):
            ops = [dist.P2POp(dist.isend, bufs[i], peer) for i in range(n)] + [dist.P2POp(dist.irecv, rb[i], peer) for i in range(n)]
            t0 = time.perf_counter()
            works = dist.batch_isend_irecv(ops)
            t1 = time.perf_counter()
            for x in works: x.wait()
            ts.append(t1 - t0)
        if r == 0: print(f"{n} sends+{n} recvs: issue {1e6*sorted(ts)[100]:.1f} us median", flush=True)
    dist.destroy_process_group()
if __name__ == "__main__":
    mp.spawn(w, args=(29733,), nprocs=2)
