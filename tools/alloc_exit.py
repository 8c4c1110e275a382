"""A GPU process that starts HIP, allocates --gib GiB of device memory (0: none), writes it once,
and exits, printing the wall time of each phase as one JSON line: the predecessor in
scripts/r06_socclk_seq.sh, which asks whether the SOC clock's high window after a process exits
scales with the memory that process held."""

import argparse
import json
import time

T0 = time.time()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, required=True)
    args = ap.parse_args()
    import torch

    marks = {"start": T0}
    torch.zeros(1, device="cuda:0")
    torch.cuda.synchronize()
    marks["hip_ready"] = time.time()
    if args.gib > 0:
        x = torch.empty(int(args.gib * (1 << 30)) // 4, dtype=torch.float32, device="cuda:0")
        x.fill_(1.0)
        torch.cuda.synchronize()
        marks["filled"] = time.time()
        del x
        torch.cuda.empty_cache()
        torch.cuda.synchronize()
        marks["freed"] = time.time()
    marks["exit"] = time.time()
    print(json.dumps({"gib": args.gib, "marks": {k: round(v, 4) for k, v in marks.items()}}), flush=True)


if __name__ == "__main__":
    main()
