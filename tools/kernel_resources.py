#!/usr/bin/env python3
"""Register / LDS / occupancy of every kernel instantiation in fedagg.hip, from the compiler's
code-object metadata (hipcc -Rpass-analysis=kernel-resource-usage; gfx950).  Prints one line per
kernel: template arguments, VGPRs, AGPRs, scratch bytes per lane, LDS bytes, waves per SIMD.
Usage: tools/kernel_resources.py [--filter scaffold_kernel] > profiles/<tag>_kernel_resources.txt"""

import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filter", default="", help="substring of the demangled kernel name")
    ap.add_argument("--tuning", action="store_true", help="the FEDAGG_TUNING build (every experiment variant)")
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                            "-fPIC", "-c", f"-I{ROOT / 'include'}", str(ROOT / "substrafl_amd" / "csrc" / "fedagg.hip"),
                            "-o", str(Path(d) / "fa.o"), "-Rpass-analysis=kernel-resource-usage"]
                           + (["-DFEDAGG_TUNING=1"] if args.tuning else []),
                           capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-2000:])
    for block in re.split(r"remark: Function Name: ", r.stderr)[1:]:
        name = block.split()[0]
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dem = dem.replace("(anonymous namespace)::", "")
        short = dem.split("(")[0] if "<" not in dem else dem[: dem.index(">(") + 1]
        if args.filter and args.filter not in short:
            continue

        def get(key):
            m = re.search(key + r": (\d+)", block)
            return m.group(1) if m else "?"

        scratch = get(r"ScratchSize \[bytes/lane\]")
        lds = get(r"LDS Size \[bytes/block\]")
        occ = get(r"Occupancy \[waves/SIMD\]")
        print(f"{short}  VGPR {get('VGPRs')}  AGPR {get('AGPRs')}  scratch {scratch}  LDS {lds}  waves/SIMD {occ}")


if __name__ == "__main__":
    main()
