#!/bin/bash
# HBM read/write turnaround evidence (VERDICT r04 "Next 5"): for C2 (output 1/8 of input), C4
# (Scaffold, 1/8, fp64 out) and C3 (1/64), two --pmc passes of the product kernels --
#   A: TCC_EA0_RDREQ / WRREQ (memory-side requests) and their _LEVEL integrals (in-flight requests
#      per cycle: average latency = LEVEL / REQ), with GRBM_GUI_ACTIVE;
#   B: DRAM credit stalls of reads and writes, the EA write-request stall and "too many EA write
#      requests" stall, with GRBM_GUI_ACTIVE --
# then tools/turnaround_counters.py summarises per kernel.  Outputs under gpurun_out/TAG_*.
set -euo pipefail
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PASS_A="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE"
PASS_B="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum GRBM_GUI_ACTIVE"
for WL in "$@"; do
  for P in A B; do
    eval CTRS=\$PASS_$P
    echo "[$TAG] $WL: pass $P" >&2
    rm -rf "$OUT/${TAG}_pmc${P}_${WL}"
    timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/${TAG}_pmc${P}_${WL}" -o run -- \
      python3 "$ROOT/bench.py" --workload "$WL" --steps 10 --warmup 2 --no-cpu-baseline > /dev/null
    cp "$(find "$OUT/${TAG}_pmc${P}_${WL}" -name '*counter_collection.csv' | head -1)" "$OUT/${TAG}_${WL}_pmc${P}.csv"
  done
done
python3 "$ROOT/tools/turnaround_counters.py" --tag "$TAG" --dir "$OUT" "$@" > "$OUT/${TAG}_turnaround.json"
echo "[$TAG] done" >&2
