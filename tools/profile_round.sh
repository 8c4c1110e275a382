#!/bin/bash
# One profiling session per workload, on the GPU box (DESIGN.md §5 evidence):
#   1. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) -> HBM bytes per launch (tools/pmc_traffic.py);
#   2. the bench line itself, whose roofline.traffic is that file (same build, same session);
#   3. rocprofv3 --kernel-trace --stats of the same bench command (kernel average duration);
#   4. tools/roofline_check.py: the plain line's HIP-event kernel time, the profiled line's (the
#      process rocprof traced) and rocprof's average / min side by side, with the fraction each gives.
# Usage: tools/profile_round.sh TAG WORKLOAD [WORKLOAD ...]   (outputs under gpurun_out/TAG_*)
set -euo pipefail
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for WL in "$@"; do
  case $WL in
    c2) KERN=fedavg_kernel; ALG=900000000; STEPS=200; GROUP=1 ;;
    c3) KERN=fedavg_kernel; ALG=32500000000; STEPS=100; GROUP=1 ;;
    c4) KERN=scaffold; ALG=3700000000; STEPS=100
        # launches per Scaffold call under the library's defaults (1 fused walk, or 2 one-bucket launches)
        GROUP=$(python3 -c "import sys; sys.path.insert(0, '$ROOT'); from substrafl_amd import _native; \
print(_native.load().fedagg_scaffold_launches(16, 4, 25000000, 1))") ;;
    c5) KERN=fedavg_kernel; ALG=91000000000; STEPS=30; GROUP=1 ;;
    *) echo "unknown workload $WL"; exit 2 ;;
  esac
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "[$TAG] $WL: pmc $C" >&2
    rm -rf "$OUT/${TAG}_pmc_${C}_${WL}"
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/${TAG}_pmc_${C}_${WL}" -o run -- \
      python3 "$ROOT/bench.py" --workload "$WL" --steps 10 --warmup 2 --no-cpu-baseline > /dev/null
    cp "$(find "$OUT/${TAG}_pmc_${C}_${WL}" -name '*counter_collection.csv' | head -1)" "$OUT/${TAG}_${WL}_pmc_${C}.csv"
  done
  python3 "$ROOT/tools/pmc_traffic.py" --fetch "$OUT/${TAG}_${WL}_pmc_FETCH_SIZE.csv" \
    --write "$OUT/${TAG}_${WL}_pmc_WRITE_SIZE.csv" --kernel $KERN --group $GROUP --bytes-alg $ALG \
    --lib "$ROOT/substrafl_amd/libfedagg.so" --collected "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, session $TAG" \
    --out "$OUT/${TAG}_traffic_${WL}.json" > /dev/null
  # the bench line of this session carries the traffic just measured on this very build
  echo "[$TAG] $WL: bench" >&2
  timeout -k 10 400 python3 "$ROOT/bench.py" --workload "$WL" --steps $STEPS --warmup 10 \
    --traffic "$OUT/${TAG}_traffic_${WL}.json" > "$OUT/${TAG}_bench_${WL}.json"
  echo "[$TAG] $WL: kernel trace" >&2
  rm -rf "$OUT/${TAG}_prof_${WL}"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_${WL}" -o run -- \
    python3 "$ROOT/bench.py" --workload "$WL" --steps $STEPS --warmup 10 --no-cpu-baseline \
    --traffic "$OUT/${TAG}_traffic_${WL}.json" > "$OUT/${TAG}_profiled_bench_${WL}.json"
  STATS=$(find "$OUT/${TAG}_prof_${WL}" -name '*kernel_stats.csv' | head -1)
  cp "$STATS" "$OUT/${TAG}_${WL}_kernel_stats.csv"
  TRACE=$(find "$OUT/${TAG}_prof_${WL}" -name '*kernel_trace.csv' | head -1)
  cp "$TRACE" "$OUT/${TAG}_${WL}_kernel_trace.csv"
  KPFX=$([ "$KERN" = scaffold ] && echo scaffold || echo fedavg_kernel)
  python3 "$ROOT/tools/roofline_check.py" --bench "$OUT/${TAG}_bench_${WL}.json" \
    --profiled "$OUT/${TAG}_profiled_bench_${WL}.json" --stats "$OUT/${TAG}_${WL}_kernel_stats.csv" \
    --kernel "$KPFX" --group $GROUP --trace "$OUT/${TAG}_${WL}_kernel_trace.csv" \
    --out "$OUT/${TAG}_${WL}_roofline_check.json" > /dev/null
done
echo "[$TAG] done" >&2
