#!/usr/bin/env bash
# Round evidence: GPU parity suite, smoke, the bench line of every workload, and the rocprofv3
# kernel-trace + PMC passes of the default workload (c2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
SMOKE=1 FILES=tests bash scripts/gpu_check.sh || exit $?
for wl in ${BENCH:-c2 c3 c4 c5}; do
  echo "=== bench_$wl"
  timeout -k 10 600 python bench.py --workload $wl > $OUT/bench_$wl.log 2>&1 || exit $?
  grep -h '"metric"' $OUT/bench_$wl.log | cut -c1-200
done
[ "${PROFILE:-1}" = "1" ] && { WL=c2 STEPS=30 bash scripts/gpu_profile.sh || exit $?; }
echo "=== done"
