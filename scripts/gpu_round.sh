#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script
# (test FAILURES, exit 1, do not: the later steps are still informative).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r01}
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 600 python bench.py --steps 50 --warmup 10
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof_c2 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_${TAG}_c2 -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline
fi
echo "=== done"
