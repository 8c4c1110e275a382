#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, tuning sweep, bench.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script
# (test FAILURES, exit 1, do not: the later steps are still informative).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${TESTS:-1}" = "1" ] && step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
[ "${TESTS:-1}" = "1" ] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${TUNE:-0}" = "1" ] && step tune_c2 600 python tools/tune_fedavg.py --K 8 --M 25000000
[ "${TUNE:-0}" = "1" ] && step tune_c3 600 python tools/tune_fedavg.py --K 64 --M 125000000 --rounds 3 --iters 5
[ "${TUNESC:-0}" = "1" ] && step tune_c4 600 python tools/tune_scaffold.py --K 16 --M 25000000
[ "${TUNE5:-0}" = "1" ] && step tune_c5 900 python tools/tune_fedavg.py --K 128 --M 350000000 --kind bf16 --rounds 2 --iters 3
for wl in ${BENCH:-c2}; do step bench_$wl 600 python bench.py --workload $wl --steps 50 --warmup 10; done
echo "=== done"
