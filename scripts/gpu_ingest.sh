#!/usr/bin/env bash
# Host ingest + end-to-end runs: in-process warm/cold phases, both
# wire formats, threaded loading, and fresh-process (subprocess-mode) aggregate tasks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 900 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 4 gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
[ "${PROBE:-0}" = "1" ] && run ingest_c2 python tools/ingest_probe.py --K 8 --M 25000000
run task_c2 python tests/perf/task_probe.py --K 8 --M 25000000 --reps 3
run task_k64 python tests/perf/task_probe.py --K 64 --M 4000000 --reps 2
run e2e_c2_prewarm python tests/perf/e2e_bench.py --K 8 --M 25000000 --reps 3 --wire layers --loader threads --prewarm
[ "${E2E_ALL:-0}" = "1" ] && run e2e_c2_flat_thr python tests/perf/e2e_bench.py --K 8 --M 25000000 --reps 3 --wire flat --loader threads
echo done
