#!/usr/bin/env bash
# End-to-end (host pickles -> GPU -> host) timing of the drop-in path + cold-start probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 600 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 4 gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
run cold_native python tools/coldstart_probe.py --mode native
run cold_torch python tools/coldstart_probe.py --mode torch
run e2e_c2 python tests/perf/e2e_bench.py --K 8 --M 25000000 --reps 3
run e2e_k64 python tests/perf/e2e_bench.py --K 64 --M 4000000 --reps 2
echo done
