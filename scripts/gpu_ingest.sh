#!/usr/bin/env bash
# Host ingest probe + end-to-end runs in both wire formats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 600 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 4 gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
run ingest_c2 python tools/ingest_probe.py --K 8 --M 25000000
run ingest_k64 python tools/ingest_probe.py --K 64 --M 4000000 --reps 2
run e2e_c2_layers python tools/e2e_bench.py --K 8 --M 25000000 --reps 3 --wire layers
run e2e_c2_flat python tools/e2e_bench.py --K 8 --M 25000000 --reps 3 --wire flat
run e2e_c2_flat_thr python tools/e2e_bench.py --K 8 --M 25000000 --reps 3 --wire flat --loader threads
run e2e_c2_layers_thr python tools/e2e_bench.py --K 8 --M 25000000 --reps 3 --wire layers --loader threads
run e2e_k64_flat python tools/e2e_bench.py --K 64 --M 4000000 --reps 2 --wire flat
echo done
