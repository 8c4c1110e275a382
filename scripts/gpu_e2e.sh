#!/usr/bin/env bash
# End-to-end (host pickles -> GPU -> host) timing of the drop-in path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/e2e_bench.py --K 8 --M 25000000 --reps 3 > gpurun_out/e2e_c2.log 2>&1 || exit $?
timeout -k 10 900 python tools/e2e_bench.py --K 8 --M 25000000 --reps 2 --threads 16 > gpurun_out/e2e_c2_t16.log 2>&1 || exit $?
timeout -k 10 900 python tools/e2e_bench.py --K 64 --M 4000000 --reps 2 --threads 16 > gpurun_out/e2e_k64.log 2>&1 || exit $?
echo done
