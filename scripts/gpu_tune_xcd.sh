#!/usr/bin/env bash
# XCD-contiguous tile order vs identity order: FedAvg (C2, C3, C5) and Scaffold (C4) sweeps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; head -n 20 "$OUT/$name.log"; [ $rc -eq 0 ] || exit $rc; }
run xcd_c2 300 python tools/tune_fedavg.py --K 8 --M 25000000
run xcd_c3 300 python tools/tune_fedavg.py --K 64 --M 125000000 --rounds 3 --iters 5
run xcd_c4 300 python tools/tune_scaffold.py --K 16 --M 25000000
run xcd_c5 600 python tools/tune_fedavg.py --K 128 --M 350000000 --kind bf16 --rounds 2 --iters 3
echo "=== done"
