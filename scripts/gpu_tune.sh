#!/usr/bin/env bash
# FedAvg / Scaffold launch-shape sweeps (tools/tune_*.py); $WL selects c2 c3 c4 c5; $ARGS extra flags.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-tune}
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; head -n 14 "$OUT/$name.log"; [ $rc -eq 0 ] || exit $rc; }
for wl in ${WL:-c2 c3 c5}; do
  case $wl in
    c2) run ${TAG}_c2 300 python tools/tune_fedavg.py --K 8 --M 25000000 ${ARGS:-} ;;
    c3) run ${TAG}_c3 300 python tools/tune_fedavg.py --K 64 --M 125000000 --rounds 3 --iters 5 ${ARGS:-} ;;
    c4) run ${TAG}_c4 300 python tools/tune_scaffold.py --K 16 --M 25000000 ;;
    c5) run ${TAG}_c5 600 python tools/tune_fedavg.py --K 128 --M 350000000 --kind bf16 --rounds 2 --iters 3 ${ARGS:-} ;;
  esac
done
echo "=== done"
