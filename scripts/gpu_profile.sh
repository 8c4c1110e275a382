#!/usr/bin/env bash
# rocprofv3 kernel-trace/stats + two separate PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r01}
WL=${WL:-c2}
STEPS=${STEPS:-30}
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"; [ $rc -eq 0 ] || exit $rc; }
run prof_${TAG}_${WL}_trace 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_${TAG}_${WL} -o trace --output-format csv -- python3 bench.py --workload $WL --steps $STEPS --warmup 5 --no-cpu-baseline
run prof_${TAG}_${WL}_fetch 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_${TAG}_${WL} -o fetch --output-format csv -- python3 bench.py --workload $WL --steps $STEPS --warmup 5 --no-cpu-baseline
run prof_${TAG}_${WL}_write 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_${TAG}_${WL} -o write --output-format csv -- python3 bench.py --workload $WL --steps $STEPS --warmup 5 --no-cpu-baseline
ls -R $OUT/prof_${TAG}_${WL} | head -30
echo "=== done"
