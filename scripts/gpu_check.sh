#!/usr/bin/env bash
# Parity tests (all, or the files in $FILES), smoke, and a 2-rank torchrun rehearsal of bench.py
# on one GPU (ranks share the card; the driver's N>1 runs use one GPU per rank).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 8 "$OUT/$name.log"; [ $rc -eq 0 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest ${FILES:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
[ "${SMOKE:-1}" = "1" ] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${TORCHRUN:-0}" = "1" ] && run bench_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5
echo "=== done"
