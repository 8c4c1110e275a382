#!/bin/bash
# Round-3 probes (gpurun from the repo root): short-run chain-kernel tiles (tuning build), and the
# cold start of a one-shot task process with the product library against the full (tuning) one.
export TMPDIR=/tmp
TAG=${1:-r03e}
TUNE=$PWD/substrafl_amd/libfedagg_tuning.so
FEDAGG_LIB=$TUNE timeout -k 10 240 python -u tools/chunk_probe.py --no-tiled --sizes 0.5e6,1e6,2e6,3.9e6,7.8e6 \
  --knobs "vpt=4,unroll=4;vpt=2,unroll=8;vpt=4,unroll=2;vpt=8,unroll=2;vpt=16,unroll=2" > gpurun_out/${TAG}_small_runs_probe.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 60 python -u tools/coldstart_probe.py --mode breakdown >> gpurun_out/${TAG}_coldstart_product.jsonl 2>/dev/null || exit 1
  FEDAGG_LIB=$TUNE timeout -k 10 60 python -u tools/coldstart_probe.py --mode breakdown >> gpurun_out/${TAG}_coldstart_fulllib.jsonl 2>/dev/null || exit 1
done
timeout -k 10 300 python -u tests/perf/task_probe.py --K 8 --M 25000000 --reps 3 > gpurun_out/${TAG}_task_c2_product.jsonl 2>&1 || exit 1
FEDAGG_LIB=$TUNE timeout -k 10 300 python -u tests/perf/task_probe.py --K 8 --M 25000000 --reps 3 > gpurun_out/${TAG}_task_c2_fulllib.jsonl 2>&1
