#!/bin/bash
# One GPU session of round 3 (run by gpurun from the repo root): tests, then profiling of this build.
export TMPDIR=/tmp
TAG=${1:-r03}
timeout -k 10 300 python -u -m pytest tests/test_client_shard_gpu.py -x -v --timeout 200 --timeout-method thread -k "native or tiled_client or host_entry" > gpurun_out/${TAG}_native_tests.log 2>&1 || exit 1
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 bash tools/profile_round.sh ${TAG} c3 c2 c4 c5 > gpurun_out/${TAG}_profile.log 2>&1
FEDAGG_LIB=$PWD/substrafl_amd/libfedagg_tuning.so timeout -k 10 200 python -u tools/chunk_probe.py --no-tiled --sizes 0.5e6,1e6,2e6,3.9e6,7.8e6 --knobs "vpt=4,unroll=4;vpt=2,unroll=8;vpt=4,unroll=2;vpt=8,unroll=2" > gpurun_out/${TAG}_small_runs_probe.log 2>&1
