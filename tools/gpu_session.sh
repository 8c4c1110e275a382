#!/bin/bash
# One GPU session of round 3 (run by gpurun from the repo root): tests, probes, then (PROFILE=1)
# the profiling of this build.
export TMPDIR=/tmp
TAG=${1:-r03}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 300 python -u -m pytest tests/test_client_shard_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_shard_tests.log 2>&1 || exit 1
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || exit 1
fi
timeout -k 10 200 python -u tools/chunk_probe.py --sizes 0.5e6,1e6,1.5e6,2e6,3e6,3.9e6,7.8e6,15.6e6,31.25e6 --no-tiled > gpurun_out/${TAG}_chunk_probe.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || exit 1
timeout -k 10 200 python -u bench.py --mode client-shard --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_client_shard_n1.json 2> gpurun_out/${TAG}_bench_client_shard_n1.err || exit 1
if [ "${PROFILE:-0}" = 1 ]; then
  timeout -k 10 900 bash tools/profile_round.sh ${TAG} c3 c2 c4 c5 > gpurun_out/${TAG}_profile.log 2>&1
fi
