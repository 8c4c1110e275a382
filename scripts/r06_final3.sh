# Round 6, bench.py waiting out the driver's clear of the previous process's freed VRAM before it
# times (device_quiet): the GPU tests that run bench.py, the evidence set again on the same final
# library (tools/profile_round.sh: PMC traffic, bench lines, rocprof stats + traces, roofline
# checks with the per-launch view) and the no-flag line.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06w}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_bench_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_bench_tests.log 2>&1 &&
bash tools/profile_round.sh $T c3 c2 c4 c5 > gpurun_out/${T}_profile.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --traffic gpurun_out/${T}_traffic_c3.json > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err
