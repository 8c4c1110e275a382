# Round 6, the final product library (one-call multi-device entry with fp16): the push
# executor's suite, the evidence set (tools/profile_round.sh: PMC traffic tagged with this build,
# bench lines, rocprof stats + traces, roofline checks with the per-launch view), the push
# order-kernel cost, the no-flag line, then the rest of the GPU suite and smoke().
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06p}
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_push_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_push_tests.log 2>&1 &&
bash tools/profile_round.sh $T c3 c2 c4 c5 > gpurun_out/${T}_profile.log 2>&1 &&
timeout -k 10 200 python3 -u tools/push_overhead_probe.py --trials 3 > gpurun_out/${T}_push_overhead_probe.jsonl 2>&1 &&
timeout -k 10 300 python3 -u bench.py --traffic gpurun_out/${T}_traffic_c3.json > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err &&
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_push_gpu.py > gpurun_out/${T}_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
