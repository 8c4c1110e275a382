# Round 6, second GPU session: the push executor's whole suite (the fail-fast waits now scan the
# peers' error words every 16 polls; no collective after a failed call, a rank that dies mid-call),
# NewtonRaphson's sums over fp16 and mixed client dtypes, then the C5 launch-step probe and the
# task-mode start-up with the prewarm's phases.  Each step under its own limit; the first failure
# ends the script.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06c}
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_push_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_push_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_newton_raphson.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_nr_tests.log 2>&1 &&
timeout -k 10 400 python3 -u tools/c5_step_probe.py --out gpurun_out/${T}_c5_step.json > gpurun_out/${T}_c5_step.log 2>&1 &&
timeout -k 10 300 python3 -u tests/perf/task_probe.py --K 16 --M 25000000 --reps 5 --strategy scaffold > gpurun_out/${T}_task_scaffold_c4.jsonl 2>&1 &&
timeout -k 10 300 python3 -u tests/perf/task_probe.py --K 8 --M 25000000 --reps 3 > gpurun_out/${T}_task_c2.jsonl 2>&1
