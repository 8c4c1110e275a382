# Round 6, first GPU session: the tests of this round's changes (the one-call multi-device C entry,
# the staging resolver's named paths, the hand-off's mixed pairings, a push rank that dies
# mid-call), then the C5 launch-step probe, then the task-mode start-up with the prewarm's phases.
# Each step under its own time limit; the first failure ends the script.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06b}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_abi.py tests/test_staging_paths_gpu.py tests/test_handoff.py \
  "tests/test_accelerate_algo.py" > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_push_gpu.py -k "fails_cleanly or memory_flat" > gpurun_out/${T}_push_fault.log 2>&1 &&
timeout -k 10 400 python3 -u tools/c5_step_probe.py --out gpurun_out/${T}_c5_step.json > gpurun_out/${T}_c5_step.log 2>&1 &&
timeout -k 10 300 python3 -u tests/perf/task_probe.py --K 16 --M 25000000 --reps 5 --strategy scaffold > gpurun_out/${T}_task_scaffold_c4.jsonl 2>&1 &&
timeout -k 10 300 python3 -u tests/perf/task_probe.py --K 8 --M 25000000 --reps 3 > gpurun_out/${T}_task_c2.jsonl 2>&1
