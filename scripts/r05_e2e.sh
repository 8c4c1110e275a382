# The drop-in's host paths on the round's final library: subprocess-mode aggregate tasks (fresh
# process per task) and the in-process engine call, beside the reference's NumPy sequence.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r05ak}
timeout -k 10 300 python3 -u tests/perf/task_probe.py --K 8 --M 25000000 --reps 3 > gpurun_out/${T}_task_c2.jsonl 2>&1 &&
timeout -k 10 300 python3 -u tests/perf/task_probe.py --K 16 --M 25000000 --reps 3 --strategy scaffold > gpurun_out/${T}_task_scaffold_c4.jsonl 2>&1 &&
timeout -k 10 300 python3 -u tests/perf/e2e_bench.py --K 8 --M 25000000 --reps 3 > gpurun_out/${T}_e2e_c2.jsonl 2>&1
