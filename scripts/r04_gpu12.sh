# The push probes on the ABI-14 library (tools keep working after the executor's signature change).
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 200 python3 -u tools/push_overhead_probe.py --trials 3 > gpurun_out/r04e_push_overhead_probe.jsonl 2>&1 &&
timeout -k 10 200 python3 -u tools/push_overhead_probe.py --trials 3 --push-runs >> gpurun_out/r04e_push_overhead_probe.jsonl 2>&1 &&
timeout -k 10 300 python3 -u tools/push_tail_probe.py --modes kernel,legacy --reps 1 > gpurun_out/r04e_push_tail_probe.jsonl 2>&1
