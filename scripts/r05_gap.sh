# Host->device staging of one client's update: back to back vs after idle / GPU work / fresh arrays.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r05j}
timeout -k 10 200 python3 -u tools/stage_gap_probe.py --mb 100 --layers 24 > gpurun_out/${T}_stage_gap.jsonl 2>&1 &&
timeout -k 10 200 python3 -u tools/stage_gap_probe.py --mb 200 --layers 24 --dtype float64 >> gpurun_out/${T}_stage_gap.jsonl 2>&1
