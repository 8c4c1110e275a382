# One simulated round end to end at 8 clients x 200M parameters (200 Linear), three paths.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r05u}
timeout -k 10 500 python3 -u tests/perf/simulation_round_bench.py --strategy fedavg --clients 8 --params 200000000 --layers 200 --rounds 3 > gpurun_out/${T}_sim_round_fedavg_200M.jsonl 2>&1 &&
timeout -k 10 600 python3 -u tests/perf/simulation_round_bench.py --strategy scaffold --clients 8 --params 200000000 --layers 200 --rounds 3 > gpurun_out/${T}_sim_round_scaffold_200M.jsonl 2>&1
