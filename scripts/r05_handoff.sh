# Simulation-mode device hand-off: its GPU tests, then one simulated round end to end (8 clients).
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r05q}
timeout -k 10 400 python3 -u -m pytest tests/test_accelerate_algo.py tests/test_abi.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_handoff_tests.log 2>&1 &&
timeout -k 10 400 python3 -u tests/perf/simulation_round_bench.py --strategy fedavg --clients 8 --params 25000000 --rounds 5 > gpurun_out/${T}_sim_round_fedavg.jsonl 2>&1 &&
timeout -k 10 400 python3 -u tests/perf/simulation_round_bench.py --strategy scaffold --clients 8 --params 25000000 --rounds 5 > gpurun_out/${T}_sim_round_scaffold.jsonl 2>&1
