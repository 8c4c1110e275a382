# accelerate_algo client round: per-round times, then the per-phase breakdown (synchronised phases).
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r05i}
timeout -k 10 300 python3 -u tools/accelerate_algo_bench.py --params 25000000 --layers 24 --rounds 10 > gpurun_out/${T}_accel_bench_25M.jsonl 2>&1 &&
timeout -k 10 300 python3 -u tools/accelerate_algo_bench.py --params 25000000 --layers 24 --rounds 10 --breakdown > gpurun_out/${T}_accel_breakdown_25M.jsonl 2>&1 &&
timeout -k 10 400 python3 -u tools/accelerate_algo_bench.py --params 200000000 --layers 200 --rounds 5 --breakdown > gpurun_out/${T}_accel_breakdown_200M.jsonl 2>&1
