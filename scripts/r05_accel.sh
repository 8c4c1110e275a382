# accelerate_algo: its GPU tests, then the client-round bench at 25M / 200M parameters.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r05g}
timeout -k 10 400 python3 -u -m pytest tests/test_accelerate_algo.py tests/test_newton_raphson.py tests/test_client_buckets.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_accel_tests.log 2>&1 &&
timeout -k 10 300 python3 -u tools/accelerate_algo_bench.py --params 25000000 --layers 24 --rounds 8 > gpurun_out/${T}_accel_bench_25M.jsonl 2>&1 &&
timeout -k 10 400 python3 -u tools/accelerate_algo_bench.py --params 200000000 --layers 200 --rounds 5 > gpurun_out/${T}_accel_bench_200M.jsonl 2>&1
