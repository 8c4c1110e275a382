# bf16 push runs: the push executor tests (f32 + bf16 cases, the direct push-run test), the
# client-shard GPU tests, the bench legs forced on one GPU.
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests/test_push_gpu.py tests/test_client_shard_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_push_bf16_tests.log 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests/test_bench_gpu.py -x -v --timeout 450 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_bench_gpu_tests.log 2>&1
