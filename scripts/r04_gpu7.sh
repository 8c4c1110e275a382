# Scaffold on the push executor (new kernels + the multi-process cases), then the whole GPU suite,
# smoke and the default bench line on this build.
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u -m pytest tests/test_push_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_push_tests.log 2>&1 &&
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_push_gpu.py > gpurun_out/r04b_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04b_smoke.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04b_bench_default.json 2> gpurun_out/r04b_bench_default.err
