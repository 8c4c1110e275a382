# Round-end check of the final tree: the whole GPU suite, smoke, the default bench line.
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04f_bench_default.json 2> gpurun_out/r04f_bench_default.err
