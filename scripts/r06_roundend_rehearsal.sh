# Round 6: the driver's round-end order on one box -- the GPU suite, smoke(), then `python bench.py`
# with no flags -- to see what the default line reads right after the suite's processes (its
# device_quiet: whether the driver was still clearing the suite's freed memory).
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06z}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err
