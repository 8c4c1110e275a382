# Round 6, the final tree (bench.py's wait for the driver's clear, its tests): the whole GPU suite
# on the final library, the push executor's tests first in their own process, then smoke().
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06y}
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_push_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_push_tests.log 2>&1 &&
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_push_gpu.py > gpurun_out/${T}_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
