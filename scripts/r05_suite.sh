# The round's product library: the whole GPU suite (push executor first) and smoke().
# Usage: bash scripts/r05_suite.sh [tag]   (logs under gpurun_out/<tag>_*.log, default r05e)
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r05e}
timeout -k 10 500 python3 -u -m pytest tests/test_push_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_push_tests.log 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_push_gpu.py > gpurun_out/${T}_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
