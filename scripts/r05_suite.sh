# The round's product library: the whole GPU suite (push executor first) and smoke().
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u -m pytest tests/test_push_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05e_push_tests.log 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_push_gpu.py > gpurun_out/r05e_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05e_smoke.log 2>&1
