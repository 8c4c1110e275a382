# The push executor's GPU tests incl. the seeded random schedules.
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_push_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04e_push_tests.log 2>&1
