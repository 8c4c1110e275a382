# Stability of the push executor: its GPU test file three times in a row on one box (stops at the
# first failure; every run's log kept).
set -o pipefail
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  timeout -k 10 400 python3 -u -m pytest tests/test_push_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_push_stability_$i.log 2>&1 || exit $?
done
