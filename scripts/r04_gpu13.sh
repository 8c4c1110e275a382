# The gather leg's pipelined variant: the bench GPU test of the forced legs, then every leg at C3.
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u -m pytest tests/test_bench_gpu.py -x -v -k "n_gt_1_legs" --timeout 450 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_bench_legs_test.log 2>&1 &&
bash scripts/r04_gpu10.sh
