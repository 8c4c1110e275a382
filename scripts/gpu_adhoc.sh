set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -k "scaffold_launch_variants" --timeout 120 --timeout-method thread > gpurun_out/lv.log 2>&1 || { tail -30 gpurun_out/lv.log; exit 1; }
tail -1 gpurun_out/lv.log
timeout -k 10 300 python tools/tune_scaffold.py --K 16 --M 25000000 --rounds 5 > gpurun_out/tune8_c4.log 2>&1 || exit $?
grep -h '"median_us"' gpurun_out/tune8_c4.log | grep -v equal_count | head -6 | cut -c1-200
