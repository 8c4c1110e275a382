set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -k "equal_count or scaffold" --timeout 120 --timeout-method thread > gpurun_out/eq.log 2>&1 || { tail -30 gpurun_out/eq.log; exit 1; }
tail -2 gpurun_out/eq.log
timeout -k 10 300 python tools/tune_scaffold.py --K 16 --M 25000000 > gpurun_out/tune6_c4.log 2>&1 || exit $?
grep -h equal_count gpurun_out/tune6_c4.log
echo done
