set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -k "launch_variants" --timeout 120 --timeout-method thread > gpurun_out/lv.log 2>&1 || { tail -30 gpurun_out/lv.log; exit 1; }
tail -2 gpurun_out/lv.log
timeout -k 10 300 python tools/tune_fedavg.py --K 8 --M 25000000 > gpurun_out/tune7_c2.log 2>&1 || exit $?
timeout -k 10 300 python tools/tune_fedavg.py --K 64 --M 125000000 --rounds 3 --iters 5 > gpurun_out/tune7_c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/tune_scaffold.py --K 16 --M 25000000 > gpurun_out/tune7_c4.log 2>&1 || exit $?
for f in tune7_c2 tune7_c3 tune7_c4; do echo "== $f"; grep -h '"median_us"' gpurun_out/$f.log | grep -v "probe\|equal_count" | head -4 | cut -c1-220; done
echo done
