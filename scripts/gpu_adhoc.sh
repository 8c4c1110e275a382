set -u
mkdir -p gpurun_out
FILES=tests SMOKE=1 bash scripts/gpu_check.sh || exit $?
timeout -k 10 300 python tools/tune_fedavg.py --K 8 --M 25000000 --kind f64 > gpurun_out/tune4_f64_k8.log 2>&1 || exit $?
timeout -k 10 300 python tools/tune_scaffold.py --K 64 --M 25000000 --rounds 3 > gpurun_out/tune4_sc_k64.log 2>&1 || exit $?
for f in tune4_f64_k8 tune4_sc_k64; do grep -h '"median_us"' gpurun_out/$f.log | grep -v probe | head -3; done
echo done
