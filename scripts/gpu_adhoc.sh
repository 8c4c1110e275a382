set -u
FILES=tests bash scripts/gpu_check.sh || exit $?
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_scaffold.py --K 16 --M 25000000 > gpurun_out/sc82_c4.log 2>&1 || exit $?
timeout -k 10 300 python tools/tune_fedavg.py --K 16 --M 125000000 --rounds 3 --iters 5 > gpurun_out/vpt16_k16.log 2>&1 || exit $?
timeout -k 10 300 python tools/tune_fedavg.py --K 32 --M 125000000 --rounds 3 --iters 5 > gpurun_out/vpt16_k32.log 2>&1 || exit $?
for wl in c3 c5; do timeout -k 10 600 python bench.py --workload $wl --steps 20 --warmup 5 > gpurun_out/bench_$wl.log 2>&1 || exit $?; done
grep -h GBps gpurun_out/sc82_c4.log | head -4; grep -h '"vpt"' gpurun_out/vpt16_k16.log | head -3; grep -h '"vpt"' gpurun_out/vpt16_k32.log | head -3
grep -h metric gpurun_out/bench_c*.log | cut -c1-60,400-900
