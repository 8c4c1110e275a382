# The N = 2 line at the driver's default workload (C3) with both ranks on the one GPU, legs forced:
# the push leg across two rank processes at full size (IPC, landing tags, spot check).
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u bench.py --gpus 2 --client-shard force --multi-device-leg off > gpurun_out/r04f_bench_c3_n2_shared_gpu.json 2> gpurun_out/r04f_bench_c3_n2_shared_gpu.err
