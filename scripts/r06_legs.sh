# The N > 1 line's legs on the round-6 tree (each leg now reports its set-up time, connect_s, beside its deadlines): every leg forced at N = 1, then 2 ranks sharing the GPU.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06k}
timeout -k 10 900 python3 -u bench.py --client-shard force --multi-device-leg force > gpurun_out/${T}_bench_legs_forced_c3_n1.json 2> gpurun_out/${T}_bench_legs_forced_c3_n1.err &&
timeout -k 10 900 python3 -u bench.py --gpus 2 --client-shard force --multi-device-leg off > gpurun_out/${T}_bench_c3_n2_shared_gpu.json 2> gpurun_out/${T}_bench_c3_n2_shared_gpu.err
