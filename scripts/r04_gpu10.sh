# Every N > 1 leg forced at the driver's default workload (C3) on one GPU: the legs' plumbing,
# deadlines and output checksums at full size, timed end to end.
set -o pipefail
export PYTHONUNBUFFERED=1
start=$(date +%s)
timeout -k 10 900 python3 -u bench.py --client-shard force --multi-device-leg force > gpurun_out/r04e_bench_legs_forced_c3_n1.json 2> gpurun_out/r04e_bench_legs_forced_c3_n1.err
echo "wall_s $(( $(date +%s) - start ))" >> gpurun_out/r04e_bench_legs_forced_c3_n1.err
