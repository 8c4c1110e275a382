# Round 6 evidence set on the round's final product library: PMC traffic, bench lines, rocprof
# kernel stats + traces and roofline checks (first launch, steady state, step) for every workload
# (tools/profile_round.sh), the push executor's per-step order-kernel cost on this tree, and the
# no-flag bench line.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06f}
mkdir -p gpurun_out
bash tools/profile_round.sh $T c3 c2 c4 c5 > gpurun_out/${T}_profile.log 2>&1 &&
timeout -k 10 200 python3 -u tools/push_overhead_probe.py --trials 3 > gpurun_out/${T}_push_overhead_probe.jsonl 2>&1 &&
timeout -k 10 200 python3 -u tools/push_overhead_probe.py --trials 3 --push-runs >> gpurun_out/${T}_push_overhead_probe.jsonl 2>&1 &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err
