# Round 6: does the C5 step (and the SOC clock's fall that coincides with it, r06q) move with the
# 91 GB allocation or stay at a fixed time from HIP start-up?  Two processes as r06q, then two
# with 1.5 s of idle between HIP start-up and the allocation.  Every process keeps its whole
# sampled clock trace and the wall time of each phase.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06r}
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python3 -u tools/c5_step_probe.py --no-sync-after-synth --first 120 --second 0 --fresh 0 --old 0 \
    --out gpurun_out/${T}_a$i.json > gpurun_out/${T}_a$i.log 2>&1 || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python3 -u tools/c5_step_probe.py --no-sync-after-synth --sleep-before-synth 1.5 --first 120 \
    --second 0 --fresh 0 --old 0 --out gpurun_out/${T}_b$i.json > gpurun_out/${T}_b$i.log 2>&1 || exit $?
done
