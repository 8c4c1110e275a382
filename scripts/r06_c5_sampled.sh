# Round 6: the C5 sustained-load step with the power-management state sampled every 2 ms (every
# gpu_metrics field the probe knows, raw samples kept): six processes with their launches queued
# right behind the synthesis, bench.py's order, where the step shows up.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06q}
mkdir -p gpurun_out
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python3 -u tools/c5_step_probe.py --no-sync-after-synth --first 90 --second 0 --fresh 0 --old 0 \
    --out gpurun_out/${T}_p$i.json > gpurun_out/${T}_p$i.log 2>&1 || exit $?
done
