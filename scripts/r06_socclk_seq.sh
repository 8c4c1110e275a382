# Round 6: the SOC clock across a sequence of GPU processes, sampled by a process that does no
# HIP work (tools/socclk_trace.py, in the background for a fixed time): predecessors holding
# 91, 45 and 8 GiB and one holding none, 5 s apart, then two C5 probes back to back.  Does the
# high-SOC-clock window after a process exits (and C5's step inside it) scale with the memory
# the process held -- the driver clearing freed VRAM -- or not?
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06s}
mkdir -p gpurun_out
timeout -k 5 100 python3 -u tools/socclk_trace.py --seconds 85 --out gpurun_out/${T}_trace.json > gpurun_out/${T}_trace.log 2>&1 &
SAMPLER=$!
sleep 3
for g in 91 45 8 0 91; do
  timeout -k 10 120 python3 -u tools/alloc_exit.py --gib $g >> gpurun_out/${T}_pred.jsonl 2>> gpurun_out/${T}_pred.err || { kill $SAMPLER; exit 1; }
  echo "{\"exited\": $(date +%s.%N)}" >> gpurun_out/${T}_pred.jsonl
  sleep 5
done
timeout -k 10 120 python3 -u tools/c5_step_probe.py --no-sync-after-synth --no-sampler --first 120 --second 0 --fresh 0 \
  --old 0 --out gpurun_out/${T}_c1.json > gpurun_out/${T}_c1.log 2>&1 || { kill $SAMPLER; exit 1; }
echo "{\"exited\": $(date +%s.%N)}" >> gpurun_out/${T}_pred.jsonl
timeout -k 10 120 python3 -u tools/c5_step_probe.py --no-sync-after-synth --no-sampler --first 120 --second 0 --fresh 0 \
  --old 0 --out gpurun_out/${T}_c2.json > gpurun_out/${T}_c2.log 2>&1 || { kill $SAMPLER; exit 1; }
wait $SAMPLER
