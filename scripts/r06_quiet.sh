# Round 6: bench.py right after a process that held 91 GB (the driver still clearing it), without
# and with the wait for the clear (wait_device_quiet), C5 then the no-flag line.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06t}
mkdir -p gpurun_out
B() { timeout -k 10 120 python3 -u tools/alloc_exit.py --gib 91 >> gpurun_out/${T}_pred.jsonl && \
      timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "${@:2}" > gpurun_out/${T}_$1.json 2> gpurun_out/${T}_$1.err; }
B c5_nowait --workload c5 --steps 60 --warmup 2 --no-wait-quiet && \
B c5_wait --workload c5 --steps 60 --warmup 2 && \
B default_nowait --no-wait-quiet && \
B default_wait
