# Round 6: tools/alloc_probe.hip again with 8 s of idle before the first allocation and after each
# free (the driver's clear of the freed VRAM over before the next buffer is timed): is the
# per-allocation spread, and the contiguous buffer's time, still there without the clear?
set -o pipefail
T=${1:-r06u}
mkdir -p gpurun_out
timeout -k 10 240 tools/_alloc_probe 30 8 > gpurun_out/${T}_alloc_probe.jsonl 2> gpurun_out/${T}_alloc_probe.err
