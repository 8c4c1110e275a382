# Round 6: round 6's one --pmc pass over tools/alloc_probe.hip again, now with 8 s of idle before
# the first allocation and after each free (r06d's pass ran right after the plain probe, inside the
# driver's clear of the VRAM that run freed): translation, memory-side read concurrency and clock
# for the first buffer, the second co-resident one, and the ones allocated after the frees.
set -o pipefail
T=${1:-r06v}
ROOT=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_THRASHING_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT \
  --kernel-trace --output-format csv -d "$ROOT/gpurun_out/${T}_pmc_alloc" -o run -- "$ROOT/tools/_alloc_probe" 8 8 > "$ROOT/gpurun_out/${T}_pmc_alloc_probe.jsonl" 2> "$ROOT/gpurun_out/${T}_pmc_alloc_probe.err"
