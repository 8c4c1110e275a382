# Round 6: does C5's kernel time depend on which allocation it reads (tools/alloc_probe.hip: two
# hipMalloc'd 90 GB buffers held together, a physically contiguous one, one after the frees), and
# the ONE --pmc pass of C5 (VERDICT r05 "Next 2") over the same process: address translation
# (UTCL1 misses, thrashing stalls), memory-side read latency (TCC_EA0_RDREQ_LEVEL / RDREQ) and the
# effective clock (GRBM_GUI_ACTIVE / GRBM_COUNT) per launch.
set -o pipefail
T=${1:-r06d}
ROOT=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 ./tools/_alloc_probe 30 > gpurun_out/${T}_alloc_probe.jsonl 2> gpurun_out/${T}_alloc_probe.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_THRASHING_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT \
  --kernel-trace --output-format csv -d "$ROOT/gpurun_out/${T}_pmc_alloc" -o run -- "$ROOT/tools/_alloc_probe" 8 > "$ROOT/gpurun_out/${T}_pmc_alloc_probe.jsonl" 2> "$ROOT/gpurun_out/${T}_pmc_alloc_probe.err"
