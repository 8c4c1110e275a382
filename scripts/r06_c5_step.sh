# C5's launch-duration step (VERDICT r05 "Next 2"): the per-launch probe with the GPU's sampled
# power-management state (tools/c5_step_probe.py), then ONE --pmc pass of the bench's C5 process
# with the effective-clock and read-latency counters (GRBM_GUI_ACTIVE, GRBM_COUNT,
# TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ) beside the kernel trace of the same launches.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06a}
ROOT=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/c5_step_probe.py --out gpurun_out/${T}_c5_step.json > gpurun_out/${T}_c5_step.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum \
  --kernel-trace --output-format csv -d "$ROOT/gpurun_out/${T}_pmc_c5" -o run -- \
  python3 "$ROOT/bench.py" --workload c5 --steps 30 --warmup 10 --no-cpu-baseline > "$ROOT/gpurun_out/${T}_pmc_c5_bench.json" 2> "$ROOT/gpurun_out/${T}_pmc_c5.err"
