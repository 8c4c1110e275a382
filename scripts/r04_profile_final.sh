# Round-4 final-build evidence (the library the driver benches): PMC traffic, bench line, rocprof
# kernel stats and the roofline cross-check per workload (tools/profile_round.sh).  WL: workloads.
set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/profile_round.sh r04c $WL > gpurun_out/r04c_profile_$(echo $WL | tr " " _).log 2>&1
