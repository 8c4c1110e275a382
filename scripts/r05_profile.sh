# The evidence set on the round's product library: PMC traffic, bench lines, rocprof kernel stats
# and roofline checks for every workload (tools/profile_round.sh).
set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/profile_round.sh ${1:-r05e} c3 c2 c4 c5 > gpurun_out/${1:-r05e}_profile.log 2>&1
