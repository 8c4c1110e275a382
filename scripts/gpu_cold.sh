set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for args in "--mode breakdown" "--mode breakdown" "--mode breakdown --slots 6 --chunk-mib 8" "--mode breakdown --slots 18 --chunk-mib 4" "--mode native" "--mode torch"; do
  timeout -k 10 120 python tools/coldstart_probe.py $args >> gpurun_out/cold_breakdown.log 2>&1 || exit 1
done
cat gpurun_out/cold_breakdown.log | grep '^{'
