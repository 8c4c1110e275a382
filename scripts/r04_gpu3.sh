# C4 write-burst probe, then the whole GPU suite on this build (product library), then smoke.
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 240 ./tools/_scaffold_burst_probe 25000000 30 > gpurun_out/r04_scaffold_burst_probe.log 2>&1 &&
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1
