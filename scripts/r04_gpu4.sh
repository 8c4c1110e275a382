# The GPU suite from where it stopped (bench legs onward), smoke, then the tuning-build variant tests.
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 &&
FEDAGG_LIB=substrafl_amd/libfedagg_tuning.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m "gpu and tuning" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_tuning_build_variant_tests.log 2>&1
