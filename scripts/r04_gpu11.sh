# The experiment-variant tests against a fresh FEDAGG_TUNING build of the current fedagg.hip.
set -o pipefail
export PYTHONUNBUFFERED=1
FEDAGG_LIB=substrafl_amd/libfedagg_tuning.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m "gpu and tuning" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04e_tuning_build_variant_tests.log 2>&1
