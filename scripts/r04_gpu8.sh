# Final build of the round: the GPU suite (push executor first), smoke, then the evidence set
# (tools/profile_round.sh) for every workload on this very library.
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u -m pytest tests/test_push_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d_push_tests.log 2>&1 &&
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_push_gpu.py > gpurun_out/r04d_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04d_smoke.log 2>&1 &&
bash tools/profile_round.sh r04d c3 c2 c4 c5 > gpurun_out/r04d_profile.log 2>&1
