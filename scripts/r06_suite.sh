# Round 6: the whole GPU suite on the round's tree (push executor first), smoke(), then the C5
# launch question without the clock sampler (does the polling matter?) and a plain C5 bench line
# over 60 steps (its timed mean against the later per-launch median shows any in-process step).
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06e}
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_push_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_push_tests.log 2>&1 &&
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_push_gpu.py > gpurun_out/${T}_gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 300 python3 -u tools/c5_step_probe.py --no-sampler --out gpurun_out/${T}_c5_step_nosampler.json > gpurun_out/${T}_c5_step_nosampler.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/${T}_bench_c5_60.json 2> gpurun_out/${T}_bench_c5_60.err
