# Round 6: is C5's in-process step (1.7-2.4 % over the first ~0.4 s of launches, seen in bench.py
# processes of the profiling sessions, not in the probes) the previous process's released 91 GB?
# C5 processes back to back: p1 first (nothing large freed before it), p2 right after p1 (which
# freed 91 GB), p3 after 30 s idle, p4 = the plain bench line right after p3, p5 right after p4.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06h}
mkdir -p gpurun_out
P() { timeout -k 10 300 python3 -u tools/c5_step_probe.py --no-sampler --first 100 --second 0 --fresh 0 --old 0 \
        --out gpurun_out/${T}_$1.json > gpurun_out/${T}_$1.log 2>&1; }
stamp() { echo "$1 $(date +%s.%N)" >> gpurun_out/${T}_times.txt; }
stamp start && P p1 && stamp p1_end && P p2 && stamp p2_end && sleep 30 && stamp idle_end && P p3 && stamp p3_end &&
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_p4_bench_c5.json 2> gpurun_out/${T}_p4_bench_c5.err &&
stamp p4_end && P p5 && stamp p5_end
