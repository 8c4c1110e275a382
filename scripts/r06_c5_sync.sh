# Round 6: the C5 step appears in bench.py processes (launches queued right behind the
# asynchronous synthesis) and not in the probes (which synchronise after it).  Same probe, three
# ways: launches queued behind the synthesis (bench.py's order), synchronised first (the probes'
# order), synchronised and 1 s idle; then the bench line itself.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r06i}
mkdir -p gpurun_out
P() { timeout -k 10 300 python3 -u tools/c5_step_probe.py --no-sampler --first 60 --second 0 --fresh 0 --old 0 \
        --out gpurun_out/${T}_$1.json "${@:2}" > gpurun_out/${T}_$1.log 2>&1; }
P nosync --no-sync-after-synth && P sync && P sleep1 --sleep-after-synth 1.0 && P nosync2 --no-sync-after-synth
