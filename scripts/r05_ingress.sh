# Host ingress of the multi-device engine (VERDICT r04 "Next 4"): stage rate vs pack threads
# (C2, C3; unbound / NUMA-bound), the host pack ceiling of P pipelines x T threads (<= 16 CPUs,
# this box's share), and the multi-device bench line with its placement report.
set -o pipefail
export PYTHONUNBUFFERED=1
lscpu > gpurun_out/r05_lscpu.txt 2>&1 || true
cat /sys/bus/pci/devices/*/numa_node > /dev/null 2>&1 || true
timeout -k 10 60 ./tools/_host_pack_probe --configs 1x1,1x2,1x4,1x8,1x16,2x8,4x4,8x2 --mib-per-pipeline 2048 > gpurun_out/r05_host_pack.jsonl
timeout -k 10 60 ./tools/_host_pack_probe --configs 1x16,2x8,4x4,8x2 --mib-per-pipeline 2048 --bind > gpurun_out/r05_host_pack_bind.jsonl
timeout -k 10 400 python3 -u tools/stage_threads_probe.py --workloads c2,c3 --threads 2,4,8,16 > gpurun_out/r05_stage_threads.jsonl
timeout -k 10 200 python3 -u bench.py --engine multi-device --gpus 1 --workload c3 --steps 3 --warmup 1 > gpurun_out/r05_md_c3.json
