set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u tools/stream_order_probe.py > gpurun_out/r04_stream_order.jsonl 2> gpurun_out/r04_stream_order.err &&
timeout -k 10 300 python3 -u -m pytest tests/test_push_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r04_push_gpu.log 2>&1 &&
timeout -k 10 200 python3 -u tools/push_overhead_probe.py --n 3900000 --clients 65 > gpurun_out/r04_push_overhead.jsonl 2>&1 &&
timeout -k 10 200 python3 -u tools/push_overhead_probe.py --n 1600000 --clients 65 --push-runs >> gpurun_out/r04_push_overhead.jsonl 2>&1 &&
timeout -k 10 200 python3 -u tools/push_overhead_probe.py --n 7800000 --clients 9 --steps 16 >> gpurun_out/r04_push_overhead.jsonl 2>&1 &&
timeout -k 10 200 python3 -u tools/push_overhead_probe.py --n 62500000 --clients 65 --steps 4 --push-runs >> gpurun_out/r04_push_overhead.jsonl 2>&1
