"""bench.py's JSON contract on the GPU (small step counts): the fields the driver and the judge read,
the parity spot check, the roofline block with its PMC-traffic provenance, and the other modes
(client-shard on one rank, strong scaling with two ranks sharing the GPU, the one-process
multi-device engine)."""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def _bench(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, env=env,
                       timeout=timeout, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_default_line_fields():
    line = _bench("--workload", "c2", "--steps", "5", "--warmup", "2", "--cpu-seconds", "1")
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in line
    assert line["n_gpus"] == 1 and line["steps"] == 5 and line["unit"] == "GB/s" and line["value"] > 0
    assert line["config"]["workload"] == "fedavg_fp32_8x25M"
    roof = line["roofline"]
    assert roof["bound"] == "hbm" and roof["peak"] == 8000.0 and 0 < roof["frac"] < 1
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    assert roof["traffic_source"] is None or "same_build" in roof["traffic_source"]
    # best of the grid-strided and tile-walk read probes over the same buffer
    assert roof["read_stream_ceiling_GBps"] > 1000 and 0.5 < roof["frac_of_read_ceiling"] < 1.1
    assert line["cpu_baseline"]["cores"] == 1 and line["cpu_baseline"]["kind"] == "port"
    assert line["parity"]["mismatches"] == 0


def test_scaffold_line():
    line = _bench("--workload", "c4", "--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    assert line["dtype"] == "f32-in/f64-acc" and line["parity"]["mismatches"] == 0
    assert line["roofline"]["kernel"].startswith("scaffold_bucket_kernel<float> x2")  # 16 clients: one bucket per launch


@pytest.mark.parametrize("combine", ["striped", "relay"])
def test_client_shard_single_rank(combine):
    """--mode client-shard on one rank: the lockstep schedule's runs with no exchange, spot-checked
    bit-exact, its block-kernel time and the single-GPU reference reported."""
    line = _bench("--workload", "c2", "--mode", "client-shard", "--combine", combine, "--steps", "3", "--warmup", "1",
                  "--no-cpu-baseline")
    assert line["parity"]["mismatches"] == 0 and line["config"]["clients_per_gpu"] == 8
    cs = line["client_shard"]
    assert cs["combine"] == combine and cs["block_kernel_ms"] > 0 and cs["single_gpu_ms"] > 0
    assert cs["bit_exact_by_construction"] and 0 < cs["weak_efficiency"] < 1.5


def test_shared_gpu_ranks_skip_the_client_shard_leg():
    """Two ranks sharing the one GPU of a test box: the parameter-range line is measured, the
    client-shard leg (RCCL needs a GPU per rank) is reported as skipped."""
    line = _bench("--workload", "c2", "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    assert line["n_gpus"] == 2 and "skipped" in line["client_shard"]
    assert line["process_group"]["timeout_s"] > 0


def test_shared_gpu_ranks_push_leg_forced():
    """Two ranks sharing the GPU, legs forced: the push leg runs (IPC between the rank processes,
    landing tags), bit-exact on its spot check, with no late tag and no wait error; its full
    comparison against the native executor is reported as skipped (RCCL refuses two ranks on one
    GPU) instead of failing the leg."""
    line = _bench("--workload", "c2", "--gpus", "2", "--client-shard", "force", "--multi-device-leg", "off",
                  "--steps", "3", "--warmup", "1", "--client-shard-steps", "3", "--no-cpu-baseline", timeout=400)
    push = line["client_shard_push"]
    assert "error" not in push, push
    assert push["parity"]["mismatches"] == 0 and push["wait_errors"] == {}
    assert "skipped" in push["full_compare"]


def test_shared_gpu_ranks_scaffold_push_leg_forced():
    """The same for Scaffold (c4): the push leg runs its two fp64 accumulators per element
    (delta and control-variate launches per run), spot-checked bit-exact, no wait error."""
    line = _bench("--workload", "c4", "--gpus", "2", "--client-shard", "force", "--multi-device-leg", "off",
                  "--steps", "3", "--warmup", "1", "--client-shard-steps", "3", "--no-cpu-baseline", timeout=400)
    push = line["client_shard_push"]
    assert "error" not in push, push
    assert push["parity"]["mismatches"] == 0 and push["wait_errors"] == {}
    assert "skipped" in push["full_compare"]


def test_strong_scaling_two_ranks_shared_gpu():
    line = _bench("--workload", "c2", "--scaling", "strong", "--gpus", "2", "--steps", "3", "--warmup", "1",
                  "--no-cpu-baseline")
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["global_params"] == 25_000_000
    assert line["config"]["params_per_gpu"] < 25_000_000
    assert line["config"]["bytes_alg_per_step_job"] == 8 * 25_000_000 * 4 + 25_000_000 * 4


def test_multi_device_engine_line():
    line = _bench("--engine", "multi-device", "--workload", "c2", "--gpus", "2", "--steps", "2", "--warmup", "1")
    assert line["n_gpus"] == 2 and len(line["shards"]) == 2
    assert all(s["kernel_ms"] > 0 for s in line["shards"])


def test_tiled_layout_line():
    """--layout tiles (c2: the few-client tile) and the default auto (c2: rows, below the
    recommended shape): both parity-clean, the layout named in the config."""
    tiles = _bench("--workload", "c2", "--layout", "tiles", "--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    assert tiles["parity"]["mismatches"] == 0
    assert tiles["config"]["layout"].startswith("tile-interleaved (2048")
    auto = _bench("--workload", "c2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    assert auto["config"]["layout"] == "rows"


def test_default_workload_line():
    """The driver's own command shape on the default workload (C3, tile-interleaved buckets)."""
    line = _bench("--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    assert line["config"]["workload"] == "fedavg_fp32_64x125M"
    assert line["config"]["layout"].startswith("tile-interleaved (8192")
    assert line["parity"]["mismatches"] == 0 and 0.5 < line["roofline"]["frac"] < 1


def test_n_gt_1_legs_rehearsed_on_one_gpu():
    """The legs an N > 1 line carries (client-shard weak with the native and the torch executor
    and with RCCL's copy-engine P2P path, client-shard strong, the one-process multi-device engine), forced at N = 1: each runs in its
    child process through the same spawn / deadline / JSON plumbing and reports without error,
    bit-exact on its spot check."""
    line = _bench("--workload", "c2", "--client-shard", "force", "--multi-device-leg", "force", "--steps", "5",
                  "--warmup", "2", "--client-shard-steps", "5", "--no-cpu-baseline", timeout=400)
    for key, scaling, executor in (("client_shard", "weak", "native"), ("client_shard_torch_pg", "weak", "torch"),
                                   ("client_shard_copy_engine", "weak", "native"),
                                   ("client_shard_strong", "strong", "native")):
        leg = line[key]
        assert "error" not in leg, leg
        assert leg["scaling"] == scaling and leg["executor"] == executor and leg["parity"]["mismatches"] == 0
        assert leg["ms_per_step"] > 0 and leg["wall_s"] > 0
    assert line["client_shard"]["weak_efficiency"] > 0 and line["client_shard_strong"]["speedup"] > 0
    assert line["client_shard_copy_engine"]["env"] == {"NCCL_P2P_USE_CUDA_MEMCPY": "1"}
    variants = line["client_shard"]["rounds_variants"]  # the other round splits, same communicator
    assert [v["rounds"] for v in variants] == [[1.0], [0.75, 0.25]], variants
    assert all("error" not in v and v["ms_per_step"] > 0 for v in variants), variants
    md = line["multi_device"]
    assert "error" not in md and md["value"] > 0 and md["n_gpus"] == 1
    assert line["legs_order"][:3] == ["client_shard_push", "client_shard", "param_range_strong_gather"]
    push = line["client_shard_push"]  # one rank: no peers, so the leg's plumbing only (no transport)
    assert "error" not in push, push
    assert push["executor"] == "push" and push["parity"]["mismatches"] == 0
    # (one rank: the legs run over the loopback transport; ncclCommCount / late tags / the full
    # comparison are N > 1 fields -- rehearsed over gloo in tests/test_bench_launcher.py)
    # every weak leg reduced the same (client, element) values: one output, whatever the executor
    sums = line["client_shard_output_checksums"]
    assert sums["agree"] is True and {"client_shard", "client_shard_push", "client_shard_torch_pg"} <= set(sums["legs"])
    assert all(v["output_matches_leg"] is True for v in variants), variants
    g = line["param_range_strong_gather"]  # C3 as written, here on one rank (no gather)
    assert "error" not in g, g
    assert g["parity"] == {"sampled_per_rank": 1024, "mismatches": 0, "gathered_slice_checksum_mismatches": 0}
    assert g["kernel_ms"] > 0 and g["speedup"] > 0 and g["params_per_gpu"] >= 25_000_000
    pipe = g["pipelined"]  # chunked kernels (no gather at one rank), same result
    assert "error" not in pipe and pipe["chunks"] == 4 and pipe["gathered_slice_checksum_mismatches"] == 0
    assert pipe["ms_per_step"] > 0 and pipe["speedup"] > 0
