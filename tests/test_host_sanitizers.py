"""Host-side runtime of libfedagg under g++ sanitizers (race detection): the pack
worker pool, the per-chunk completion flags and the segment-range gather of
substrafl_amd/csrc/host_pool.h, driven like fedagg_session_stage / _fetch drive them
(tests/c/host_pool_test.cpp).  ThreadSanitizer found a real race here (a completion flag
notified after its mutex was released, racing with the flag's destruction); these tests keep it
fixed.  GPU-side sanitizers are not available on the GPU pool; the kernels are pure streaming
maps with no shared mutable state."""

import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "c" / "host_pool_test.cpp"


@pytest.mark.parametrize("flags,env", [
    (["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1:exitcode=66"}),
    (["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
     {"ASAN_OPTIONS": "detect_leaks=1:verify_asan_link_order=0"}),
], ids=["tsan", "asan_ubsan"])
def test_host_pool_under_sanitizer(tmp_path, flags, env):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "host_pool_test"
    subprocess.run([gxx, "-std=c++17", "-O1", "-g", *flags, "-pthread", f"-I{ROOT / 'substrafl_amd' / 'csrc'}",
                    str(SRC), "-o", str(exe)], check=True, capture_output=True, text=True)
    run_env = dict(os.environ)
    run_env.update(env)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=run_env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "host_pool_test: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
