"""Host-side sanitizer job for the native index math ("ASan build ... in a
debug test job").  GPU AddressSanitizer is not available on the MI355X pool, so the index
helpers every persistent kernel uses (csrc/persist_common.h: fragment-tiled hand-off layout,
block -> tile mapping) are compiled __host__ __device__ and checked on the CPU with the host
half built under ASan + UBSan (`hipcc -Xarch_host -fsanitize=...`).  Runs without a GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_layout_index_math_under_asan_ubsan(tmp_path):
    exe = tmp_path / "layout_check"
    cmd = [HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=all", "-Xarch_host", "-fno-omit-frame-pointer",
           "-I", os.path.join(ROOT, "csrc"),
           os.path.join(ROOT, "tests", "native", "layout_check.hip"), "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "layout checks ok" in r.stdout
