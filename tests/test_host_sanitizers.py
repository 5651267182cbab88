"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (GPU sanitizers are not
available on the pool, so this covers the host side only): tests/sanitize/host_sanitize.cpp drives the CPU
oracle (every window shape, checkpoint bytes written, restored and re-written, the wire decoder on whole,
cut and corrupt streams) and the engine's host checkpoint codec (flink_amd/csrc/flink_kg_format.h), built
with g++ -fsanitize=address,undefined -fno-sanitize-recover=all.  Any report fails the run."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "host_sanitize")
        cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
               "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
               os.path.join(ROOT, "tests", "sanitize", "host_sanitize.cpp"), os.path.join(ROOT, "oracle", "fw_oracle.cpp"),
               "-lpthread", "-o", exe]
        subprocess.run(cmd, check=True, capture_output=True, timeout=600)
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
        r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        assert "host sanitize driver: ok" in r.stdout
        assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
