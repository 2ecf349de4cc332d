"""the framework's host-side native code under AddressSanitizer + UBSan.

GPU sanitizers (xnack+ ASan) are not available on the MI355X pool, so the host code is
checked here: the CPU AdamW core (csrc/cpu/adamw_host.h, the FSDP CPU-offload optimizer) is
compiled with -fsanitize=address,undefined into a standalone harness and run over odd sizes
that exercise every blocking tail."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_adamw_host_asan_ubsan(tmp_path):
    exe = tmp_path / "sanitize_adamw_host"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fopenmp",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           f"-I{os.path.join(ROOT, 'csrc')}", os.path.join(ROOT, "tests", "native", "sanitize_adamw_host.cpp"),
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="4")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout + r.stderr)[-3000:]
