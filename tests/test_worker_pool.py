"""The runtime's host worker pool (scanner_colmap_amd/csrc/scm_pool.h: content
hashing and upload staging of the drop-in path, scm_runtime.cpp) under
ThreadSanitizer: a job ends with its last task while late workers may still
be waking, and jobs alternate between two slots (tests/pool_stress.cc).  CPU
only; skipped when the compiler cannot build with -fsanitize=thread."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "scanner_colmap_amd", "csrc")


def test_worker_pool_tsan(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "pool_stress"
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I", CSRC,
                        os.path.join(HERE, "pool_stress.cc"), "-o", str(exe), "-lpthread"],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("cannot build with -fsanitize=thread: " + r.stderr[-300:])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([str(exe), "3000"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.strip().endswith("ok")
