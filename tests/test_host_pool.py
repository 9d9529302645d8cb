"""The host thread pool (marshrutka_amd/csrc/mr_pool.hpp) under ThreadSanitizer: many
short jobs back to back, every item run exactly once per job, no data race reported
(tests/cpp/pool_stress.cpp; ADVICE r04's stale-ticket race).  CPU only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_host_pool_tsan(tmp_path):
    exe = str(tmp_path / "pool_stress")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=thread", "-pthread",
                    os.path.join(HERE, "cpp", "pool_stress.cpp"), "-o", exe], check=True)
    env = dict(os.environ, MR_HOST_THREADS="8", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, "4000"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stdout + r.stderr[-4000:]
    assert "bad=0" in r.stdout
