"""Host-side native code under ThreadSanitizer (CPU; no GPU needed): the worker pool that
runs the MSM's per-window Horner segments is exercised by several caller threads at once,
as concurrent C-ABI calls from several devices / Haskell capabilities would."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zikkurat-algebra_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_hostpool_tsan(tmp_path):
    exe = str(tmp_path / "test_hostpool")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I", CSRC,
                           os.path.join(ROOT, "tests", "native", "test_hostpool.cpp"),
                           os.path.join(CSRC, "zk_hostpool.cpp"), "-o", exe, "-lpthread"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ThreadSanitizer" not in r.stderr, r.stderr
    assert r.stdout.strip() == "ok"
