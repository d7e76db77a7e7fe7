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


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_montgomery_arith(tmp_path):
    """zk_host.hpp's portable CIOS product, SOS square, branch-free add / sub and (when the CPU
    has ADX + BMI2) the generated MULX/ADCX/ADOX product (zk_host_adx.inc), against Python
    big integers: a b / 2^(64 N) mod p, a^2 / 2^(64 N) mod p, a + b mod p, a - b mod p."""
    exe = str(tmp_path / "test_host_arith")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", CSRC,
                           os.path.join(ROOT, "tests", "native", "test_host_arith.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, check=True).stdout.split("\n")
    checked = 0
    p = rinv = None
    for line in out:
        f = line.split()
        if not f:
            continue
        if f[0] == "field":
            nw, p = int(f[2]), int(f[3], 16)
            rinv = pow(2 ** (64 * nw), -1, p)
        elif f[0] == "v":
            a, b, m, s, x, y = (int(v, 16) for v in f[1:7])
            assert a < p and b < p
            assert m == a * b * rinv % p
            assert s == a * a * rinv % p
            assert x == (a + b) % p and y == (a - b) % p
            if len(f) > 7:
                assert int(f[7], 16) == m
            checked += 1
    assert checked == 4 * 400
