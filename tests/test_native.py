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


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_safegcd_inverse(tmp_path):
    """zk_inv.hpp (the device inversion by Bernstein-Yang divsteps, compiled here for the CPU) against
    Python's pow(x, -1, p) on all four fields, both limb forms (62-bit limbs with 62-step batches:
    0, 1, 2, p - 1 and 1996 random values; 60-bit limbs with 2 x 30-step batches, the device default:
    the same four and 996 random values)"""
    exe = str(tmp_path / "test_safegcd")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", CSRC,
                           os.path.join(ROOT, "tests", "native", "test_safegcd.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, check=True).stdout.split("\n")
    P = {"bls12_381_fp": 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab,
         "bls12_381_fr": 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
         "bn128_fp": 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47,
         "bn128_fr": 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001}
    seen = {k: 0 for k in P}
    for line in out:
        if not line.strip():
            continue
        f, x, y = line.split()
        x, y, p = int(x, 16), int(y, 16), P[f]
        assert y == (pow(x, -1, p) if x else 0), (f, hex(x))
        seen[f] += 1
    assert all(v == 3000 for v in seen.values()), seen
