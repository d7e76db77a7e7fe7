import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "zikkurat-algebra_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE-size parity)")


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Oracle
    lib = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"])
    return Oracle()


@pytest.fixture(scope="session")
def reference():
    from oracle.oracle import Reference
    if not Reference.available():
        pytest.skip("oracle/_ref/libzkref.so not built (needs /root/reference at build time)")
    return Reference()


@pytest.fixture(scope="session")
def zk():
    import zkalgebra
    zkalgebra.load()
    return zkalgebra


@pytest.fixture(scope="session")
def gpu(zk):
    if zk.device_count() < 1:
        pytest.fail("GPU test ran without a visible GPU")
    return zk
