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


_COMM = []


@pytest.fixture(scope="session")
def comm(zk):
    """the library's own RCCL communicator, world 1 (sharded.LibComm), shared by the session:
    the process layout of bench.py --gpus N (one HIP runtime, no torch, a live communicator)"""
    if not _COMM:
        from sharded import LibComm
        os.environ.setdefault("ZKG_RDZV_KEY", f"pytest_{os.getpid()}")
        zk.load().zkg_set_device(0)
        _COMM.append(LibComm(0, 1))
    yield _COMM[0]


@pytest.fixture(scope="session")
def gpu(zk, request):
    if zk.device_count() < 1:
        pytest.fail("GPU test ran without a visible GPU")
    if os.environ.get("ZKG_TEST_COMM") == "1":  # run every GPU test beside a live communicator
        request.getfixturevalue("comm")
    return zk


def pytest_sessionfinish(session, exitstatus):
    while _COMM:
        _COMM.pop().close()
