"""The recoverable error mode (zkg_set_error_mode(1), zkg_last_error): a failing call returns
instead of aborting the caller's process -- a GHC program keeps running after a transient device
error -- and the library keeps working afterwards.  (The default mode aborts like the
reference's asserts, bls12_381_G1_proj.c:518,632; that path is not exercised here.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def recoverable(gpu):
    gpu.set_error_mode(True)
    assert gpu.last_error() is None
    yield gpu
    gpu.set_error_mode(False)
    gpu.arena_set_limit(0)
    gpu.last_error()


def test_bad_device_and_oversized_alloc(recoverable, oracle):
    zk = recoverable
    zk.load().zkg_set_device(zk.device_count() + 7)
    assert zk.last_error() is not None
    assert zk.last_error() is None  # cleared once read
    assert zk.load().zkg_device_malloc(1 << 52) is None  # 4 PiB: refused, NULL returned
    assert zk.last_error() is not None
    zk.load().zkg_set_device(0)
    sc, pts = zk.gen_fr("bn128", 5, 300), zk.gen_points("bn128", 6, 300)
    assert np.array_equal(zk.msm_affine("bn128", sc, pts), oracle.msm("bn128", sc, pts, mont=True))
    assert zk.last_error() is None


@pytest.mark.parametrize("curve", ["bn128", "bls12_381"])
def test_msm_working_set_refused_then_recovers(recoverable, oracle, curve):
    """an arena cap below one window's working set: the MSM reports an error and returns (it used
    to abort the process); with the cap lifted the same call succeeds, bit-exact"""
    zk = recoverable
    n = 1 << 17  # host inputs: the split pipeline with its copy thread
    sc, pts = zk.gen_fr(curve, 11, n), zk.gen_points(curve, 12, n)
    zk.release()
    zk.arena_set_limit(1 << 20)
    zk.msm_affine(curve, sc, pts)
    msg = zk.last_error()
    assert msg is not None and "memory" in msg
    zk.arena_set_limit(0)
    got = zk.msm_affine(curve, sc[:4096].copy(), pts[:4096].copy())
    assert zk.last_error() is None
    assert np.array_equal(got, oracle.msm(curve, sc[:4096].copy(), pts[:4096].copy(), mont=True))
