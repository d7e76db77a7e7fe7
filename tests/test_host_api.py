"""The host mirror keeps the reference's argument checks and error behaviour (no GPU)."""
import numpy as np
import pytest


def test_msm_dimension_mismatch(zk):
    with pytest.raises(ValueError, match="msm: incompatible array dimensions"):
        zk.msm("bls12_381", np.zeros((3, 4), np.uint64), np.zeros((4, 12), np.uint64))


def test_ntt_size_mismatch(zk):
    sg = zk.get_fft_subgroup("bn128", 3)
    with pytest.raises(ValueError, match="forwardNTT: subgroup size differs"):
        zk.forward_ntt(sg, np.zeros((4, 4), np.uint64))
    with pytest.raises(ValueError, match="inverseNTT: subgroup size differs"):
        zk.inverse_ntt(sg, np.zeros((16, 4), np.uint64))


def test_subgroup_too_large(zk):
    with pytest.raises(ValueError):
        zk.get_fft_subgroup("bn128", 29)


def test_gpu_only_no_fallback(zk, monkeypatch):
    monkeypatch.setattr(zk, "device_count", lambda: 0)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        zk.msm("bn128", np.zeros((1, 4), np.uint64), np.zeros((1, 8), np.uint64))
