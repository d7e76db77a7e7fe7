"""The product's synthetic-input generator (C++, zk_gen.cpp) equals the oracle's
independent restatement of the same specification.  CPU only."""
import numpy as np
import pytest


@pytest.mark.parametrize("curve", ["bn128", "bls12_381"])
def test_gen_fr_equal(oracle, zk, curve):
    for seed, start, count in [(1, 0, 500), (0x5A4B0002, 12345, 300), (2**63 + 5, 2**40, 10)]:
        assert np.array_equal(zk.gen_fr(curve, seed, count, start), oracle.gen_fr(curve, seed, start, count))


@pytest.mark.parametrize("curve", ["bn128", "bls12_381"])
def test_gen_points_equal(oracle, zk, curve):
    for seed, start, count in [(3, 0, 20), (0x5A4B0002, 4090, 12), (0x5A4B0005, 2**25 + 7, 5)]:
        assert np.array_equal(zk.gen_points(curve, seed, count, start), oracle.gen_points(curve, seed, start, count))


@pytest.mark.parametrize("curve", ["bn128", "bls12_381"])
def test_gen_points_chunking_independent(zk, curve):
    a = zk.gen_points(curve, 9, 9000)
    b = np.concatenate([zk.gen_points(curve, 9, 5000), zk.gen_points(curve, 9, 4000, start=5000)])
    assert np.array_equal(a, b)


@pytest.mark.parametrize("curve", ["bn128", "bls12_381"])
def test_fft_generator(oracle, zk, curve):
    for m in [0, 1, 5, 14, 24]:
        assert np.array_equal(zk.get_fft_subgroup(curve, m).gen_array(), oracle.fft_generator(curve, m))
