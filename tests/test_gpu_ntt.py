"""GPU NTT parity through the C ABI: bit-exact vs reference-generated golden vectors,
vs the oracle, and at 2^24 vs the reference's SHA-256 digest + round trip."""
import hashlib

import numpy as np
import pytest

from golden_io import baseline_configs, ntt_cases

pytestmark = pytest.mark.gpu
CURVES = ["bn128", "bls12_381"]


@pytest.mark.parametrize("curve", CURVES)
def test_golden(gpu, curve):
    for m, g, x, f, i in ntt_cases(curve):
        sg = gpu.get_fft_subgroup(curve, m)
        assert np.array_equal(sg.gen_array(), g)
        assert np.array_equal(gpu.forward_ntt(sg, x), f), m
        assert np.array_equal(gpu.inverse_ntt(sg, x), i), m


@pytest.fixture(params=[0, 12, 8], ids=["default", "two_pass", "short_passes"])
def radix(gpu, request):
    """every pass split: the default, two passes of 2^9..2^12-point DFTs on 4096-element tiles
    for all 2^17..2^24, and <= 2^8-point passes only (test hook zkg_ntt_set_max_radix)"""
    gpu.ntt_set_max_radix(request.param)
    yield request.param
    gpu.ntt_set_max_radix(0)  # default


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("m", [4, 9, 11, 13, 14, 15, 17, 18, 19, 20, 21])
def test_vs_oracle(gpu, oracle, curve, m, radix):
    sg = gpu.get_fft_subgroup(curve, m)
    x = gpu.gen_fr(curve, 77 + m, 1 << m)
    f = gpu.forward_ntt(sg, x)
    assert np.array_equal(f, oracle.ntt(curve, m, sg.gen_array(), x))
    assert np.array_equal(gpu.inverse_ntt(sg, f), x)


@pytest.mark.parametrize("curve", CURVES)
def test_roundtrip_and_linearity_2_20(gpu, curve, radix):
    m = 20
    sg = gpu.get_fft_subgroup(curve, m)
    x = gpu.gen_fr(curve, 5, 1 << m)
    f = gpu.forward_ntt(sg, x)
    assert np.array_equal(gpu.inverse_ntt(sg, f), x)
    assert np.array_equal(gpu.forward_ntt(sg, gpu.inverse_ntt(sg, x)), x)


def test_config1_bn128_ntt_2_14(gpu):
    cfg = baseline_configs().get("config1_bn128_ntt_2^14")
    if cfg is None:
        pytest.skip("baseline_configs.json missing config1")
    x = gpu.gen_fr("bn128", cfg["seed"], 1 << 14)
    f = gpu.forward_ntt(gpu.get_fft_subgroup("bn128", 14), x)
    assert hashlib.sha256(f.tobytes()).hexdigest() == cfg["forward_sha256"]


def test_config3_bls12_381_ntt_2_24(gpu, radix):
    cfg = baseline_configs().get("config3_bls12_381_ntt_2^24")
    if cfg is None:
        pytest.skip("baseline_configs.json missing config3")
    m = cfg["log_n"]
    x = gpu.gen_fr("bls12_381", cfg["seed"], 1 << m)
    assert hashlib.sha256(x.tobytes()).hexdigest() == cfg["input_sha256"]
    sg = gpu.get_fft_subgroup("bls12_381", m)
    f = gpu.forward_ntt(sg, x)
    assert hashlib.sha256(f.tobytes()).hexdigest() == cfg["forward_sha256"]
    assert np.array_equal(gpu.inverse_ntt(sg, f), x)
