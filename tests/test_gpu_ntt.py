"""GPU NTT parity through the C ABI: bit-exact vs reference-generated golden vectors,
vs the oracle, and at 2^24 vs the reference's SHA-256 digests (forward and inverse) + round
trip; adversarial inputs (tests/golden_io.py NTT_PATTERNS) vs the reference's digests up to
2^20 and vs their closed forms up to 2^26; the on-the-fly twiddle path forced at small sizes."""
import hashlib

import numpy as np
import pytest

from golden_io import (NTT_PATTERNS, baseline_configs, check_pattern_output, ntt_cases, ntt_pattern,
                       ntt_pattern_expected, ntt_patterns_golden)

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


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_config3_inverse_2_24_vs_reference(gpu, radix):
    """the inverse applied to the config-3 input itself, against the reference's digest
    (bls12_381_poly_mont.c:472-522) -- the inverse's own tables (w^-1, 1/N) at full size"""
    cfg = baseline_configs().get("config3_bls12_381_ntt_2^24")
    if cfg is None or "inverse_sha256" not in cfg:
        pytest.skip("baseline_configs.json lacks the config-3 inverse digest")
    m = cfg["log_n"]
    x = gpu.gen_fr("bls12_381", cfg["seed"], 1 << m)
    y = gpu.inverse_ntt(gpu.get_fft_subgroup("bls12_381", m), x)
    assert _sha(y) == cfg["inverse_sha256"]


def _golden_case(curve, name, m, inverse):
    g = ntt_patterns_golden().get("cases", {})
    key = f"{curve}/{name}/m{m}/{'inverse' if inverse else 'forward'}"
    if key not in g:
        pytest.skip(f"tests/golden/ntt_patterns.json lacks {key}")
    return g[key]


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("m", [5, 12, 14, 20])
def test_patterns_vs_reference(gpu, curve, m, radix):
    """adversarial inputs (all r-1, alternating 0 / r-1, deltas, a constant, the largest distinct
    words) against the reference's own forward / inverse digests, under every pass split"""
    sg = gpu.get_fft_subgroup(curve, m)
    for name in NTT_PATTERNS:
        x = ntt_pattern(curve, name, m)
        for inverse in (False, True):
            case = _golden_case(curve, name, m, inverse)
            assert _sha(x) == case["input_sha256"]
            y = gpu.inverse_ntt(sg, x) if inverse else gpu.forward_ntt(sg, x)
            assert _sha(y) == case["sha256"], (name, inverse)


@pytest.mark.parametrize("curve", CURVES)
def test_random_2_20_vs_reference(gpu, curve, radix):
    m = 20
    sg = gpu.get_fft_subgroup(curve, m)
    x = gpu.gen_fr(curve, 0x5A4B0003, 1 << m)
    for inverse in (False, True):
        case = _golden_case(curve, "random", m, inverse)
        assert _sha(x) == case["input_sha256"]
        y = gpu.inverse_ntt(sg, x) if inverse else gpu.forward_ntt(sg, x)
        assert _sha(y) == case["sha256"], inverse


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("m", [22, 24])
def test_patterns_closed_form_large(gpu, curve, m):
    """the patterns with a closed form (constant, deltas, alternating) at full size: the lazy
    butterflies see their extreme limb values in every pass"""
    sg = gpu.get_fft_subgroup(curve, m)
    for name in NTT_PATTERNS:
        if ntt_pattern_expected(curve, name, m, False) is None:
            continue
        x = ntt_pattern(curve, name, m)
        for inverse in (False, True):
            y = gpu.inverse_ntt(sg, x) if inverse else gpu.forward_ntt(sg, x)
            assert check_pattern_output(curve, name, m, inverse, y), (name, inverse)


@pytest.fixture
def otf(gpu):
    """every non-last pass computes its inter-pass twiddles on the fly (zkg_ntt_set_table_max), the
    path transforms of 2^26 and more take, and the inverse's 1/N moves to the last pass"""
    gpu.ntt_set_table_max(1)
    yield
    gpu.ntt_set_table_max(0)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("m", [13, 17, 20])
def test_otf_twiddles_vs_oracle(gpu, oracle, curve, m, radix, otf):
    sg = gpu.get_fft_subgroup(curve, m)
    x = gpu.gen_fr(curve, 0x5A4B0003 if m == 20 else 90 + m, 1 << m)
    f = gpu.forward_ntt(sg, x)
    i = gpu.inverse_ntt(sg, x)
    if m == 20:  # against the reference's digests
        assert _sha(f) == _golden_case(curve, "random", m, False)["sha256"]
        assert _sha(i) == _golden_case(curve, "random", m, True)["sha256"]
    else:
        assert np.array_equal(f, oracle.ntt(curve, m, sg.gen_array(), x))
    assert np.array_equal(gpu.inverse_ntt(sg, f), x)
    assert np.array_equal(gpu.forward_ntt(sg, i), x)
    for name in ("all_rm1", "alt_0_rm1", "delta_rm1"):
        p = ntt_pattern(curve, name, m)
        for inverse in (False, True):
            y = gpu.inverse_ntt(sg, p) if inverse else gpu.forward_ntt(sg, p)
            assert check_pattern_output(curve, name, m, inverse, y), (name, inverse)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("m", [25, 26])
def test_large_sizes_properties(gpu, curve, m):
    """2^25 (four passes, tables) and 2^26 (pass 0 on the fly: its table would be 2 GiB) --
    above the reference's limit (its scratch size overflows an int at m >= 25, poly.c:459):
    round trip both ways, linearity NTT(x + y) = NTT(x) + NTT(y), and the closed forms of the
    delta / constant / alternating patterns"""
    sg = gpu.get_fft_subgroup(curve, m)
    n = 1 << m
    x = gpu.gen_fr(curve, 0x5A4B0025 + m, n)
    y = gpu.gen_fr(curve, 0x5A4B0035 + m, n)
    fx = gpu.forward_ntt(sg, x)
    assert np.array_equal(gpu.inverse_ntt(sg, fx), x)
    fy = gpu.forward_ntt(sg, y)
    assert np.array_equal(gpu.forward_ntt(sg, gpu.arr_add(curve, x, y)), gpu.arr_add(curve, fx, fy))
    del fx, fy
    assert np.array_equal(gpu.forward_ntt(sg, gpu.inverse_ntt(sg, y)), y)
    del x, y
    for name in ("delta_one", "constant", "alt_0_rm1"):
        p = ntt_pattern(curve, name, m)
        for inverse in (False, True):
            out = gpu.inverse_ntt(sg, p) if inverse else gpu.forward_ntt(sg, p)
            assert check_pattern_output(curve, name, m, inverse, out), (name, inverse)
