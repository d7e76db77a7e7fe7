"""The oracle (our C restatement) is pinned against the reference: bit-exact against the
reference's own compiled C (when present) and against the committed golden vectors that
the reference produced (tools/make_golden.py).  CPU only."""
import numpy as np
import pytest

from golden_io import msm_cases, ntt_cases

CURVES = ["bn128", "bls12_381"]


@pytest.mark.parametrize("curve", CURVES)
def test_oracle_msm_matches_golden(oracle, curve):
    for name, sc, pts, mont, aff, projn in msm_cases(curve):
        got = oracle.msm(curve, sc, pts, mont=mont, out="affine")
        assert np.array_equal(got, aff), name
        gp = oracle.normalize(curve, oracle.msm(curve, sc, pts, mont=mont, out="proj"))
        assert np.array_equal(gp, projn), name


@pytest.mark.parametrize("curve", CURVES)
def test_oracle_ntt_matches_golden(oracle, curve):
    for m, g, x, f, i in ntt_cases(curve):
        assert np.array_equal(oracle.ntt(curve, m, g, x), f), m
        assert np.array_equal(oracle.ntt(curve, m, g, x, inverse=True), i), m
        assert np.array_equal(oracle.ntt(curve, m, g, f, inverse=True), x), m


@pytest.mark.parametrize("curve", CURVES)
def test_oracle_projective_bit_exact_vs_reference(oracle, reference, curve):
    # same operation order as the reference => even the un-normalised projective output agrees
    for name, sc, pts, mont, aff, projn in msm_cases(curve):
        if sc.shape[0] > 1000:
            continue
        assert np.array_equal(oracle.msm(curve, sc, pts, mont=mont, out="proj"),
                              reference.msm(curve, sc, pts, mont=mont, out="proj")), name


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("window", [1, 3, 7, 11, 16])
def test_oracle_variable_window_vs_reference(oracle, reference, zk, curve, window):
    sc = oracle.to_std(1 if curve == "bn128" else 3, zk.gen_fr(curve, 5, 40))
    pts = zk.gen_points(curve, 6, 40)
    assert np.array_equal(oracle.msm(curve, sc, pts, mont=False, out="proj", window=window),
                          reference.msm(curve, sc, pts, mont=False, out="proj", window=window))


@pytest.mark.parametrize("curve", CURVES)
def test_naive_equals_bucket(oracle, zk, curve):
    sc = oracle.to_std(1 if curve == "bn128" else 3, zk.gen_fr(curve, 15, 30))
    pts = zk.gen_points(curve, 16, 30)
    assert np.array_equal(oracle.msm_naive(curve, sc, pts), oracle.msm(curve, sc, pts, mont=False))


@pytest.mark.parametrize("curve", CURVES)
def test_oracle_ntt_patterns_vs_reference_digests(oracle, zk, curve):
    """the oracle's NTT / iNTT on the adversarial inputs (golden_io.NTT_PATTERNS) against the
    reference's own digests (tools/make_golden.py patterns) and the closed forms"""
    import hashlib
    from golden_io import NTT_PATTERNS, check_pattern_output, ntt_pattern, ntt_patterns_golden
    cases = ntt_patterns_golden()["cases"]
    for m in (5, 12, 14):
        g = zk.get_fft_subgroup(curve, m).gen_array()
        for name in NTT_PATTERNS:
            x = ntt_pattern(curve, name, m)
            for inverse in (False, True):
                y = oracle.ntt(curve, m, g, x, inverse=inverse)
                key = f"{curve}/{name}/m{m}/{'inverse' if inverse else 'forward'}"
                assert hashlib.sha256(y.tobytes()).hexdigest() == cases[key]["sha256"], key
                assert check_pattern_output(curve, name, m, inverse, y) in (None, True), key


def test_ntt_pattern_closed_forms_are_pinned():
    """every closed form the GPU tests use at 2^22..2^26 was confirmed by the reference itself
    at m = 5, 12, 14 and 20 when the fixtures were generated"""
    from golden_io import ntt_patterns_golden
    cases = ntt_patterns_golden()["cases"]
    checked = [k for k, v in cases.items() if v["reference_closed_form_ok"] is not None]
    assert len(checked) == 80 and all(cases[k]["reference_closed_form_ok"] for k in checked)
