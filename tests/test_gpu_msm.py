"""GPU MSM parity through the C ABI: bit-exact against the reference-generated golden
vectors, the oracle, and (at BASELINE sizes) the reference's own outputs."""
import numpy as np
import pytest

from golden_io import baseline_configs, msm_cases

pytestmark = pytest.mark.gpu
CURVES = ["bn128", "bls12_381"]
FR_FLD = {"bn128": 1, "bls12_381": 3}


@pytest.mark.parametrize("curve", CURVES)
def test_golden_affine_and_projective(gpu, curve):
    for name, sc, pts, mont, aff, projn in msm_cases(curve):
        got = gpu.msm_affine(curve, sc, pts, std=not mont)
        assert np.array_equal(got, aff), name
        proj = gpu.msm(curve, sc, pts) if mont else gpu.msm_std(curve, sc, pts)
        assert np.array_equal(proj, projn), name


@pytest.mark.parametrize("curve", CURVES)
def test_golden_jacobian(gpu, reference, curve):
    NP = gpu.NLIMBS_P[curve]
    for name, sc, pts, mont, aff, projn in msm_cases(curve):
        jac = gpu.msm_jac(curve, sc, pts, std=not mont)
        if np.all(aff == np.uint64(0xFFFFFFFFFFFFFFFF)):
            # exactly the reference's Montgomery (1:1:0), G1_jac.c:182-187 (its MSM leaves
            # the set_infinity value untouched when every term is infinity)
            assert np.array_equal(jac, reference.msm_jac(curve, sc, pts, mont=mont)), name
            assert not jac[2 * NP:].any() and np.array_equal(jac[:NP], jac[NP:2 * NP]), name
        else:
            assert np.array_equal(jac[:2 * NP], aff), name          # Z = 1 => (x, y)


@pytest.mark.parametrize("curve", CURVES)
# c = 1..3 and > 24 are clamped into 4..24 by the `_variable` entry (the reference takes 1..64,
# bls12_381_G1_proj.c:509); the result does not depend on the window, so every c must give the same sum
@pytest.mark.parametrize("window", [1, 3, 4, 5, 9, 13, 16, 20, 21, 22, 24, 30, 64])
def test_window_independence(gpu, oracle, curve, window):
    sc = oracle.to_std(FR_FLD[curve], gpu.gen_fr(curve, 31, 3000))
    pts = gpu.gen_points(curve, 32, 3000)
    want = oracle.normalize(curve, oracle.msm(curve, sc, pts, mont=False, out="proj"))
    assert np.array_equal(gpu.msm_variable(curve, sc, pts, window), want)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n", [0, 1, 2, 7, 255, 4097, 65536])
def test_random_sizes_vs_oracle(gpu, oracle, curve, n):
    sc = gpu.gen_fr(curve, 1000 + n, n)
    pts = gpu.gen_points(curve, 2000 + n, n)
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), oracle.msm(curve, sc, pts, mont=True))


@pytest.mark.parametrize("curve", CURVES)
def test_skewed_buckets(gpu, oracle, curve):
    # every scalar equal -> one bucket per window holds all points (chunk stitching)
    n = 20000
    sc = np.tile(gpu.gen_fr(curve, 5, 1), (n, 1))
    pts = gpu.gen_points(curve, 6, n)
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), oracle.msm(curve, sc, pts, mont=True))


@pytest.mark.parametrize("curve", CURVES)
def test_skewed_large_vs_reference(gpu, reference, curve):
    """2^16 pairs drawn from 3 scalars plus zeros: a few buckets per window hold ~n/3
    points each, so the partial-run stitching runs several levels at full chunk size;
    checked against the reference's own C"""
    n = 1 << 16
    rng = np.random.default_rng(77)
    vals = gpu.gen_fr(curve, 78, 3)
    sc = vals[rng.integers(0, 3, n)].copy()
    sc[rng.random(n) < 0.05] = 0
    pts = gpu.gen_points(curve, 79, n)
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), reference.msm(curve, sc, pts, mont=True))


@pytest.mark.parametrize("key", ["skew_mix3_bls12_381_msm_2^22", "skew_binary_bn128_msm_2^22"])
def test_skewed_2_22_sub_bin_sort_vs_reference(gpu, key):
    """2^22 pairs with skewed scalars (three values + zeros, or 0 / 1: a few buckets hold ~n/3 or
    n/2 entries), against the reference's own output (tools/make_golden.py, shards added by the
    reference's proj_add): through the host-buffer entry (split pipelines at c = 16, each split
    sorted in its own list region) and device-resident at c = 20, where the coarse bins (16K
    entries, 2048 fine buckets each) outgrow level 2's LDS staging and the sort runs the sub-bin
    level (k_split)."""
    from golden_io import skew_scalars
    cfg = baseline_configs().get(key)
    if cfg is None:
        pytest.skip(f"{key} missing")
    curve, n = cfg["curve"], 1 << cfg["log_n"]
    sc = skew_scalars(gpu.gen_fr, curve, cfg["seed"], n, cfg["kind"])
    pts = gpu.gen_points(curve, cfg["seed"], n)
    assert [int(x) for x in gpu.msm_affine(curve, sc, pts)] == cfg["affine"]
    ds, dp = gpu.DeviceBuffer(sc), gpu.DeviceBuffer(pts)
    try:
        proj = gpu.msm_device(curve, n, ds, dp, window=20)
    finally:
        ds.free()
        dp.free()
    assert [int(x) for x in gpu.batch_to_affine(curve, proj.reshape(1, -1))[0]] == cfg["affine"]


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("window,logn", [(0, 18), (0, 20), (17, 18)])
def test_binary_scalars_vs_oracle(gpu, oracle, curve, window, logn):
    """0/1 coefficient vectors (selector-like polynomials): every nonzero entry lands in ONE
    bucket of window 0, i.e. one level-2 sort bin of ~n/2 entries (2^20: the 1024-thread k_fine
    with wavefront-aggregated counters; 2^18: the 256-thread one); c = 17 adds the carry-only
    top window of BLS12-381 Montgomery scalars"""
    n = 1 << logn
    rng = np.random.default_rng(91)
    sc = np.zeros((n, 4), dtype=np.uint64)
    sc[:, 0] = rng.integers(0, 2, n).astype(np.uint64)
    pts = gpu.gen_points(curve, 92, n)
    want = oracle.normalize(curve, oracle.msm(curve, sc, pts, mont=False, out="proj"))
    if window:
        got = gpu.msm_variable(curve, sc, pts, window)
    elif logn >= 20:  # device-resident: one pipeline pass over all 2^20 points (host buffers split them)
        ds, dp = gpu.DeviceBuffer(sc), gpu.DeviceBuffer(pts)
        got = oracle.normalize(curve, gpu.msm_device(curve, n, ds, dp, mont=False))
        ds.free()
        dp.free()
    else:
        got = oracle.normalize(curve, gpu.msm_std(curve, sc, pts))
    assert np.array_equal(got, want)
    if window:  # Montgomery scalars through the default entry: the full 255/254-bit recoding
        msc = gpu.gen_fr(curve, 93, n)
        assert np.array_equal(gpu.msm_variable(curve, oracle.to_std(FR_FLD[curve], msc), pts, window),
                              oracle.normalize(curve, oracle.msm(curve, msc, pts, mont=True, out="proj")))


def _skewed_scalars(gpu, curve, kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "binary":  # std 0/1: ~n/2 entries in one bucket of window 0
        sc = np.zeros((n, 4), dtype=np.uint64)
        sc[:, 0] = rng.integers(0, 2, n).astype(np.uint64)
        return sc, False
    if kind == "equal":  # every scalar equal: one bucket per window holds all n points
        return np.tile(gpu.gen_fr(curve, seed, 1), (n, 1)), True
    vals = gpu.gen_fr(curve, seed, 3)  # 3 values + 5 % zeros: a few buckets of ~n/3 per window
    sc = vals[rng.integers(0, 3, n)].copy()
    sc[rng.random(n) < 0.05] = 0
    return sc, True


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("logn", [17, 20])
@pytest.mark.parametrize("kind", ["binary", "equal", "mix3"])
def test_host_split_pipeline_skewed(gpu, oracle, curve, logn, kind):
    """Host-buffer MSMs run split pipelines from 2^17 pairs (2 splits; 4 from 2^19): split h is
    sorted and accumulated while split h+1 crosses PCIe, and a bucket run of a later split starts
    from the earlier splits' sum (k_fill_mark / start_run).  Skewed scalars make runs cross
    chunk, wavefront AND split boundaries.  Checked against the device-resident call (one
    unsplit pipeline) and, at 2^17 and for one 2^20 case, against the oracle."""
    n = 1 << logn
    sc, mont = _skewed_scalars(gpu, curve, kind, n, 700 + logn)
    pts = gpu.gen_points(curve, 701 + logn, n)
    got = gpu.msm_affine(curve, sc, pts, std=not mont)
    ds, dp = gpu.DeviceBuffer(sc), gpu.DeviceBuffer(pts)
    try:
        dev = gpu.g1_to_affine(curve, gpu.msm_device(curve, n, ds, dp, mont=mont))
    finally:
        ds.free()
        dp.free()
    assert np.array_equal(got, dev)
    if logn == 17 or (kind == "mix3" and curve == "bls12_381"):
        assert np.array_equal(got, oracle.msm(curve, sc, pts, mont=mont))


@pytest.mark.parametrize("curve", CURVES)
def test_device_resident_api(gpu, curve):
    n = 5000
    sc = gpu.gen_fr(curve, 41, n)
    pts = gpu.gen_points(curve, 42, n)
    ds, dp = gpu.DeviceBuffer(sc), gpu.DeviceBuffer(pts)
    try:
        assert np.array_equal(gpu.msm_device(curve, n, ds, dp), gpu.msm(curve, sc, pts))
    finally:
        ds.free(); dp.free()


def _baseline(key):
    cfg = baseline_configs().get(key)
    if cfg is None:
        pytest.skip(f"{key} not in tests/golden/baseline_configs.json")
    return cfg


def test_config2_bls12_381_msm_2_20_vs_reference(gpu):
    cfg = _baseline("config2_bls12_381_msm_2^20")
    n = 1 << cfg["log_n"]
    sc = gpu.gen_fr("bls12_381", cfg["seed"], n)
    pts = gpu.gen_points("bls12_381", cfg["seed"], n)
    got = gpu.msm_affine("bls12_381", sc, pts)
    assert [int(x) for x in got] == cfg["affine"]


def test_config4_bn128_msm_2_24_vs_reference(gpu):
    cfg = _baseline("config4_bn128_msm_2^24")
    n = 1 << cfg["log_n"]
    sc = gpu.gen_fr("bn128", cfg["seed"], n)
    pts = gpu.gen_points("bn128", cfg["seed"], n)
    got = gpu.msm_affine("bn128", sc, pts)
    assert [int(x) for x in got] == cfg["affine"]


def test_config5_bls12_381_msm_2_26_vs_reference(gpu):
    """BASELINE config 5 at full size on ONE GPU (the reference's Montgomery entry aborts
    at 2^26, G1_proj.c:631-632 -- ours must not), then as the 8-GPU job splits it: 8
    contiguous shards whose projective partials are summed in rank order."""
    cfg = _baseline("config5_bls12_381_msm_2^26")
    curve = "bls12_381"
    n = 1 << cfg["log_n"]
    sc = gpu.gen_fr(curve, cfg["seed"], n)
    pts = gpu.gen_points(curve, cfg["seed"], n)
    got = gpu.msm_affine(curve, sc, pts)
    assert [int(x) for x in got] == cfg["affine"]
    step = n // 8
    acc = None
    for k in range(8):
        part = gpu.msm(curve, sc[k * step:(k + 1) * step], pts[k * step:(k + 1) * step])
        acc = part if acc is None else gpu.g1_add(curve, acc, part)
    assert [int(x) for x in gpu.g1_to_affine(curve, acc)] == cfg["affine"]


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("nl,high", [(5, "zero"), (5, "random"), (6, "random"), (9, "random")])
def test_std_wide_scalars_vs_reference(gpu, reference, curve, nl, high):
    """std coefficients of more than 4 limbs are used verbatim (G1_proj.c:511,552): the
    reference accepts any expo_nlimbs -- so must we (256-bit slices, Horner on the host)"""
    n = 300
    rng = np.random.default_rng(nl * 10 + (high == "random"))
    sc = np.zeros((n, nl), dtype=np.uint64)
    sc[:, :4] = gpu.gen_fr(curve, 90 + nl, n)
    if high == "random":
        sc[:, 4:] = rng.integers(0, 2**63, size=(n, nl - 4), dtype=np.uint64) * np.uint64(2) + \
            rng.integers(0, 2, size=(n, nl - 4), dtype=np.uint64)
    pts = gpu.gen_points(curve, 91 + nl, n)
    want = reference.msm(curve, sc, pts, mont=False)
    assert np.array_equal(gpu.msm_affine(curve, sc, pts, std=True), want)
    if high == "zero":
        assert np.array_equal(want, gpu.msm_affine(curve, np.ascontiguousarray(sc[:, :4]), pts, std=True))


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("nl", [1, 2, 3, 5])
def test_mont_other_nlimbs_does_not_abort(gpu, curve, nl):
    """Montgomery coefficients with expo_nlimbs != 4: the reference's result is undefined
    (Fr_mont_to_std reads 4 limbs per row, G1_proj.c:637-641); ours uses the row's first
    min(nl, 4) limbs as the Montgomery value -- and, like the reference, does not abort"""
    n = 500
    base = gpu.gen_fr(curve, 95, n)
    pts = gpu.gen_points(curve, 96, n)
    sc = np.zeros((n, nl), dtype=np.uint64)
    k = min(nl, 4)
    sc[:, :k] = base[:, :k]
    ext = np.zeros((n, 4), dtype=np.uint64)
    ext[:, :k] = base[:, :k]
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), gpu.msm_affine(curve, ext, pts))


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("window,limit", [(4, 3 * 4000), (9, 4000), (16, 1)])
def test_window_groups_vs_oracle(gpu, oracle, curve, window, limit):
    """MSMs whose (window, point) entries exceed one pipeline pass (W n >= 2^30 by default:
    int counts of the sort) run in window groups; the cap is lowered here to reach that path"""
    n = 4000
    sc = oracle.to_std(FR_FLD[curve], gpu.gen_fr(curve, 97, n))
    pts = gpu.gen_points(curve, 98, n)
    want = oracle.normalize(curve, oracle.msm(curve, sc, pts, mont=False, out="proj"))
    try:
        gpu.msm_set_group_limit(limit)
        got = gpu.msm_variable(curve, sc, pts, window)
    finally:
        gpu.msm_set_group_limit(0)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("curve", CURVES)
def test_repeated_points_linearity(gpu, oracle, curve):
    """2^16 pairs over 64 distinct points: bucket and Y-sum additions meet equal and opposite
    partial sums (the doubling / infinity branches of the two-chain Y sums); checked against
    the oracle and by linearity msm(a + b) = msm(a || b) over the doubled point list"""
    n = 1 << 16
    base = gpu.gen_points(curve, 0x5A4B0011, 64)
    pts = np.ascontiguousarray(np.resize(base, (n, base.shape[1])))
    a, b = gpu.gen_fr(curve, 702, n), gpu.gen_fr(curve, 703, n)
    ab = gpu.arr_add(curve, a, b)
    lhs = gpu.msm_affine(curve, ab, pts)
    assert np.array_equal(lhs, oracle.msm(curve, ab, pts, mont=True))
    rhs = gpu.msm_affine(curve, np.concatenate([a, b]), np.concatenate([pts, pts]))
    assert np.array_equal(lhs, rhs)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("window,n", [(13, 3000), (16, 20000), (20, 5000)])
def test_ysum_kernels_vs_oracle(gpu, oracle, curve, mode, window, n):
    """both G1 Y-sum kernels -- k_ysum2 (one wave per SIMD, register prefetch, quad fold) and
    k_ysum3 (two waves per SIMD, LDS prefetch, one-lane fold; chosen by size at c = 20 from 2^23)
    -- forced on the same inputs, mostly-empty buckets included, against the oracle"""
    sc = oracle.to_std(FR_FLD[curve], gpu.gen_fr(curve, 800 + window, n))
    pts = gpu.gen_points(curve, 801 + window, n)
    pts[::97] = np.uint64(0xFFFFFFFFFFFFFFFF)  # infinity inputs
    want = oracle.normalize(curve, oracle.msm(curve, sc, pts, mont=False, out="proj"))
    try:
        gpu.msm_set_ysum_mode(mode)
        got = gpu.msm_variable(curve, sc, pts, window)
    finally:
        gpu.msm_set_ysum_mode(-1)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("window,n", [(0, 5000), (13, 9001), (16, 70000), (20, 20000), (0, (1 << 18) + 5)])
def test_sort_ahead_groups_vs_oracle(gpu, oracle, curve, window, n):
    """the sort-ahead shape -- two window groups with both sorts on the second stream (by default
    from 2^23 device-resident BN128 pairs) -- forced down to small inputs: equal to the oracle,
    to the plain pipeline and to the default, odd window counts included"""
    sc = gpu.gen_fr(curve, 900 + window, n)
    pts = gpu.gen_points(curve, 901 + window, n)
    pts[::113] = np.uint64(0xFFFFFFFFFFFFFFFF)
    ds, dp = gpu.DeviceBuffer(sc), gpu.DeviceBuffer(pts)
    try:
        gpu.msm_set_ahead_min(0)
        one = gpu.msm_device(curve, n, ds, dp, window=window)
        gpu.msm_set_ahead_min(12)
        two = gpu.msm_device(curve, n, ds, dp, window=window)
        assert gpu.msm_last_groups() == 2
        gpu.msm_set_ahead_min(-1)
        dflt = gpu.msm_device(curve, n, ds, dp, window=window)
    finally:
        gpu.msm_set_ahead_min(-1)
        ds.free()
        dp.free()
    assert np.array_equal(one, two) and np.array_equal(one, dflt)
    want = oracle.normalize(curve, oracle.msm(curve, sc, pts, mont=True, out="proj"))
    assert np.array_equal(oracle.normalize(curve, two), want)
