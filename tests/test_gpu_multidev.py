"""The library's own device set behind the reference symbols (zkg_set_devices / ZKG_DEVICES):
the host-buffer MSM entry points split the pairs into contiguous chunks, one per listed device
(a device listed k times gets k contexts: streams and arenas of its own), and add the partial
sums in list order.  On the one-GPU box the set lists device 0 two or eight times -- the same
code path an 8-GPU node takes with ids 0..7.  Also: zkg_release, the out-of-memory degrade of
the MSM working set, and window sizes the reference accepts beyond the default range."""
import numpy as np
import pytest

from golden_io import baseline_configs, msm_cases

pytestmark = pytest.mark.gpu
CURVES = ["bn128", "bls12_381"]


@pytest.fixture
def shards(gpu, request):
    gpu.set_devices([0] * request.param)
    yield request.param
    gpu.set_devices([])


def test_device_set_api(gpu):
    assert gpu.get_devices() == []
    gpu.set_devices([0, 0, 0])
    try:
        assert gpu.get_devices() == [0, 0, 0]
        with pytest.raises(ValueError):
            gpu.set_devices([0, gpu.device_count()])  # invalid id: rejected, set unchanged
        assert gpu.get_devices() == [0, 0, 0]
    finally:
        gpu.set_devices([])
    assert gpu.get_devices() == []


@pytest.mark.parametrize("curve", CURVES)
def test_one_entry_device_set(gpu, oracle, curve):
    """a one-entry set pins the host-buffer MSM and NTT to that device: get_devices
    reports it and the results are unchanged (on the one-GPU box the entry is device 0, so this
    runs the pinned path -- hipSetDevice to the listed device around the call)"""
    n = 5000
    sc = gpu.gen_fr(curve, 81, n)
    pts = gpu.gen_points(curve, 82, n)
    m = 16
    sg = gpu.get_fft_subgroup(curve, m)
    x = gpu.gen_fr(curve, 83, 1 << m)
    want_msm = gpu.msm_affine(curve, sc, pts)
    want_ntt = gpu.forward_ntt(sg, x)
    gpu.set_devices([0])
    try:
        assert gpu.get_devices() == [0]
        assert np.array_equal(gpu.msm_affine(curve, sc, pts), want_msm)
        assert np.array_equal(gpu.forward_ntt(sg, x), want_ntt)
        assert np.array_equal(gpu.inverse_ntt(sg, want_ntt), x)
    finally:
        gpu.set_devices([])
    assert np.array_equal(want_msm, oracle.msm(curve, sc, pts, mont=True))


@pytest.mark.parametrize("shards", [2, 8], indirect=True)
@pytest.mark.parametrize("curve", CURVES)
def test_sharded_golden(gpu, curve, shards):
    """every reference golden case (n = 1 ... 4096, zero / equal / wide scalars, P and -P,
    infinity inputs) through the sharded entry points: affine and normalised projective"""
    for name, sc, pts, mont, aff, projn in msm_cases(curve):
        assert np.array_equal(gpu.msm_affine(curve, sc, pts, std=not mont), aff), name
        got = gpu.msm(curve, sc, pts) if mont else gpu.msm_std(curve, sc, pts)
        assert np.array_equal(got, projn), name


@pytest.mark.parametrize("shards", [2, 4, 8], indirect=True)
def test_sharded_config5_2_26(gpu, shards):
    """BASELINE config 5 (2^26 BLS12-381 pairs) through bls12_381_G1_proj_MSM_mont_coeff_affine_out
    with the device set: equal to the reference's output (chunks of 2^25 / 2^24 / 2^23 pairs -- the
    per-GPU sizes of the multi-GPU config-5 line at N = 2 / 4 / 8, c = 20 with the sub-bin sort at
    the first two)"""
    cfg = baseline_configs().get("config5_bls12_381_msm_2^26")
    if cfg is None:
        pytest.skip("config 5 missing")
    n = 1 << cfg["log_n"]
    sc = gpu.gen_fr("bls12_381", cfg["seed"], n)
    pts = gpu.gen_points("bls12_381", cfg["seed"], n)
    assert [int(x) for x in gpu.msm_affine("bls12_381", sc, pts)] == cfg["affine"]


@pytest.mark.parametrize("shards", [3], indirect=True)
@pytest.mark.parametrize("curve", CURVES)
def test_sharded_uneven_and_wide(gpu, oracle, reference, curve, shards):
    """uneven chunks (n not a multiple of the set size) and 320-bit std scalars (256-bit slices
    inside every shard)"""
    n = 1001
    sc = gpu.gen_fr(curve, 61, n)
    pts = gpu.gen_points(curve, 62, n)
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), oracle.msm(curve, sc, pts, mont=True))
    wide = np.zeros((n, 5), dtype=np.uint64)
    wide[:, :4] = sc
    wide[:, 4] = np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    assert np.array_equal(gpu.msm_affine(curve, wide, pts, std=True), reference.msm(curve, wide, pts, mont=False))


@pytest.mark.parametrize("curve", CURVES)
def test_g2_sharded_vs_reference(gpu, reference, curve):
    """the G2 entry points (<C>_G2_proj_MSM_*) take the same split"""
    from test_gpu_g2 import g2_points, ref_msm
    n = 301
    pts = g2_points(reference, curve, n)
    sc = gpu.gen_fr(curve, 63, n)
    want = ref_msm(reference, curve, sc, pts, True, affine=True)
    gpu.set_devices([0, 0, 0, 0])
    try:
        got = gpu.g2_msm(curve, sc, pts, affine=True)
    finally:
        gpu.set_devices([])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("curve", CURVES)
def test_release_then_reuse(gpu, curve):
    """zkg_release frees the arenas, staging and twiddle caches; later calls re-allocate"""
    n = 3000
    sc, pts = gpu.gen_fr(curve, 71, n), gpu.gen_points(curve, 72, n)
    want = gpu.msm_affine(curve, sc, pts)
    sg = gpu.get_fft_subgroup(curve, 16)
    x = gpu.gen_fr(curve, 73, 1 << 16)
    f = gpu.forward_ntt(sg, x)
    gpu.release()
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), want)
    assert np.array_equal(gpu.forward_ntt(sg, x), f)
    gpu.release()
    assert np.array_equal(gpu.inverse_ntt(sg, f), x)


@pytest.mark.parametrize("curve", CURVES)
def test_out_of_memory_degrades_to_window_groups(gpu, oracle, curve):
    """an arena cap between the one-pass and the two-pass working sets (test hook standing in
    for a device without the memory): the call drops its cached twiddles, halves the windows
    per pass and completes in 2 passes instead of aborting the caller's process"""
    n = 60000  # below the size from which host-input MSMs split their points (one pipeline either way)
    sc, pts = gpu.gen_fr(curve, 81, n), gpu.gen_points(curve, 82, n)
    want = oracle.msm(curve, sc, pts, mont=True)
    one = gpu.msm_workspace_bytes(curve, n, groups=1)
    two = gpu.msm_workspace_bytes(curve, n, groups=2)
    assert two < one
    gpu.release()  # the arena re-reserves under the cap
    gpu.arena_set_limit((one + two) // 2)
    try:
        got = gpu.msm_affine(curve, sc, pts)
        groups = gpu.msm_last_groups()
    finally:
        gpu.arena_set_limit(0)
        gpu.release()
    assert np.array_equal(got, want)
    assert groups == 2
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), want)
    assert gpu.msm_last_groups() == 1


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("window", [1, 3, 21, 22, 24, 40])
def test_variable_window_edges(gpu, oracle, curve, window):
    """<C>_G1_proj_MSM_std_coeff_proj_out_variable accepts 1..64 in the reference
    (G1_proj.c:509); ours clamps to 4..24 -- the result does not depend on the window, and the
    largest windows (2^23 buckets per window) run end to end"""
    n = 3000
    sc = oracle.to_std({"bn128": 1, "bls12_381": 3}[curve], gpu.gen_fr(curve, 31, n))
    pts = gpu.gen_points(curve, 32, n)
    want = oracle.normalize(curve, oracle.msm(curve, sc, pts, mont=False, out="proj"))
    assert np.array_equal(gpu.msm_variable(curve, sc, pts, window), want)


@pytest.mark.parametrize("shards", [2, 3, 8], indirect=True)
@pytest.mark.parametrize("curve", CURVES)
def test_ntt_host_io_spread(gpu, curve, shards):
    """<C>_poly_mont_ntt_{forward,inverse} with a device set: the transform runs on the first
    listed device, the host copies are split over every listed one (peer / device-to-device
    copies to the compute device) -- against the reference's digests at 2^20 and the unsharded
    results at 2^16 and 2^17 (uneven chunks), in place and out of place"""
    import hashlib
    from golden_io import ntt_patterns_golden
    cases = ntt_patterns_golden()["cases"]
    sg = gpu.get_fft_subgroup(curve, 20)
    x = gpu.gen_fr(curve, 0x5A4B0003, 1 << 20)
    for inverse, key in ((False, "forward"), (True, "inverse")):
        y = gpu.inverse_ntt(sg, x) if inverse else gpu.forward_ntt(sg, x)
        assert hashlib.sha256(y.tobytes()).hexdigest() == cases[f"{curve}/random/m20/{key}"]["sha256"]
    for m in (16, 17):
        sgm = gpu.get_fft_subgroup(curve, m)
        z = gpu.gen_fr(curve, 0x51 + m, 1 << m)
        f = gpu.forward_ntt(sgm, z)
        gpu.set_devices([])
        want = gpu.forward_ntt(sgm, z)
        gpu.set_devices([0] * shards)
        assert np.array_equal(f, want)
        buf = f.copy()
        lib = gpu.load()
        getattr(lib, f"{curve}_poly_mont_ntt_inverse")(m, gpu._p(sgm.gen_array()), gpu._p(buf), gpu._p(buf))
        assert np.array_equal(buf, z)  # in place (src == tgt)
