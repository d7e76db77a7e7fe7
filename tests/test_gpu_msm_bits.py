"""The small-input MSM path (bit jobs, zk_msm_impl.hpp k_bitacc / k_bitsum): default-window calls
with n <= msm_bits_max (4096) skip the bucket pipeline.  Checked bit-exact against the oracle
(the restatement of bls12_381_G1_proj.c:507-605, pinned to the reference's own build) and against
the bucket pipeline itself (explicit windows always take it) on the same inputs, across the
chunking edges (n around the 256 blocks), adversarial scalars (all bits set, all zero, equal
scalars), repeated points, P / -P pairs and infinity inputs, host and device buffers, and the
256-bit std scalars whose top bit is set.  The golden cases (n = 1 ... 4096) in test_gpu_msm.py
run through this path as well."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
CURVES = ["bn128", "bls12_381"]
R_MOD = {"bn128": 21888242871839275222246405745257275088548364400416034343698204186575808495617,
         "bls12_381": 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001}
P_MOD = {"bn128": 21888242871839275222246405745257275088696311157297823662689037894645226208583,
         "bls12_381": 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB}


def _limbs(v, nl):
    return [np.uint64((v >> (64 * j)) & ((1 << 64) - 1)) for j in range(nl)]


def _neg(curve, pt, NP):
    """-P of one affine point in the reference's Montgomery form: y -> p - y (the form is linear)"""
    y = sum(int(pt[NP + j]) << (64 * j) for j in range(NP))
    out = pt.copy()
    out[NP:] = _limbs((P_MOD[curve] - y) % P_MOD[curve], NP)
    return out


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n", [1, 3, 64, 255, 256, 257, 511, 1000, 4095, 4096])
def test_bits_sizes_vs_oracle_and_buckets(gpu, oracle, curve, n):
    sc = gpu.gen_fr(curve, 7000 + n, n)
    pts = gpu.gen_points(curve, 8000 + n, n)
    want = oracle.msm(curve, sc, pts, mont=True)
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), want)
    # device-resident: default window (bit jobs) against an explicit window (bucket pipeline)
    ds, dp = gpu.DeviceBuffer(sc), gpu.DeviceBuffer(pts)
    try:
        c = gpu.load().zkg_msm_default_window(n)
        a = gpu.msm_device(curve, n, ds, dp)
        b = gpu.msm_device(curve, n, ds, dp, window=max(c, 4))
    finally:
        ds.free()
        dp.free()
    assert np.array_equal(a, b)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("kind", ["all_ones", "zero", "equal", "one", "top_bit"])
def test_bits_adversarial_scalars(gpu, oracle, curve, kind):
    n = 777
    pts = gpu.gen_points(curve, 91, n)
    if kind == "top_bit":  # verbatim 256-bit std scalars: bit 255 set (nread 4 -> 256 bit jobs)
        sc = gpu.gen_fr(curve, 92, n).copy()
        sc[:, 3] |= np.uint64(1 << 63)
        want = oracle.msm(curve, sc, pts, mont=False)
        assert np.array_equal(gpu.msm_affine(curve, sc, pts, std=True), want)
        return
    if kind == "all_ones":  # r - 1 in standard form: every bit job holds many points
        std = np.zeros((n, 4), dtype=np.uint64)
        std[:] = _limbs(R_MOD[curve] - 1, 4)
        want = oracle.msm(curve, std, pts, mont=False)
        assert np.array_equal(gpu.msm_affine(curve, std, pts, std=True), want)
        return
    if kind == "zero":
        sc = np.zeros((n, 4), dtype=np.uint64)
    elif kind == "equal":
        sc = np.tile(gpu.gen_fr(curve, 93, 1), (n, 1))
    else:  # "one": std scalar 1 -> the plain sum of the points (only bit job 0 is non-empty)
        one_std = np.zeros((n, 4), dtype=np.uint64)
        one_std[:, 0] = 1
        want = oracle.msm(curve, one_std, pts, mont=False)
        assert np.array_equal(gpu.msm_affine(curve, one_std, pts, std=True), want)
        return
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), oracle.msm(curve, sc, pts, mont=True))


@pytest.mark.parametrize("curve", CURVES)
def test_bits_repeated_points_and_infinity(gpu, oracle, curve):
    """one point repeated (a lane's accumulator meets the same point: the madd's doubling case),
    infinity inputs mixed in, and a point next to its negation (cancellation to infinity inside a
    chunk, then more additions)"""
    n = 600
    base = gpu.gen_points(curve, 94, 3)
    pts = np.tile(base[0], (n, 1))
    pts[::7] = np.uint64(0xFFFFFFFFFFFFFFFF)  # infinity sentinel (all 0xFF), the reference's
    sc = gpu.gen_fr(curve, 95, n)
    assert np.array_equal(gpu.msm_affine(curve, sc, pts), oracle.msm(curve, sc, pts, mont=True))
    # P followed by -P with equal scalars: the pair cancels in every bit job it enters
    NP = gpu.NLIMBS_P[curve]
    neg = _neg(curve, base[1], NP)
    pts2 = np.empty((n, 2 * NP), dtype=np.uint64)
    pts2[0::2] = base[1]
    pts2[1::2] = neg
    sc2 = np.tile(gpu.gen_fr(curve, 96, 1), (n, 1))
    got = gpu.msm_affine(curve, sc2, pts2)
    assert np.array_equal(got, oracle.msm(curve, sc2, pts2, mont=True))
    assert np.all(got == np.uint64(0xFFFFFFFFFFFFFFFF))
    # every third point replaced by another one: pairs no longer all cancel
    pts3 = pts2.copy()
    pts3[2::3] = base[2]
    assert np.array_equal(gpu.msm_affine(curve, sc2, pts3), oracle.msm(curve, sc2, pts3, mont=True))


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("nl", [1, 2, 5])
def test_bits_std_short_and_wide(gpu, oracle, reference, curve, nl):
    """std scalars of 1 / 2 limbs (64 / 128 bit jobs) and 5 limbs (a 256-bit slice and a 64-bit
    slice, each its own bit-job MSM, combined on the host)"""
    n = 300
    pts = gpu.gen_points(curve, 97, n)
    sc = np.zeros((n, nl), dtype=np.uint64)
    src = gpu.gen_fr(curve, 98, n)
    for j in range(nl):
        sc[:, j] = src[:, j % 4] ^ np.uint64(0x9E3779B97F4A7C15 * (j + 1) & ((1 << 64) - 1))
    want = reference.msm(curve, sc, pts, mont=False)
    assert np.array_equal(gpu.msm_affine(curve, sc, pts, std=True), want)
