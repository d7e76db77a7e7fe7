"""GPU G2 MSM through the reference-named C ABI
(<C>_G2_proj_MSM_{mont,std}_coeff_{proj,affine}_out, bls12_381_G2_proj.c:498-660),
bit-exact against the reference's own C (oracle/_ref).  Test points are built with the
reference library itself: an arithmetic progression P0 + i H of generator multiples,
converted by its batch_to_affine."""
import hashlib

import numpy as np
import pytest

import golden_io

pytestmark = pytest.mark.gpu
CURVES = ["bn128", "bls12_381"]


def g2_points(reference, curve, n, k0=12345, k1=67890):
    return golden_io.g2_points(reference.lib, curve, n, k0, k1)


def ref_msm(reference, curve, sc, pts, mont, affine):
    NP = {"bn128": 4, "bls12_381": 6}[curve]
    out = np.zeros((4 if affine else 6) * NP, np.uint64)
    name = f"G2_proj_MSM_{'mont' if mont else 'std'}_coeff_{'affine' if affine else 'proj'}_out"
    reference.arr(curve, name, sc.shape[0], sc, pts, out, sc.shape[1])
    return out


def ref_normalize(reference, curve, proj):
    out = np.zeros_like(proj)
    reference.arr(curve, "G2_proj_normalize", proj, out)
    return out


@pytest.fixture(scope="module")
def points(reference):
    return {c: g2_points(reference, c, 2048) for c in CURVES}


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n", [1, 2, 17, 300, 2048])
def test_g2_msm_vs_reference(gpu, reference, points, curve, n):
    pts = points[curve][:n].copy()
    sc = gpu.gen_fr(curve, 500 + n, n)
    for mont in (True, False):
        want = ref_msm(reference, curve, sc, pts, mont, affine=True)
        assert np.array_equal(gpu.g2_msm(curve, sc, pts, std=not mont, affine=True), want), (n, mont)
    want = ref_normalize(reference, curve, ref_msm(reference, curve, sc, pts, True, affine=False))
    assert np.array_equal(gpu.g2_msm(curve, sc, pts, affine=False), want)


@pytest.mark.parametrize("curve", CURVES)
def test_g2_msm_edge_cases(gpu, reference, points, curve):
    n = 257
    pts = points[curve][:n].copy()
    sc = gpu.gen_fr(curve, 600, n)
    pts[[3, 100]] = np.uint64(0xFFFFFFFFFFFFFFFF)  # affine infinity inputs are skipped
    sc[[5, 6]] = 0                                  # zero scalars
    pts[10] = pts[11]                               # duplicate points
    std = sc.copy()
    std[7] = np.uint64(0xFFFFFFFFFFFFFFFF)          # 2^256 - 1 on the std path (used verbatim)
    for mont, s in ((True, sc), (False, std)):
        want = ref_msm(reference, curve, s, pts, mont, affine=True)
        assert np.array_equal(gpu.g2_msm(curve, s, pts, std=not mont, affine=True), want), mont
    # all-zero scalars -> infinity (all-0xFF affine)
    z = np.zeros_like(sc)
    assert np.all(gpu.g2_msm(curve, z, pts, affine=True) == np.uint64(0xFFFFFFFFFFFFFFFF))


@pytest.mark.parametrize("curve", CURVES)
def test_g2_msm_linearity_large(gpu, points, curve):
    """size-independent property at 2^16: msm(a + b) = msm(a) + msm(b) on the same points
    (checked as msm over the doubled point list with concatenated scalars)"""
    base = points[curve]
    n = 1 << 16
    pts = np.ascontiguousarray(np.resize(base, (n, base.shape[1])))
    a, b = gpu.gen_fr(curve, 700, n), gpu.gen_fr(curve, 701, n)
    ab = gpu.arr_add(curve, a, b)
    lhs = gpu.g2_msm(curve, ab, pts, affine=True)
    rhs = gpu.g2_msm(curve, np.concatenate([a, b]), np.concatenate([pts, pts]), affine=True)
    assert np.array_equal(lhs, rhs)


# ---------------------------------------------------------------------------- bench sizes (round 6)
G2L = golden_io.g2_large_golden()


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("key", sorted(G2L))
def test_g2_msm_vs_reference_at_bench_sizes(gpu, oracle, reference, key):
    """2^16 and 2^18 DISTINCT points on both curves (the sizes bench_ext times: large windows, the
    G2 bucket sort and Y sums), with infinities and zero scalars, against the reference's own
    <C>_G2_proj_MSM_mont_coeff_affine_out (tools/make_golden.py g2large); at 2^16 also the std entry
    with a 2^256 - 1 scalar row (used verbatim)"""
    g = G2L[key]
    curve = g["curve"]
    sc, pts = golden_io.g2_case_inputs(reference.lib, curve, g["log_n"], g["seed"], gpu.gen_fr)
    assert _sha(sc) == g["scalars_sha256"] and _sha(pts) == g["points_sha256"]
    got = gpu.g2_msm(curve, sc, pts, affine=True)
    assert [int(x) for x in got] == g["mont_affine"], key
    if "std_affine_row3_all_ones" in g:
        std = oracle.to_std({"bn128": 1, "bls12_381": 3}[curve], sc)
        std[3] = np.uint64(0xFFFFFFFFFFFFFFFF)
        got = gpu.g2_msm(curve, std, pts, std=True, affine=True)
        assert [int(x) for x in got] == g["std_affine_row3_all_ones"], key
