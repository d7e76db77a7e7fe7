"""GPU G2 MSM through the reference-named C ABI
(<C>_G2_proj_MSM_{mont,std}_coeff_{proj,affine}_out, bls12_381_G2_proj.c:498-660),
bit-exact against the reference's own C (oracle/_ref).  Test points are built with the
reference library itself: an arithmetic progression P0 + i H of generator multiples,
converted by its batch_to_affine."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
CURVES = ["bn128", "bls12_381"]


def g2_points(reference, curve, n, k0=12345, k1=67890):
    NP = {"bn128": 4, "bls12_381": 6}[curve]
    lib = reference.lib
    gen = np.ctypeslib.as_array((ctypes.c_uint64 * (6 * NP)).in_dll(lib, f"{curve}_G2_proj_gen_G2")).copy()
    scl = getattr(lib, f"{curve}_G2_proj_scl_small")
    scl.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    p0, h = np.zeros(6 * NP, np.uint64), np.zeros(6 * NP, np.uint64)
    scl(k0, gen.ctypes.data, p0.ctypes.data)
    scl(k1, gen.ctypes.data, h.ctypes.data)
    proj = np.zeros((n, 6 * NP), np.uint64)
    add = getattr(lib, f"{curve}_G2_proj_add")
    cur = p0.copy()
    for i in range(n):
        proj[i] = cur
        nxt = np.zeros_like(cur)
        add(cur.ctypes.data_as(ctypes.c_void_p), h.ctypes.data_as(ctypes.c_void_p),
            nxt.ctypes.data_as(ctypes.c_void_p))
        cur = nxt
    aff = np.zeros((n, 4 * NP), np.uint64)
    reference.arr(curve, "G2_proj_batch_to_affine", n, proj, aff)
    return aff


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
