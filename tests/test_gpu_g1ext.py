"""GPU G1 batch affine conversion and group FFT through the
reference-named C ABI, bit-exact against the reference's own C (oracle/_ref):
  <C>_G1_proj_batch_{from,to}_affine   bls12_381_G1_proj.c:147-167
  <C>_G1_proj_fft_{forward,inverse}    bls12_381_G1_proj.c:679-790
and (round 6) their Jacobian twins <C>_G1_jac_batch_{from,to}_affine / _fft_{forward,inverse}
(bls12_381_G1_jac.c:139-158, 727-838).
Inputs: projective points with non-trivial Z, points at infinity, and (BLS12-381) points
OUTSIDE the order-r subgroup -- for those the result depends on the exact per-level
scalars, so they pin the per-level structure, not just the linear map mod r."""
import hashlib

import numpy as np
import pytest

import golden_io

pytestmark = pytest.mark.gpu
CURVES = ["bn128", "bls12_381"]


def projective(gpu, oracle, curve, n, seed, n_inf=3):
    return golden_io.projective_points(gpu, oracle, curve, n, seed, n_inf)


def bls_nonsubgroup_points(n, seed):
    return golden_io.bls_nonsubgroup_points(n, seed)


def ref_call(reference, curve, name, *args):
    return reference.arr(curve, name, *args)


@pytest.mark.parametrize("curve", CURVES)
def test_batch_from_affine(gpu, reference, curve):
    n = 1000
    aff = gpu.gen_points(curve, 101, n)
    aff[[3, 500]] = np.uint64(0xFFFFFFFFFFFFFFFF)  # affine infinity sentinel
    want = np.zeros((n, 3 * gpu.NLIMBS_P[curve]), dtype=np.uint64)
    ref_call(reference, curve, "G1_proj_batch_from_affine", n, aff, want)
    assert np.array_equal(gpu.batch_from_affine(curve, aff), want)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n", [1, 31, 33, 1000, 1 << 16, (1 << 20) + 37])  # 2^20 + 37: 16 points per inversion, ragged
def test_batch_to_affine(gpu, oracle, reference, curve, n):
    proj = projective(gpu, oracle, curve, n, 102 + n) if n <= 1000 else None
    if proj is None:  # large: cheap inputs (Z = 1 after from_affine, plus infinities)
        aff = gpu.gen_points(curve, 103, n)
        aff[::1000] = np.uint64(0xFFFFFFFFFFFFFFFF)
        proj = gpu.batch_from_affine(curve, aff)
    want = np.zeros((n, 2 * gpu.NLIMBS_P[curve]), dtype=np.uint64)
    ref_call(reference, curve, "G1_proj_batch_to_affine", n, proj, want)
    assert np.array_equal(gpu.batch_to_affine(curve, proj), want)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("m", [0, 1, 2, 3, 5, 8, 10])
def test_fft_vs_reference(gpu, oracle, reference, curve, m):
    """subgroup points (with infinities): the GLV stages run (pair-split multiplications,
    decomposed twiddles, the inverse's 1/2 per level deferred to one N^-1) and the normalised
    output equals the reference's bit for bit"""
    n = 1 << m
    pts = projective(gpu, oracle, curve, n, 200 + m, n_inf=min(2, n))
    sg = gpu.get_fft_subgroup(curve, m)
    for name, f in (("G1_proj_fft_forward", gpu.forward_fft), ("G1_proj_fft_inverse", gpu.inverse_fft)):
        want = np.zeros_like(pts)
        ref_call(reference, curve, name, m, sg.gen_array(), pts, want)
        assert np.array_equal(f(sg, pts), want), (name, m)
        assert gpu.g1_fft_last_glv() == (1 if m > 0 else 0), (name, m)


def test_fft_one_nonsubgroup_point_falls_back(gpu, oracle, reference):
    """BLS12-381: one input outside the r-subgroup among subgroup points -> the membership check
    fails and the integer-scalar stages run (the reference's exact schedule)"""
    curve, m = "bls12_381", 6
    n = 1 << m
    pts = projective(gpu, oracle, curve, n, 250, n_inf=1)
    pts[5] = gpu.batch_from_affine(curve, bls_nonsubgroup_points(1, 251))[0]
    sg = gpu.get_fft_subgroup(curve, m)
    for name, f in (("G1_proj_fft_forward", gpu.forward_fft), ("G1_proj_fft_inverse", gpu.inverse_fft)):
        want = np.zeros_like(pts)
        ref_call(reference, curve, name, m, sg.gen_array(), pts, want)
        assert np.array_equal(f(sg, pts), want), name
        assert gpu.g1_fft_last_glv() == 0, name


@pytest.mark.parametrize("m", [1, 3, 6])
def test_fft_nonsubgroup_points_bls(gpu, reference, m):
    """points outside the r-subgroup: only the exact per-level scalar schedule matches"""
    curve = "bls12_381"
    n = 1 << m
    proj = gpu.batch_from_affine(curve, bls_nonsubgroup_points(n, 300 + m))
    sg = gpu.get_fft_subgroup(curve, m)
    for name, f in (("G1_proj_fft_forward", gpu.forward_fft), ("G1_proj_fft_inverse", gpu.inverse_fft)):
        want = np.zeros_like(proj)
        ref_call(reference, curve, name, m, sg.gen_array(), proj, want)
        assert np.array_equal(f(sg, proj), want), (name, m)
        assert gpu.g1_fft_last_glv() == 0, (name, m)


@pytest.mark.parametrize("curve", CURVES)
def test_fft_roundtrip_2_12(gpu, curve):
    """size-independent property at a larger size: iFFT(FFT(P)) = P for subgroup points"""
    m = 12
    aff = gpu.gen_points(curve, 400, 1 << m)
    proj = gpu.batch_from_affine(curve, aff)
    sg = gpu.get_fft_subgroup(curve, m)
    back = gpu.inverse_fft(sg, gpu.forward_fft(sg, proj))
    assert np.array_equal(back, proj)


# ---------------------------------------------------------------------------- Jacobian twins (round 6)
# <C>_G1_jac_batch_{from,to}_affine (bls12_381_G1_jac.c:139-158) and <C>_G1_jac_fft_{forward,inverse}
# (:727-838), bound by the Jacobian G1 instance (G1/Jac.hs:188-196, 264-291, 374-389)

def jacobian(gpu, oracle, curve, n, seed, n_inf=3, affine=None):
    return golden_io.jacobian_points(gpu, oracle, curve, n, seed, n_inf, affine)


@pytest.mark.parametrize("curve", CURVES)
def test_jac_batch_from_affine(gpu, reference, curve):
    n = 1000
    aff = gpu.gen_points(curve, 111, n)
    aff[[3, 500, 999]] = np.uint64(0xFFFFFFFFFFFFFFFF)  # -> the Jacobian infinity (1 : 1 : 0)
    want = np.zeros((n, 3 * gpu.NLIMBS_P[curve]), dtype=np.uint64)
    ref_call(reference, curve, "G1_jac_batch_from_affine", n, aff, want)
    assert np.array_equal(gpu.batch_from_affine(curve, aff, coords="jac"), want)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n", [1, 31, 33, 1000, 1 << 16, (1 << 20) + 37])
def test_jac_batch_to_affine(gpu, oracle, reference, curve, n):
    """Jacobian rows with random Z (x l^2, y l^3, l) and infinities (l^2 : l^3 : 0) up to 1000 rows;
    beyond, from_affine rows (Z = 1) with infinities -- ragged counts per inversion chunk"""
    if n <= 1000:
        jac = jacobian(gpu, oracle, curve, n, 112 + n)
    else:
        aff = gpu.gen_points(curve, 113, n)
        aff[::997] = np.uint64(0xFFFFFFFFFFFFFFFF)
        jac = gpu.batch_from_affine(curve, aff, coords="jac")
    want = np.zeros((n, 2 * gpu.NLIMBS_P[curve]), dtype=np.uint64)
    ref_call(reference, curve, "G1_jac_batch_to_affine", n, jac, want)
    assert np.array_equal(gpu.batch_to_affine(curve, jac, coords="jac"), want)


@pytest.mark.parametrize("curve", CURVES)
def test_jac_batch_to_affine_bls_nonsubgroup(gpu, oracle, reference, curve):
    """points off the order-r subgroup (BLS12-381) and a non-trivial Z: the conversion is the same
    field arithmetic; checked against the reference anyway"""
    if curve != "bls12_381":
        pytest.skip("BN254 G1 has cofactor 1")
    n = 333
    jac = jacobian(gpu, oracle, curve, n, 114, n_inf=4, affine=bls_nonsubgroup_points(n, 115))
    want = np.zeros((n, 12), dtype=np.uint64)
    ref_call(reference, curve, "G1_jac_batch_to_affine", n, jac, want)
    assert np.array_equal(gpu.batch_to_affine(curve, jac, coords="jac"), want)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("m", [0, 1, 2, 3, 5, 8])
def test_jac_fft_vs_reference(gpu, oracle, reference, curve, m):
    n = 1 << m
    pts = jacobian(gpu, oracle, curve, n, 210 + m, n_inf=min(2, n))
    sg = gpu.get_fft_subgroup(curve, m)
    for name, f in (("G1_jac_fft_forward", gpu.forward_fft), ("G1_jac_fft_inverse", gpu.inverse_fft)):
        want = np.zeros_like(pts)
        ref_call(reference, curve, name, m, sg.gen_array(), pts, want)
        assert np.array_equal(f(sg, pts, coords="jac"), want), (name, m)
        assert gpu.g1_fft_last_glv() == (1 if m > 0 else 0), (name, m)


@pytest.mark.parametrize("m", [1, 3, 6])
def test_jac_fft_nonsubgroup_points_bls(gpu, oracle, reference, m):
    """Jacobian points outside the r-subgroup: the integer-scalar stages, the reference's exact schedule"""
    curve = "bls12_381"
    n = 1 << m
    pts = jacobian(gpu, oracle, curve, n, 310 + m, n_inf=1, affine=bls_nonsubgroup_points(n, 320 + m))
    sg = gpu.get_fft_subgroup(curve, m)
    for name, f in (("G1_jac_fft_forward", gpu.forward_fft), ("G1_jac_fft_inverse", gpu.inverse_fft)):
        want = np.zeros_like(pts)
        ref_call(reference, curve, name, m, sg.gen_array(), pts, want)
        assert np.array_equal(f(sg, pts, coords="jac"), want), (name, m)
        assert gpu.g1_fft_last_glv() == 0, (name, m)


@pytest.mark.parametrize("curve", CURVES)
def test_jac_fft_equals_proj_fft(gpu, oracle, curve):
    """the same points in both coordinate systems give the same normalised output (the Jacobian
    and projective FFTs are one algorithm over the same group elements)"""
    m = 10
    aff = gpu.gen_points(curve, 401, 1 << m)
    aff[[7, 300]] = np.uint64(0xFFFFFFFFFFFFFFFF)
    sg = gpu.get_fft_subgroup(curve, m)
    for f in (gpu.forward_fft, gpu.inverse_fft):
        a = f(sg, gpu.batch_from_affine(curve, aff, coords="jac"), coords="jac")
        b = f(sg, gpu.batch_from_affine(curve, aff))
        assert np.array_equal(a, b)


@pytest.mark.parametrize("curve", CURVES)
def test_msm_jac_points_vs_reference(gpu, oracle, reference, curve):
    """Jac's Curve.msm = msm cs (batchToAffine gs) (G1/Jac.hs:188, 220): the reference's Jacobian
    MSM over the reference's own batch_to_affine of the same Jacobian rows"""
    n = 777
    jac = jacobian(gpu, oracle, curve, n, 500, n_inf=5)
    sc = gpu.gen_fr(curve, 501, n)
    aff = np.zeros((n, 2 * gpu.NLIMBS_P[curve]), dtype=np.uint64)
    ref_call(reference, curve, "G1_jac_batch_to_affine", n, jac, aff)
    want = reference.msm_jac(curve, sc, aff, mont=True)
    nrm = np.zeros_like(want)
    ref_call(reference, curve, "G1_jac_normalize", want, nrm)
    got = gpu.msm_jac_points(curve, sc, jac)
    if nrm[2 * gpu.NLIMBS_P[curve]:].any():
        assert np.array_equal(got, nrm)
    else:  # infinity: ours (1 : 1 : 0) like the reference's jac_out
        assert not got[2 * gpu.NLIMBS_P[curve]:].any()


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


GFFT = golden_io.group_fft_golden()


@pytest.mark.parametrize("key", sorted(GFFT))
def test_fft_vs_reference_digests(gpu, oracle, key):
    """KZG-SRS sizes (the reference's curveIFFT builds the Lagrange SRS with fft_inverse,
    examples/KZG.hs:55): 2^12 and 2^14 subgroup points with random Z and infinities on both curves
    (the GLV stages at full occupancy, the 4-lane first inverse stage, shared-table lane pairs),
    and BLS12-381 points outside the r-subgroup at 2^10 (the integer stages).  The reference's
    outputs are stored as SHA-256 digests (tools/make_golden.py groupfft)."""
    g = GFFT[key]
    curve, m, kind = g["curve"], g["log_n"], g["input"]
    n = 1 << m
    coords = "jac" if "jacobian" in kind else "proj"
    if kind == "subgroup_projective":
        pts = projective(gpu, oracle, curve, n, g["seed"], n_inf=g["n_inf"])
    elif kind == "subgroup_jacobian":
        pts = jacobian(gpu, oracle, curve, n, g["seed"], n_inf=g["n_inf"])
    elif kind == "nonsubgroup_jacobian":
        pts = jacobian(gpu, oracle, curve, n, g["seed"], n_inf=g["n_inf"],
                       affine=bls_nonsubgroup_points(n, g["seed"]))
    else:
        pts = gpu.batch_from_affine(curve, bls_nonsubgroup_points(n, g["seed"]))
    assert _sha(pts) == g["input_sha256"]
    sg = gpu.get_fft_subgroup(curve, m)
    fwd = gpu.forward_fft(sg, pts, coords=coords)
    assert gpu.g1_fft_last_glv() == (1 if kind.startswith("subgroup") else 0)
    assert _sha(fwd) == g["forward_sha256"], key
    inv = gpu.inverse_fft(sg, pts, coords=coords)
    assert _sha(inv) == g["inverse_sha256"], key
