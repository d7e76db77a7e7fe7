"""Host-side mirror of the reference's MSM / NTT API, over the gfx950 C-ABI library.

The reference exposes this path to users through Haskell:

    ZK.Algebra.Curves.<C>.G1.Proj.msm      :: FlatArray Fr -> FlatArray Affine.G1 -> G1   (G1/Proj.hs:237-246)
    ZK.Algebra.Curves.<C>.G1.Proj.msmStd   :: FlatArray Std.Fr -> FlatArray Affine.G1 -> G1 (G1/Proj.hs:253-262)
    ZK.Algebra.Curves.<C>.G1.Proj.msmProj  :: FlatArray Fr -> FlatArray G1 -> G1         (G1/Proj.hs:222-223)
    ZK.Algebra.Curves.<C>.G1.Affine.msm    = toAffine . Proj.msm                           (G1/Affine.hs:143-149)
    ZK.Algebra.Curves.<C>.Poly.forwardNTT  :: FFTSubgroup Fr -> Poly -> FlatArray Fr       (Poly.hs:400-410)
    ZK.Algebra.Curves.<C>.Poly.inverseNTT  :: FFTSubgroup Fr -> FlatArray Fr -> Poly       (Poly.hs:412-422)
    ZK.Algebra.Class.FFT.getFFTSubgroup    :: Log2 -> FFTSubgroup                          (Class/FFT.hs:60-66)

GHC is not available in this image, so this module is the host-language mirror
(same names in snake_case, same argument meaning, same error messages) used by the
tests and the benchmark.  ``FlatArray`` is a C-contiguous ``numpy.uint64`` array of
shape (n, limbs) -- byte-identical to the reference's pinned FlatArray memory
(Class/Flat.hs:81-83).  Every call goes through the C ABI of
``lib/libzkalgebra_gpu.so`` and runs on the GPU; if the library or a GPU is missing,
calls raise -- there is no CPU fallback.
"""
import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ZK_LIB_PATH: A/B experiments with variant builds of the same library (default: in-tree build)
LIB_PATH = os.environ.get("ZK_LIB_PATH") or os.path.join(HERE, "lib", "libzkalgebra_gpu.so")
U64P = ctypes.POINTER(ctypes.c_uint64)

CURVES = ("bn128", "bls12_381")
CURVE_ID = {"bn128": 0, "bls12_381": 1}
NLIMBS_P = {"bn128": 4, "bls12_381": 6}   # base field limbs (NLIMBS_P in G1_proj.c:17)
NLIMBS_R = 4                               # scalar field limbs
FFT_LOG = {"bn128": 28, "bls12_381": 32}   # 2-adicity of the FFT domain (Fr/Mont.hs fftDomain)

# every exported symbol of include/zkalgebra_gpu.h (checked by tests/test_capi.py)
REFERENCE_SYMBOLS = [
    f"{c}_G1_proj_MSM_{k}_coeff_{o}_out" for c in CURVES for k in ("mont", "std") for o in ("proj", "affine")
] + [f"{c}_G1_proj_MSM_std_coeff_proj_out_variable" for c in CURVES] + [
    f"{c}_G1_jac_MSM_{k}_coeff_{o}_out" for c in CURVES for k in ("mont", "std") for o in ("jac", "affine")
] + [f"{c}_poly_mont_ntt_{d}" for c in CURVES for d in ("forward", "inverse")]
# Fr vector ops (lib/cbits/curves/array/mont/<C>_arr_mont.h:3-48) + division by a vanishing polynomial
ARR_OPS = ["is_valid", "is_zero", "is_one", "is_equal", "set_zero", "set_one", "set_const", "copy", "from_std",
           "to_std", "append", "neg", "add", "sub", "sqr", "mul", "inv", "div", "neg_inplace", "add_inplace",
           "sub_inplace", "sqr_inplace", "mul_inplace", "inv_inplace", "div_inplace", "sub_inplace_reverse",
           "mul_add", "mul_sub", "dot_prod", "powers", "scale", "scale_inplace", "Ax_plus_y", "Ax_plus_y_inplace",
           "Ax_plus_By", "Ax_plus_By_inplace"]
REFERENCE_SYMBOLS += [f"{c}_arr_mont_{o}" for c in CURVES for o in ARR_OPS] + [
    f"{c}_poly_mont_{k}_by_vanishing" for c in CURVES for k in ("div", "quot")] + [
    f"{c}_G1_{co}_{f}" for c in CURVES for co in ("proj", "jac")
    for f in ("batch_from_affine", "batch_to_affine", "fft_forward", "fft_inverse")] + [
    f"{c}_G2_proj_MSM_{k}_coeff_{o}_out" for c in CURVES for k in ("mont", "std") for o in ("proj", "affine")]
EXTENSION_SYMBOLS = [
    "zkg_version", "zkg_device_count", "zkg_set_device", "zkg_device_malloc", "zkg_device_free",
    "zkg_memcpy_htod", "zkg_memcpy_dtoh", "zkg_device_synchronize", "zkg_g1_msm_device", "zkg_ntt_device",
    "zkg_g1_proj_add", "zkg_g1_proj_normalize", "zkg_g1_proj_to_affine", "zkg_gen_fr", "zkg_gen_g1_points",
    "zkg_fft_generator", "zkg_msm_default_window", "zkg_msm_window", "zkg_timer_enable", "zkg_timer_reset", "zkg_timer_read",
    "zkg_arr_op_device", "zkg_arr_dot_device", "zkg_arr_powers_device",
    "zkg_poly_div_by_vanishing_device", "zkg_g1_fft_device", "zkg_g1_batch_to_affine_device",
    "zkg_g1_jac_fft_device", "zkg_g1_jac_batch_to_affine_device", "zkg_g2_msm_device",
    "zkg_msm_profile", "zkg_msm_set_group_limit", "zkg_msm_set_ysum_mode", "zkg_msm_set_ahead_min", "zkg_ntt_set_max_radix", "zkg_ntt_set_table_max",
    "zkg_arena_set_limit", "zkg_msm_last_groups", "zkg_g1_fft_last_glv", "zkg_g1_fft_plan", "zkg_g1_fft_radix_products", "zkg_msm_workspace_bytes", "zkg_set_devices", "zkg_get_devices",
    "zkg_release", "zkg_comm_unique_id", "zkg_comm_init", "zkg_comm_destroy", "zkg_comm_rank", "zkg_comm_world",
    "zkg_comm_allgather", "zkg_comm_barrier", "zkg_comm_max_f64", "zkg_g1_comm_sum_partials",
    "zkg_g1_msm_device_sharded", "zkg_set_error_mode", "zkg_last_error",
]

_lib = None


def load():
    """Load the C-ABI library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"zkalgebra_gpu library not built: {LIB_PATH} (run __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        lib.zkg_version.restype = ctypes.c_char_p
        lib.zkg_device_malloc.restype = ctypes.c_void_p
        lib.zkg_device_malloc.argtypes = [ctypes.c_size_t]
        lib.zkg_device_free.argtypes = [ctypes.c_void_p]
        lib.zkg_memcpy_htod.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.zkg_memcpy_dtoh.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.zkg_g1_msm_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, U64P, ctypes.c_int]
        lib.zkg_ntt_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, U64P, ctypes.c_void_p,
                                       ctypes.c_void_p]
        lib.zkg_gen_fr.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, U64P]
        lib.zkg_gen_g1_points.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, U64P]
        lib.zkg_timer_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long)]
        lib.zkg_msm_set_group_limit.argtypes = [ctypes.c_size_t]
        lib.zkg_ntt_set_table_max.argtypes = [ctypes.c_size_t]
        lib.zkg_arena_set_limit.argtypes = [ctypes.c_size_t]
        lib.zkg_msm_workspace_bytes.restype = ctypes.c_size_t
        lib.zkg_msm_workspace_bytes.argtypes = [ctypes.c_int] * 7
        lib.zkg_set_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        lib.zkg_get_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        for c in CURVES:
            for o in ("is_valid", "is_zero", "is_one", "is_equal"):
                getattr(lib, f"{c}_arr_mont_{o}").restype = ctypes.c_uint8
            getattr(lib, f"{c}_poly_mont_quot_by_vanishing").restype = ctypes.c_uint8
        lib.zkg_arr_op_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, U64P, U64P, ctypes.c_void_p]
        lib.zkg_arr_dot_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, U64P]
        lib.zkg_arr_powers_device.argtypes = [ctypes.c_int, ctypes.c_int, U64P, U64P, ctypes.c_void_p]
        lib.zkg_last_error.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        lib.zkg_comm_unique_id.argtypes = [ctypes.c_void_p]
        lib.zkg_comm_init.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        lib.zkg_comm_allgather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.zkg_comm_max_f64.argtypes = [ctypes.POINTER(ctypes.c_double)]
        lib.zkg_g1_comm_sum_partials.argtypes = [ctypes.c_int, U64P, ctypes.c_int, U64P]
        lib.zkg_g1_msm_device_sharded.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, U64P]
        _lib = lib
    return _lib


def _p(a):
    if a.dtype != np.uint64 or not a.flags["C_CONTIGUOUS"]:
        raise TypeError("FlatArray buffers must be C-contiguous numpy.uint64 arrays")
    return a.ctypes.data_as(U64P)


def device_count():
    return load().zkg_device_count()


def require_gpu():
    if device_count() < 1:
        raise RuntimeError("zkalgebra_gpu: no GPU visible -- the MSM/NTT path is GPU-only (no CPU fallback)")


# ----------------------------------------------------------------------------- FFT subgroups

@dataclass(frozen=True)
class FFTSubgroup:
    """Mirror of ZK.Algebra.Class.FFT.FFTSubgroup (Class/FFT.hs:26-30): generator (Montgomery
    Fr, 4 limbs) of the multiplicative subgroup of order 2^log_size."""
    curve: str
    gen: tuple
    log_size: int

    @property
    def size(self):
        return 1 << self.log_size

    def gen_array(self):
        return np.array(self.gen, dtype=np.uint64)


def get_fft_subgroup(curve, log_size):
    """getFFTSubgroup (Class/FFT.hs:60-66): gen_m = fftDomain^(2^(M - m))."""
    if not (0 <= log_size <= FFT_LOG[curve]):
        raise ValueError("getFFTSubgroup: subgroup size is too large for this field")
    out = np.zeros(4, dtype=np.uint64)
    load().zkg_fft_generator(CURVE_ID[curve], log_size, _p(out))
    return FFTSubgroup(curve, tuple(int(x) for x in out), log_size)


# ----------------------------------------------------------------------------- MSM

def _check_msm(curve, coeffs, points):
    if coeffs.ndim != 2 or points.ndim != 2 or coeffs.shape[0] != points.shape[0]:
        raise ValueError("msm: incompatible array dimensions")   # G1/Proj.hs:239
    if points.shape[1] != 2 * NLIMBS_P[curve]:
        raise ValueError("msm: points must be affine (x, y) in Montgomery form")
    if coeffs.shape[1] < 1:
        raise ValueError("msm: coefficients need at least one limb")


def msm(curve, coeffs, points):
    """Proj.msm: Montgomery-form Fr coefficients x affine points -> projective G1 (normalised)."""
    _check_msm(curve, coeffs, points)
    require_gpu()
    out = np.zeros(3 * NLIMBS_P[curve], dtype=np.uint64)
    getattr(load(), f"{curve}_G1_proj_MSM_mont_coeff_proj_out")(
        coeffs.shape[0], _p(coeffs), _p(points), _p(out), coeffs.shape[1])
    return out


def msm_std(curve, coeffs, points):
    """Proj.msmStd: standard-form (plain integer) coefficients, used verbatim."""
    _check_msm(curve, coeffs, points)
    require_gpu()
    out = np.zeros(3 * NLIMBS_P[curve], dtype=np.uint64)
    getattr(load(), f"{curve}_G1_proj_MSM_std_coeff_proj_out")(
        coeffs.shape[0], _p(coeffs), _p(points), _p(out), coeffs.shape[1])
    return out


def msm_affine(curve, coeffs, points, std=False):
    """Affine.msm = toAffine . Proj.msm (G1/Affine.hs:143-149); infinity = all-0xFF."""
    _check_msm(curve, coeffs, points)
    require_gpu()
    out = np.zeros(2 * NLIMBS_P[curve], dtype=np.uint64)
    name = f"{curve}_G1_proj_MSM_{'std' if std else 'mont'}_coeff_affine_out"
    getattr(load(), name)(coeffs.shape[0], _p(coeffs), _p(points), _p(out), coeffs.shape[1])
    return out


def msm_variable(curve, coeffs, points, window_size):
    """<C>_G1_proj_MSM_std_coeff_proj_out_variable (exported, unbound by Haskell)."""
    _check_msm(curve, coeffs, points)
    require_gpu()
    out = np.zeros(3 * NLIMBS_P[curve], dtype=np.uint64)
    getattr(load(), f"{curve}_G1_proj_MSM_std_coeff_proj_out_variable")(
        coeffs.shape[0], _p(coeffs), _p(points), _p(out), coeffs.shape[1], int(window_size))
    return out


def msm_jac(curve, coeffs, points, std=False):
    """Jac.msm (G1/Jac.hs:225-259): Jacobian output, normalised; infinity = (1:1:0)."""
    _check_msm(curve, coeffs, points)
    require_gpu()
    out = np.zeros(3 * NLIMBS_P[curve], dtype=np.uint64)
    name = f"{curve}_G1_jac_MSM_{'std' if std else 'mont'}_coeff_jac_out"
    getattr(load(), name)(coeffs.shape[0], _p(coeffs), _p(points), _p(out), coeffs.shape[1])
    return out


def msm_jac_points(curve, coeffs, jac_points):
    """Jac's Curve.msm: msmJac cs gs = msm cs (batchToAffine gs) (G1/Jac.hs:188, 220), with the
    conversion on the GPU (<C>_G1_jac_batch_to_affine) instead of N serial CPU inversions."""
    if jac_points.ndim != 2 or jac_points.shape[1] != 3 * NLIMBS_P[curve]:
        raise ValueError("msm: incompatible array dimensions")
    return msm_jac(curve, coeffs, batch_to_affine(curve, jac_points, coords="jac"))


def msm_proj(curve, coeffs, proj_points):
    """Proj.msmProj cs gs = msm cs (batchToAffine gs) (G1/Proj.hs:222-223)."""
    if proj_points.ndim != 2 or proj_points.shape[1] != 3 * NLIMBS_P[curve]:
        raise ValueError("msm: incompatible array dimensions")
    # batchToAffine on the GPU (<C>_G1_proj_batch_to_affine, Montgomery's trick), as msmProj does
    return msm(curve, coeffs, batch_to_affine(curve, proj_points))


def g2_msm(curve, coeffs, points, std=False, affine=False):
    """G2 MSM (<C>_G2_proj_MSM_*_coeff_*_out): points are affine G2 (x0 x1 y0 y1, Montgomery Fp)"""
    if coeffs.ndim != 2 or points.ndim != 2 or coeffs.shape[0] != points.shape[0]:
        raise ValueError("msm: incompatible array dimensions")
    if points.shape[1] != 4 * NLIMBS_P[curve]:
        raise ValueError("msm: G2 points must be affine (x, y) over Fp2 in Montgomery form")
    require_gpu()
    out = np.zeros((4 if affine else 6) * NLIMBS_P[curve], dtype=np.uint64)
    name = f"{curve}_G2_proj_MSM_{'std' if std else 'mont'}_coeff_{'affine' if affine else 'proj'}_out"
    getattr(load(), name)(coeffs.shape[0], _p(coeffs), _p(points), _p(out), coeffs.shape[1])
    return out


def g1_to_affine(curve, proj):
    out = np.zeros(2 * NLIMBS_P[curve], dtype=np.uint64)
    load().zkg_g1_proj_to_affine(CURVE_ID[curve], _p(np.ascontiguousarray(proj)), _p(out))
    return out


def g1_normalize(curve, proj):
    out = np.zeros(3 * NLIMBS_P[curve], dtype=np.uint64)
    load().zkg_g1_proj_normalize(CURVE_ID[curve], _p(np.ascontiguousarray(proj)), _p(out))
    return out


def g1_add(curve, a, b):
    out = np.zeros(3 * NLIMBS_P[curve], dtype=np.uint64)
    load().zkg_g1_proj_add(CURVE_ID[curve], _p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), _p(out))
    return out


def batch_from_affine(curve, aff, coords="proj"):
    """Proj.batchFromAffine (G1/Proj.hs:409-418); coords="jac": Jac.batchFromAffine (G1/Jac.hs:374-380),
    infinity -> (1 : 1 : 0)"""
    aff = np.ascontiguousarray(aff, dtype=np.uint64)
    out = np.zeros((aff.shape[0], 3 * NLIMBS_P[curve]), dtype=np.uint64)
    require_gpu()
    getattr(load(), f"{curve}_G1_{_coords(coords)}_batch_from_affine")(aff.shape[0], _p(aff), _p(out))
    return out


def batch_to_affine(curve, proj, coords="proj"):
    """Proj.batchToAffine (G1/Proj.hs:420-430); coords="jac": Jac.batchToAffine (G1/Jac.hs:382-389);
    infinity -> all-0xFF"""
    proj = np.ascontiguousarray(proj, dtype=np.uint64)
    out = np.zeros((proj.shape[0], 2 * NLIMBS_P[curve]), dtype=np.uint64)
    require_gpu()
    getattr(load(), f"{curve}_G1_{_coords(coords)}_batch_to_affine")(proj.shape[0], _p(proj), _p(out))
    return out


def _coords(coords):
    if coords not in ("proj", "jac"):
        raise ValueError(f"coords must be 'proj' or 'jac', not {coords!r}")
    return coords


def _curve_fft(sg, pts, name, msg, coords):
    pts = np.ascontiguousarray(pts, dtype=np.uint64)
    if pts.ndim != 2 or sg.size != pts.shape[0]:
        raise ValueError(msg)
    require_gpu()
    out = np.zeros_like(pts)
    getattr(load(), f"{sg.curve}_G1_{_coords(coords)}_{name}")(sg.log_size, _p(sg.gen_array()), _p(pts), _p(out))
    return out


def forward_fft(sg, pts, coords="proj"):
    """Proj.forwardFFT = curveFFT (G1/Proj.hs:270-281; Jacobian: G1/Jac.hs:266-276):
    [L_k(tau)] -> [tau^i] points, normalised"""
    return _curve_fft(sg, pts, "fft_forward", "forwardNTT: subgroup size differs from the array size", coords)


def inverse_fft(sg, pts, coords="proj"):
    """Proj.inverseFFT = curveIFFT (G1/Proj.hs:283-294; Jacobian: G1/Jac.hs:278-288):
    [tau^i] -> [L_k(tau)] points, normalised"""
    return _curve_fft(sg, pts, "fft_inverse", "inverseNTT: subgroup size differs from the array size", coords)


curve_fft = forward_fft
curve_ifft = inverse_fft


# ----------------------------------------------------------------------------- NTT

def forward_ntt(sg, poly):
    """Poly.forwardNTT: evaluations f(gen^k), k = 0..n-1 (Poly.hs:400-410)."""
    if poly.ndim != 2 or sg.size != poly.shape[0]:
        raise ValueError("forwardNTT: subgroup size differs from the array size")   # Poly.hs:403
    require_gpu()
    out = np.empty_like(poly)  # every element is written (as the binding's mallocForeignPtrArray)
    getattr(load(), f"{sg.curve}_poly_mont_ntt_forward")(sg.log_size, _p(sg.gen_array()), _p(poly), _p(out))
    return out


def inverse_ntt(sg, values):
    """Poly.inverseNTT: interpolation (Poly.hs:412-422)."""
    if values.ndim != 2 or sg.size != values.shape[0]:
        raise ValueError("inverseNTT: subgroup size differs from the array size")   # Poly.hs:415
    require_gpu()
    out = np.empty_like(values)  # every element is written
    getattr(load(), f"{sg.curve}_poly_mont_ntt_inverse")(sg.log_size, _p(sg.gen_array()), _p(values), _p(out))
    return out


# UnivariateFFT instance (Poly.hs:424-426)
ntt = forward_ntt
intt = inverse_ntt


# ----------------------------------------------------------------------------- Fr vectors

def _fr(a):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    if a.ndim != 2 or a.shape[1] != NLIMBS_R:
        raise TypeError("FlatArray Fr must have shape (n, 4)")
    return a


def _same(name, *arrs):
    if any(x.shape[0] != arrs[0].shape[0] for x in arrs):
        raise ValueError(f"{name}: incompatible input array lengths")   # Array.hs:217-360


def _arr(curve, op):
    require_gpu()
    return getattr(load(), f"{curve}_arr_mont_{op}")


def arr_is_valid(curve, a):
    a = _fr(a)
    return bool(_arr(curve, "is_valid")(a.shape[0], _p(a)))


def arr_is_zero(curve, a):
    a = _fr(a)
    return bool(_arr(curve, "is_zero")(a.shape[0], _p(a)))


def arr_is_one(curve, a):
    a = _fr(a)
    return bool(_arr(curve, "is_one")(a.shape[0], _p(a)))


def arr_is_equal(curve, a, b):
    a, b = _fr(a), _fr(b)
    _same("isEqual", a, b)
    return bool(_arr(curve, "is_equal")(a.shape[0], _p(a), _p(b)))


def _unary(curve, op, a):
    a = _fr(a)
    out = np.zeros_like(a)
    _arr(curve, op)(a.shape[0], _p(a), _p(out))
    return out


def _binary(curve, op, name, a, b):
    a, b = _fr(a), _fr(b)
    _same(name, a, b)
    out = np.zeros_like(a)
    _arr(curve, op)(a.shape[0], _p(a), _p(b), _p(out))
    return out


def arr_from_std(curve, a): return _unary(curve, "from_std", a)
def arr_to_std(curve, a): return _unary(curve, "to_std", a)
def arr_neg(curve, a): return _unary(curve, "neg", a)
def arr_sqr(curve, a): return _unary(curve, "sqr", a)
def arr_inv(curve, a): return _unary(curve, "inv", a)
def arr_add(curve, a, b): return _binary(curve, "add", "add", a, b)
def arr_sub(curve, a, b): return _binary(curve, "sub", "sub", a, b)
def arr_mul(curve, a, b): return _binary(curve, "mul", "mul", a, b)
def arr_div(curve, a, b): return _binary(curve, "div", "div", a, b)


def arr_append(curve, a, b):
    a, b = _fr(a), _fr(b)
    out = np.zeros((a.shape[0] + b.shape[0], 4), dtype=np.uint64)
    _arr(curve, "append")(a.shape[0], b.shape[0], _p(a), _p(b), _p(out))
    return out


def arr_cons(curve, x, a): return arr_append(curve, np.asarray(x, dtype=np.uint64).reshape(1, 4), a)
def arr_snoc(curve, a, y): return arr_append(curve, a, np.asarray(y, dtype=np.uint64).reshape(1, 4))


def arr_scale(curve, k, a):
    a = _fr(a)
    out = np.zeros_like(a)
    _arr(curve, "scale")(a.shape[0], _p(np.ascontiguousarray(k, dtype=np.uint64)), _p(a), _p(out))
    return out


def arr_dot_prod(curve, a, b):
    a, b = _fr(a), _fr(b)
    _same("dotProd", a, b)
    out = np.zeros(4, dtype=np.uint64)
    _arr(curve, "dot_prod")(a.shape[0], _p(a), _p(b), _p(out))
    return out


def arr_powers(curve, a, b, n):
    """powers a b n = [a b^i | i <- [0..n-1]] (Array.hs:99)"""
    out = np.zeros((n, 4), dtype=np.uint64)
    _arr(curve, "powers")(n, _p(np.ascontiguousarray(a, dtype=np.uint64)),
                          _p(np.ascontiguousarray(b, dtype=np.uint64)), _p(out))
    return out


def _fused(curve, op, name, a, b, c):
    a, b, c = _fr(a), _fr(b), _fr(c)
    _same(name, a, b, c)
    out = np.zeros_like(a)
    _arr(curve, op)(a.shape[0], _p(a), _p(b), _p(c), _p(out))
    return out


def arr_mul_add(curve, a, b, c): return _fused(curve, "mul_add", "mulAdd", a, b, c)
def arr_mul_sub(curve, a, b, c): return _fused(curve, "mul_sub", "mulSub", a, b, c)


def arr_lin_comb1(curve, ax, y):
    """linComb1 (a, x) y = a x + y (Array.hs:135-146)"""
    (a, x), y = ax, _fr(y)
    x = _fr(x)
    if x.shape[0] != y.shape[0]:
        raise ValueError("linComb1: incompatible vector dimensions")
    out = np.zeros_like(x)
    _arr(curve, "Ax_plus_y")(x.shape[0], _p(np.ascontiguousarray(a, dtype=np.uint64)), _p(x), _p(y), _p(out))
    return out


def arr_lin_comb2(curve, ax, by):
    """linComb2 (a, x) (b, y) = a x + b y (Array.hs:148-161)"""
    (a, x), (b, y) = ax, by
    x, y = _fr(x), _fr(y)
    if x.shape[0] != y.shape[0]:
        raise ValueError("linComb2: incompatible vector dimensions")
    out = np.zeros_like(x)
    _arr(curve, "Ax_plus_By")(x.shape[0], _p(np.ascontiguousarray(a, dtype=np.uint64)),
                              _p(np.ascontiguousarray(b, dtype=np.uint64)), _p(x), _p(y), _p(out))
    return out


def div_by_vanishing(curve, poly, expo_n, eta):
    """Poly.divByVanishing (Poly.hs:367-380): (quotient, remainder) by x^n - eta."""
    poly = _fr(poly)
    n1 = poly.shape[0]
    nq, nr = max(0, n1 - expo_n), max(0, expo_n)
    q = np.zeros((nq, 4), dtype=np.uint64)
    r = np.zeros((nr, 4), dtype=np.uint64)
    require_gpu()
    getattr(load(), f"{curve}_poly_mont_div_by_vanishing")(n1, _p(poly), expo_n,
                                                            _p(np.ascontiguousarray(eta, dtype=np.uint64)),
                                                            nq, _p(q), nr, _p(r))
    return q, r


def quot_by_vanishing(curve, poly, expo_n, eta):
    """Poly.quotByVanishing (Poly.hs:383-397): the quotient, or None if the remainder is nonzero."""
    poly = _fr(poly)
    n1 = poly.shape[0]
    nq = max(0, n1 - expo_n)
    q = np.zeros((nq, 4), dtype=np.uint64)
    require_gpu()
    ok = getattr(load(), f"{curve}_poly_mont_quot_by_vanishing")(n1, _p(poly), expo_n,
                                                                  _p(np.ascontiguousarray(eta, dtype=np.uint64)),
                                                                  nq, _p(q))
    return q if ok else None


ARR_OP_CODE = {"neg": 0, "add": 1, "sub": 2, "sub_rev": 3, "sqr": 4, "mul": 5, "mul_add": 6, "mul_sub": 7,
               "scale": 8, "Ax_plus_y": 9, "Ax_plus_By": 10, "from_std": 11, "to_std": 12, "copy": 13,
               "set_const": 14, "inv": 15, "div": 16}


# ----------------------------------------------------------------------------- synthetic inputs

def gen_fr(curve, seed, count, start=0):
    out = np.zeros((count, 4), dtype=np.uint64)
    load().zkg_gen_fr(CURVE_ID[curve], seed, start, count, _p(out))
    return out


def gen_points(curve, seed, count, start=0):
    out = np.zeros((count, 2 * NLIMBS_P[curve]), dtype=np.uint64)
    load().zkg_gen_g1_points(CURVE_ID[curve], seed, start, count, _p(out))
    return out


# ----------------------------------------------------------------------------- device-resident helpers

class DeviceBuffer:
    """HBM buffer owned by the library's allocator (used by bench.py and the multi-GPU path)."""

    def __init__(self, host_array):
        self.nbytes = host_array.nbytes
        self.ptr = load().zkg_device_malloc(max(1, self.nbytes))
        load().zkg_memcpy_htod(self.ptr, host_array.ctypes.data, self.nbytes)

    @classmethod
    def empty(cls, nbytes):
        self = cls.__new__(cls)
        self.nbytes = nbytes
        self.ptr = load().zkg_device_malloc(max(1, nbytes))
        return self

    def to_host(self, like):
        out = np.empty_like(like)
        load().zkg_memcpy_dtoh(out.ctypes.data, self.ptr, self.nbytes)
        return out

    def free(self):
        if self.ptr:
            load().zkg_device_free(self.ptr)
            self.ptr = None


def msm_device(curve, n, d_scalars, d_points, mont=True, window=0, nlimbs=4):
    out = np.zeros(3 * NLIMBS_P[curve], dtype=np.uint64)
    load().zkg_g1_msm_device(CURVE_ID[curve], n, d_scalars.ptr, nlimbs, 1 if mont else 0, d_points.ptr, _p(out),
                             window)
    return out


def msm_profile(on):
    """per-phase HIP-event timing of every MSM call, printed to stderr"""
    load().zkg_msm_profile(1 if on else 0)


def msm_set_ysum_mode(mode):
    """test hook: G1 Y-sum kernel (-1 by size, 0 k_ysum2, 1 k_ysum3)"""
    load().zkg_msm_set_ysum_mode(int(mode))


def msm_set_ahead_min(lg):
    """test hook: sort-ahead window groups from 2^lg device-resident pairs (0 off, -1 default)"""
    load().zkg_msm_set_ahead_min(int(lg))


def msm_set_group_limit(entries):
    """test hook: max sorted entries per MSM pipeline pass (0 = default 2^30)"""
    load().zkg_msm_set_group_limit(int(entries))


def ntt_set_max_radix(r):
    """test hook: NTT pass split -- 12: two passes for 2^17..2^24, 8: <= 2^8-point passes, 0: default"""
    load().zkg_ntt_set_max_radix(int(r))


def arr_op_device(curve, op, n, d_a, d_b=None, d_c=None, kA=None, kB=None, d_tgt=None):
    """device-resident Fr vector op (zkg_arr_op_device); d_* are DeviceBuffers"""
    z = np.zeros(4, dtype=np.uint64)
    ka = np.ascontiguousarray(kA if kA is not None else z, dtype=np.uint64)
    kb = np.ascontiguousarray(kB if kB is not None else z, dtype=np.uint64)
    load().zkg_arr_op_device(CURVE_ID[curve], ARR_OP_CODE[op], n, d_a.ptr if d_a else None,
                             d_b.ptr if d_b else None, d_c.ptr if d_c else None, _p(ka), _p(kb), d_tgt.ptr)


def ntt_device(curve, m, gen, d_src, d_dst, inverse=False):
    load().zkg_ntt_device(CURVE_ID[curve], 1 if inverse else 0, m, _p(np.ascontiguousarray(gen)), d_src.ptr,
                          d_dst.ptr)


def ntt_set_table_max(entries):
    """test hook: inter-pass twiddle entries above which NTT passes compute twiddles on the fly (0: default)"""
    load().zkg_ntt_set_table_max(int(entries))


def arena_set_limit(nbytes):
    """test hook: cap on one working-set arena's device bytes (0: unlimited)"""
    load().zkg_arena_set_limit(int(nbytes))


def msm_last_groups():
    return load().zkg_msm_last_groups()


def g1_fft_plan(curve, m):
    """bits per Stockham radix-2^b GLV stage of a 2^m group FFT ([] = the fused radix-2 stages)"""
    bits = (ctypes.c_int * 32)()
    k = load().zkg_g1_fft_plan(CURVE_ID[curve], m, bits, 32)
    return list(bits[:k])


def g1_fft_glv_products(curve, m, inverse=False):
    """GLV lane-pair scalar multiplications one 2^m group FFT runs on subgroup inputs (the fused
    radix-2 stages: N/2 per stage, minus the j = 0 butterflies; the inverse's first stage: N; the
    radix-2^b stages: D_b N / 2^b per stage, the few unit-twiddle products (a copy) included)"""
    n = 1 << m
    plan = g1_fft_plan(curve, m)
    if not plan:
        per = [n // 2 - (n >> s) for s in range(1, m + 1)]  # the N / 2^s j = 0 butterflies copy
        if inverse:
            per[-1] = n  # the first inverse stage (s = m) multiplies both outputs (N^-1 folded in)
        return sum(per)
    lib = load()
    tot = 0
    for i, b in enumerate(plan):
        tot += lib.zkg_g1_fft_radix_products(b) * (n >> b) + ((n >> b) if inverse and i == 0 else 0)
    return tot


def g1_fft_last_glv():
    """1 when the most recent group FFT ran the GLV stages (all inputs in the order-r subgroup)"""
    return load().zkg_g1_fft_last_glv()


def msm_workspace_bytes(curve, n, nlimbs=4, mont=True, host_inputs=True, window=0, groups=1):
    """device bytes of one G1 MSM's working set with its windows in `groups` passes"""
    return load().zkg_msm_workspace_bytes(CURVE_ID[curve], n, nlimbs, 1 if mont else 0, 1 if host_inputs else 0,
                                          window, groups)


def set_devices(ids):
    """device set of the host-buffer MSM entries (zkg_set_devices); [] = calling thread's device"""
    ids = list(ids)
    arr = (ctypes.c_int * max(1, len(ids)))(*ids)
    if load().zkg_set_devices(arr, len(ids)) != 0:
        raise ValueError(f"set_devices: invalid device id in {ids}")


def get_devices():
    arr = (ctypes.c_int * 64)()
    n = load().zkg_get_devices(arr, 64)
    return list(arr[:min(n, 64)])


def set_error_mode(recoverable):
    """zkg_set_error_mode: False = abort on a device error (default), True = the failing call
    returns and last_error() reports it"""
    load().zkg_set_error_mode(1 if recoverable else 0)


def last_error():
    """the calling thread's last recorded library error (cleared), or None"""
    buf = ctypes.create_string_buffer(512)
    return buf.value.decode() if load().zkg_last_error(buf, 512) else None


def release():
    """free every device buffer the library caches (zkg_release)"""
    load().zkg_release()


def timer(enable=None, reset=False):
    lib = load()
    if enable is not None:
        lib.zkg_timer_enable(1 if enable else 0)
    if reset:
        lib.zkg_timer_reset()
    ms = ctypes.c_double()
    n = ctypes.c_long()
    lib.zkg_timer_read(ctypes.byref(ms), ctypes.byref(n))
    return ms.value, n.value
