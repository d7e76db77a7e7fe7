"""ctypes bindings to the two CPU checkers -- TEST INFRASTRUCTURE ONLY.

* ``Oracle``     -- oracle/liboracle.so, our C restatement of the reference algorithm
                   (oracle/zk_oracle.c; cites reference file:line per function).
* ``Reference``  -- oracle/_ref/libzkref.so, the reference's own generated C
                   (lib/cbits of bkomuves/zikkurat-algebra) compiled in place by
                   oracle/Makefile.  Present in this container and, prebuilt, on the
                   GPU box; absent elsewhere (then ``Reference.available()`` is False).

Never imported by the product package (zikkurat-algebra_amd/).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
U64P = ctypes.POINTER(ctypes.c_uint64)
CURVES = {"bn128": 0, "bls12_381": 1}
NP = {"bn128": 4, "bls12_381": 6}


def _p(a):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(U64P)


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE, "oracle"])
    if os.path.isdir("/root/reference/lib/cbits"):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


class Oracle:
    """Our CPU restatement (C)."""

    def __init__(self, path=None):
        path = path or os.path.join(HERE, "liboracle.so")
        self.lib = ctypes.CDLL(path)
        self.lib.zko_init()

    def _c(self, curve):
        return CURVES[curve]

    def msm(self, curve, scalars, points, mont=True, out="affine", window=None):
        n = scalars.shape[0]
        nl = scalars.shape[1] if scalars.ndim == 2 else 4
        if out == "affine":
            res = np.zeros(2 * NP[curve], dtype=np.uint64)
            f = self.lib.zko_msm_mont_affine if mont else self.lib.zko_msm_std_affine
            f(self._c(curve), n, _p(scalars), _p(points), _p(res), nl)
            return res
        res = np.zeros(3 * NP[curve], dtype=np.uint64)
        if window is not None:
            assert not mont
            self.lib.zko_msm_std_proj_variable(self._c(curve), n, _p(scalars), _p(points), _p(res), nl, window)
        else:
            f = self.lib.zko_msm_mont_proj if mont else self.lib.zko_msm_std_proj
            f(self._c(curve), n, _p(scalars), _p(points), _p(res), nl)
        return res

    def msm_naive(self, curve, std_scalars, points):
        res = np.zeros(2 * NP[curve], dtype=np.uint64)
        self.lib.zko_msm_naive_affine(self._c(curve), std_scalars.shape[0], _p(std_scalars), _p(points), _p(res),
                                      std_scalars.shape[1])
        return res

    def ntt(self, curve, m, gen, src, inverse=False):
        out = np.zeros_like(src)
        f = self.lib.zko_ntt_inverse if inverse else self.lib.zko_ntt_forward
        f(self._c(curve), m, _p(gen), _p(src), _p(out))
        return out

    def normalize(self, curve, proj):
        out = np.zeros(3 * NP[curve], dtype=np.uint64)
        self.lib.zko_proj_normalize(self._c(curve), _p(np.ascontiguousarray(proj)), _p(out))
        return out

    def to_affine(self, curve, proj):
        out = np.zeros(2 * NP[curve], dtype=np.uint64)
        self.lib.zko_proj_to_affine(self._c(curve), _p(np.ascontiguousarray(proj)), _p(out))
        return out

    def proj_add(self, curve, a, b):
        out = np.zeros(3 * NP[curve], dtype=np.uint64)
        self.lib.zko_proj_add(self._c(curve), _p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), _p(out))
        return out

    def to_std(self, fld, a):
        out = np.zeros_like(a)
        for i in range(a.shape[0]):
            self.lib.zko_to_std(fld, _p(a[i]), _p(out[i]))
        return out

    def gen_fr(self, curve, seed, start, count):
        out = np.zeros((count, 4), dtype=np.uint64)
        self.lib.zko_gen_fr(self._c(curve), ctypes.c_uint64(seed), ctypes.c_int64(start), ctypes.c_int64(count),
                            _p(out))
        return out

    def gen_points(self, curve, seed, start, count):
        out = np.zeros((count, 2 * NP[curve]), dtype=np.uint64)
        self.lib.zko_gen_g1_points(self._c(curve), ctypes.c_uint64(seed), ctypes.c_int64(start),
                                   ctypes.c_int64(count), _p(out))
        return out

    ARR_OP = {"neg": 0, "add": 1, "sub": 2, "sub_rev": 3, "sqr": 4, "mul": 5, "mul_add": 6, "mul_sub": 7,
              "scale": 8, "Ax_plus_y": 9, "Ax_plus_By": 10, "from_std": 11, "to_std": 12, "copy": 13,
              "set_const": 14, "inv": 15, "div": 16}

    def arr_op(self, curve, op, n, a=None, b=None, c=None, kA=None, kB=None):
        out = np.zeros((n, 4), dtype=np.uint64)
        z = np.zeros((max(n, 1), 4), dtype=np.uint64)
        k0 = np.zeros(4, dtype=np.uint64)
        arg = lambda x, d: _p(np.ascontiguousarray(x if x is not None else d, dtype=np.uint64))
        self.lib.zko_arr_op(self._c(curve), self.ARR_OP[op], n, arg(a, z), arg(b, z), arg(c, z), arg(kA, k0),
                            arg(kB, k0), _p(out))
        return out

    def arr_dot(self, curve, a, b):
        out = np.zeros(4, dtype=np.uint64)
        self.lib.zko_arr_dot(self._c(curve), a.shape[0], _p(a), _p(b), _p(out))
        return out

    def arr_powers(self, curve, kA, kB, n):
        out = np.zeros((n, 4), dtype=np.uint64)
        self.lib.zko_arr_powers(self._c(curve), n, _p(np.ascontiguousarray(kA)), _p(np.ascontiguousarray(kB)),
                                _p(out))
        return out

    def div_by_vanishing(self, curve, poly, n, eta):
        n1 = poly.shape[0]
        nq, nr = max(0, n1 - n), max(0, n)
        q = np.zeros((max(nq, 1), 4), dtype=np.uint64)
        r = np.zeros((max(nr, 1), 4), dtype=np.uint64)
        ok = self.lib.zko_div_by_vanishing(self._c(curve), n1, _p(poly), n, _p(np.ascontiguousarray(eta)), nq,
                                           _p(q), nr, _p(r))
        return q[:nq], r[:nr], bool(ok)

    def fft_generator(self, curve, m):
        out = np.zeros(4, dtype=np.uint64)
        self.lib.zko_fft_generator(self._c(curve), m, _p(out))
        return out


class Reference:
    """The reference's own generated C (lib/cbits), compiled in place."""

    PATH = os.path.join(HERE, "_ref", "libzkref.so")

    @classmethod
    def available(cls):
        return os.path.exists(cls.PATH)

    def __init__(self):
        self.lib = ctypes.CDLL(self.PATH)

    def msm(self, curve, scalars, points, mont=True, out="affine", window=None):
        n = scalars.shape[0]
        nl = scalars.shape[1]
        if out == "affine":
            res = np.zeros(2 * NP[curve], dtype=np.uint64)
            name = f"{curve}_G1_proj_MSM_{'mont' if mont else 'std'}_coeff_affine_out"
            getattr(self.lib, name)(n, _p(scalars), _p(points), _p(res), nl)
            return res
        res = np.zeros(3 * NP[curve], dtype=np.uint64)
        if window is not None:
            getattr(self.lib, f"{curve}_G1_proj_MSM_std_coeff_proj_out_variable")(
                n, _p(scalars), _p(points), _p(res), nl, window)
        else:
            name = f"{curve}_G1_proj_MSM_{'mont' if mont else 'std'}_coeff_proj_out"
            getattr(self.lib, name)(n, _p(scalars), _p(points), _p(res), nl)
        return res

    def msm_jac(self, curve, scalars, points, mont=True):
        """<C>_G1_jac_MSM_{mont,std}_coeff_jac_out (raw Jacobian output)"""
        res = np.zeros(3 * NP[curve], dtype=np.uint64)
        name = f"{curve}_G1_jac_MSM_{'mont' if mont else 'std'}_coeff_jac_out"
        getattr(self.lib, name)(scalars.shape[0], _p(scalars), _p(points), _p(res), scalars.shape[1])
        return res

    def ntt(self, curve, m, gen, src, inverse=False):
        out = np.zeros_like(src)
        name = f"{curve}_poly_mont_ntt_{'inverse' if inverse else 'forward'}"
        getattr(self.lib, name)(m, _p(gen), _p(src), _p(out))
        return out

    def proj_add(self, curve, a, b):
        out = np.zeros(3 * NP[curve], dtype=np.uint64)
        getattr(self.lib, f"{curve}_G1_proj_add")(_p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)),
                                                  _p(out))
        return out

    def to_affine(self, curve, proj):
        out = np.zeros(2 * NP[curve], dtype=np.uint64)
        getattr(self.lib, f"{curve}_G1_proj_to_affine")(_p(np.ascontiguousarray(proj)), _p(out))
        return out

    def normalize(self, curve, proj):
        out = np.zeros(3 * NP[curve], dtype=np.uint64)
        getattr(self.lib, f"{curve}_G1_proj_normalize")(_p(np.ascontiguousarray(proj)), _p(out))
        return out

    def arr(self, curve, name, *args, restype=None):
        """call <curve>_arr_mont_<name> / <curve>_poly_mont_<name> with numpy / int arguments"""
        f = getattr(self.lib, f"{curve}_{name}")
        if restype is not None:
            f.restype = restype
        conv = [_p(np.ascontiguousarray(a)) if isinstance(a, np.ndarray) else a for a in args]
        return f(*conv)
