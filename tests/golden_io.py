"""Loading helpers for tests/golden (data only: numpy .npz without pickle, JSON)."""
import json
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


P_BLS = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
FP_ID = {"bn128": 0, "bls12_381": 2}  # oracle field ids of the base fields


def _limbs(x, n):
    return np.array([(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)], dtype=np.uint64)


def projective_points(zk, oracle, curve, n, seed, n_inf=3):
    """n projective points (X:Y:Z) = (x l : y l : l) of the order-r subgroup with random l (the
    generator's points scaled by random field elements), a few at infinity as (0 : l : 0).
    Deterministic: the same rows here, in the GPU tests and in tools/make_golden.py."""
    import ctypes
    import random

    def ptr(a):
        return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    NP = zk.NLIMBS_P[curve]
    aff = zk.gen_points(curve, seed, n)
    lam = zk.gen_points(curve, seed + 1, n)[:, :NP]  # random field elements (canonical)
    out = np.zeros((n, 3 * NP), dtype=np.uint64)
    for i in range(n):
        for k in range(2):
            x = np.ascontiguousarray(aff[i, k * NP:(k + 1) * NP])
            o = np.zeros(NP, dtype=np.uint64)
            oracle.lib.zko_fmul(FP_ID[curve], ptr(x), ptr(np.ascontiguousarray(lam[i])), ptr(o))
            out[i, k * NP:(k + 1) * NP] = o
        out[i, 2 * NP:] = lam[i]
    rng = random.Random(seed)
    for i in rng.sample(range(n), min(n_inf, n)):
        out[i] = 0
        out[i, NP:2 * NP] = lam[i]  # (0 : y : 0) with arbitrary y is infinity too
    return out


def jacobian_points(zk, oracle, curve, n, seed, n_inf=3, affine=None):
    """n Jacobian points (X:Y:Z) = (x l^2 : y l^3 : l) with random l (the generator's points, or the
    given affine rows), a few at infinity as the reference's Jacobian infinity (l^2 : l^3 : 0)
    (Y^2 = X^3, X, Y != 0: bls12_381_G1_jac.c:164-180).  Deterministic, like projective_points."""
    import ctypes
    import random

    def ptr(a):
        return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    NP = zk.NLIMBS_P[curve]
    aff = zk.gen_points(curve, seed, n) if affine is None else affine
    lam = zk.gen_points(curve, seed + 1, n)[:, :NP]  # random field elements (canonical)
    out = np.zeros((n, 3 * NP), dtype=np.uint64)
    fid = FP_ID[curve]
    for i in range(n):
        l1 = np.ascontiguousarray(lam[i])
        l2 = np.zeros(NP, dtype=np.uint64)
        l3 = np.zeros(NP, dtype=np.uint64)
        oracle.lib.zko_fmul(fid, ptr(l1), ptr(l1), ptr(l2))
        oracle.lib.zko_fmul(fid, ptr(l2), ptr(l1), ptr(l3))
        for k, lk in ((0, l2), (1, l3)):
            x = np.ascontiguousarray(aff[i, k * NP:(k + 1) * NP])
            o = np.zeros(NP, dtype=np.uint64)
            oracle.lib.zko_fmul(fid, ptr(x), ptr(lk), ptr(o))
            out[i, k * NP:(k + 1) * NP] = o
        out[i, 2 * NP:] = l1
    rng = random.Random(seed)
    for i in rng.sample(range(n), min(n_inf, n)):
        l1 = np.ascontiguousarray(lam[i])
        l2 = np.zeros(NP, dtype=np.uint64)
        l3 = np.zeros(NP, dtype=np.uint64)
        oracle.lib.zko_fmul(fid, ptr(l1), ptr(l1), ptr(l2))
        oracle.lib.zko_fmul(fid, ptr(l2), ptr(l1), ptr(l3))
        out[i, :NP] = l2
        out[i, NP:2 * NP] = l3
        out[i, 2 * NP:] = 0
    return out


def g2_points(reflib, curve, n, k0=12345, k1=67890, n_inf=0, seed=0):
    """n DISTINCT affine G2 points P0 + i H (P0 = k0 G, H = k1 G, the reference's own G2 generator,
    scl_small, add and batch_to_affine: oracle/_ref), n_inf of them replaced by the all-0xFF
    affine infinity at positions drawn with `seed`.  Used by the G2 tests and tools/make_golden.py."""
    import ctypes
    import random
    NP = {"bn128": 4, "bls12_381": 6}[curve]
    lib = reflib
    gen = np.ctypeslib.as_array((ctypes.c_uint64 * (6 * NP)).in_dll(lib, f"{curve}_G2_proj_gen_G2")).copy()
    scl = getattr(lib, f"{curve}_G2_proj_scl_small")
    scl.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    p0, h = np.zeros(6 * NP, np.uint64), np.zeros(6 * NP, np.uint64)
    scl(k0, gen.ctypes.data, p0.ctypes.data)
    scl(k1, gen.ctypes.data, h.ctypes.data)
    proj = np.zeros((n, 6 * NP), np.uint64)
    add = getattr(lib, f"{curve}_G2_proj_add")
    add.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    if n:
        proj[0] = p0
    hp = h.ctypes.data
    base = proj.ctypes.data
    row = 6 * NP * 8
    for i in range(1, n):
        add(base + (i - 1) * row, hp, base + i * row)
    aff = np.zeros((n, 4 * NP), np.uint64)
    f = getattr(lib, f"{curve}_G2_proj_batch_to_affine")
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    f(n, proj.ctypes.data, aff.ctypes.data)
    if n_inf:
        rng = random.Random(seed)
        aff[rng.sample(range(n), n_inf)] = np.uint64(0xFFFFFFFFFFFFFFFF)
    return aff


def g2_case_inputs(reflib, curve, logn, seed, gen_fr):
    """scalars (Montgomery, 1/1000 zero rows) and 2^logn distinct affine G2 points (1/4096 at
    infinity) of one tools/make_golden.py G2_CASES row; shared by the generator and the tests"""
    n = 1 << logn
    pts = g2_points(reflib, curve, n, k0=seed & 0xFFFF, k1=(seed >> 4) + 77, n_inf=n >> 12, seed=seed)
    sc = gen_fr(curve, seed, n)
    rng = np.random.default_rng(seed)
    sc[rng.choice(n, n // 1000, replace=False)] = 0
    return sc, pts


def g2_large_golden():
    """reference G2 MSM outputs at 2^16 / 2^18 (tools/make_golden.py g2large)"""
    p = os.path.join(GOLD, "g2_msm.json")
    return json.load(open(p)) if os.path.exists(p) else {}


def bls_nonsubgroup_points(n, seed):
    """random affine points of E(Fp): y^2 = x^3 + 4, almost surely outside the order-r subgroup
    (cofactor h ~ 2^126); Montgomery form (R = 2^384)"""
    import random
    rng = random.Random(seed)
    R = 1 << 384
    pts = []
    while len(pts) < n:
        x = rng.randrange(P_BLS)
        rhs = (x * x * x + 4) % P_BLS
        y = pow(rhs, (P_BLS + 1) // 4, P_BLS)
        if y * y % P_BLS != rhs:
            continue
        pts.append(np.concatenate([_limbs(x * R % P_BLS, 6), _limbs(y * R % P_BLS, 6)]))
    return np.stack(pts)


def group_fft_golden():
    """reference digests of the group FFT at KZG SRS sizes (tools/make_golden.py groupfft)"""
    p = os.path.join(GOLD, "group_fft.json")
    return json.load(open(p)) if os.path.exists(p) else {}


def msm_cases(curve):
    z = np.load(os.path.join(GOLD, f"msm_{curve}.npz"), allow_pickle=False)
    for name in z["names"]:
        name = str(name)
        yield (name, z[f"{name}__scalars"], z[f"{name}__points"], bool(z[f"{name}__mont"][0]),
               z[f"{name}__affine"], z[f"{name}__proj_normalized"])


def ntt_cases(curve):
    z = np.load(os.path.join(GOLD, f"ntt_{curve}.npz"), allow_pickle=False)
    ms = sorted({int(k.split("__")[0][1:]) for k in z.files})
    for m in ms:
        yield m, z[f"m{m}__gen"], z[f"m{m}__input"], z[f"m{m}__forward"], z[f"m{m}__inverse"]


def skew_scalars(gen_fr, curve, seed, n, kind):
    """skewed scalar vectors of the large-sort tests (tests/test_gpu_msm.py, golden outputs from
    tools/make_golden.py): "mix3" = three Fr values (Montgomery) drawn uniformly, 5 % zeros;
    "binary" = Montgomery 0 / 1 (each with probability 1/2)"""
    rng = np.random.default_rng(seed)
    if kind == "mix3":
        vals = gen_fr(curve, seed + 1, 3)
        sc = vals[rng.integers(0, 3, n)].copy()
        sc[rng.random(n) < 0.05] = 0
        return sc
    m1 = mont_one(curve)
    one = np.array([(m1 >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)
    sc = np.zeros((n, 4), dtype=np.uint64)
    sc[rng.random(n) < 0.5] = one
    return sc


def baseline_configs():
    p = os.path.join(GOLD, "baseline_configs.json")
    return json.load(open(p)) if os.path.exists(p) else {}


# --------------------------------------------------------------------------- adversarial NTT inputs
# Raw Montgomery words chosen to drive the lazy butterflies and the closing reduction to their
# extremes (largest canonical limbs, sign flips between neighbours, all-zero columns).  Shared by
# tools/make_golden.py (reference digests) and the tests.
FR_ORDER = {
    "bn128": 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001,
    "bls12_381": 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
}
NTT_PATTERNS = ("all_rm1", "alt_0_rm1", "delta_one", "delta_rm1", "constant", "descending")


def _words(x):
    return np.array([(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)


def fr_int(row):
    return sum(int(row[i]) << (64 * i) for i in range(4))


def mont_one(curve):
    return (1 << 256) % FR_ORDER[curve]


PATTERN_CONST = 0x1F2E3D4C5B6A79880123456789ABCDEF00112233445566778899AABBCCDDEEFF


def ntt_pattern(curve, name, m):
    """raw Montgomery words of pattern `name` at size 2^m"""
    r = FR_ORDER[curve]
    n = 1 << m
    x = np.zeros((n, 4), dtype=np.uint64)
    if name == "all_rm1":
        x[:] = _words(r - 1)
    elif name == "alt_0_rm1":
        x[1::2] = _words(r - 1)
    elif name == "delta_one":
        x[0] = _words(mont_one(curve))
    elif name == "delta_rm1":
        x[0] = _words(r - 1)
    elif name == "constant":
        x[:] = _words(PATTERN_CONST % r)
    elif name == "descending":  # r-1, r-2, ...: the largest distinct canonical words
        lo = (r - 1) & 0xFFFFFFFFFFFFFFFF
        assert lo >= n
        x[:] = _words(r - 1)
        x[:, 0] = np.uint64(lo) - np.arange(n, dtype=np.uint64)
    else:
        raise KeyError(name)
    return x


def ntt_pattern_expected(curve, name, m, inverse):
    """closed form of the NTT of the constant / delta / alternating patterns (raw Montgomery words
    are linear: mont(a x) = a mont(x)), or None for patterns without one.  Returns a dict
    {index: raw value}; every other output is 0."""
    r = FR_ORDER[curve]
    n = 1 << m
    ninv = pow(n, -1, r)
    rm1 = r - 1
    if name in ("all_rm1", "constant"):
        c = rm1 if name == "all_rm1" else PATTERN_CONST % r
        return {0: c % r} if inverse else {0: n * c % r}
    if name in ("delta_one", "delta_rm1"):
        d = mont_one(curve) if name == "delta_one" else rm1
        v = d * ninv % r if inverse else d
        return {"all": v}
    if name == "alt_0_rm1":
        if m == 0:
            return {0: 0}
        # sum over odd j of a w^(+-jk) = a w^(+-k) (n/2) [k in {0, n/2}]; w^(n/2) = -1
        half = n // 2
        s = rm1 * (ninv if inverse else 1) % r
        return {0: s * half % r, half: (r - s * half % r) % r}
    return None


def check_pattern_output(curve, name, m, inverse, out):
    """True / False against the closed form, None when the pattern has none"""
    exp = ntt_pattern_expected(curve, name, m, inverse)
    if exp is None:
        return None
    n = 1 << m
    if "all" in exp:
        return bool(np.all(out == _words(exp["all"])))
    want = np.zeros((n, 4), dtype=np.uint64)
    for k, v in exp.items():
        want[k] = _words(v)
    return bool(np.array_equal(out, want))


def ntt_patterns_golden():
    p = os.path.join(GOLD, "ntt_patterns.json")
    return json.load(open(p)) if os.path.exists(p) else {}
