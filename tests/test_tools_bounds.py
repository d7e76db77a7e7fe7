"""CPU checks of the arithmetic-layout invariants the kernels rely on (no GPU):
the lazy 254-bit mixed add's value / limb bounds (tools/lazy_bounds.py) and the NTT tile
swizzle's bank-conflict freedom for every tile shape the pass kernel launches
(tools/ntt_lds_banks.py)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    return spec, mod


def test_lazy_bounds_all_paths():
    """every lazy path (both MSM base fields' mixed and full additions, the group FFT's lazy
    Jacobian doubling and cached addition on both base fields, the NTT butterflies of every radix,
    the closing reductions, the scalar REDC, the round-6 product-free radix conversions of the
    9 x 29-bit fields) satisfies its limb / value bounds"""
    spec, mod = _load("lazy_bounds")
    spec.loader.exec_module(mod)
    ok, results = mod.run_all(verbose=False)
    assert ok, [r for r in results if r[2] != "ok"]
    assert len(results) == 17
    assert {fn for _, fn, _ in results} >= {"jac_dbl_lazy", "jac_add_cached_lazy", "radix_conv"}


def test_lazy_jacobian_checker_rejects_a_tight_constant():
    """the Jacobian replays are not vacuous: with the accumulator invariant X < 10p a difference
    D + 4p - X3 (too small a K) must be rejected"""
    spec, mod = _load("lazy_bounds")
    spec.loader.exec_module(mod)
    F = mod.Field("bls12_381_fp")
    D, X3 = F.norm_val(2 * F.p), F.norm_val(9 * F.p)
    try:
        F.sub_lazy(D, X3, 4, 1)
        raise AssertionError("D + 4p - X3 accepted for X3 < 9p")
    except mod.BoundError:
        pass


def test_lazy_bounds_catch_a_broken_invariant():
    """the checker is not vacuous: the once-documented 381-bit Y < 6p form, a twiddle bounded
    only by 2p after 2^12-point DFTs, and a too-small K in a lazy difference are rejected"""
    spec, mod = _load("lazy_bounds")
    spec.loader.exec_module(mod)
    F = mod.Field("bls12_381_fp")
    y6 = F.norm_val(6 * F.p)
    try:
        F.sub_lazy(F.zero(), y6, 6, 1)
        raise AssertionError("Y < 6p accepted")
    except mod.BoundError:
        pass
    Fr = mod.Field("bls12_381_fr")
    out = mod.ntt_lds_dft(Fr, 12, Fr.norm_val(Fr.p))
    w = Fr.norm_val(2 * Fr.p)  # a twiddle only known to be < 2p (tw2's product is < 1.02p)
    y = Fr.mul(out, w)
    assert y.val > 2 * Fr.p  # 2^12-point DFT outputs (< 50p) times 2p exceed p R' (R'/p = 70.7)
    try:
        F.sub_lazy(F.norm_val(2 * F.p), F.norm_val(14 * F.p), 8, 1)
        raise AssertionError("b < 14p accepted under K = 8")
    except mod.BoundError:
        pass


def test_ntt_swizzle_conflict_free():
    src = open(os.path.join(ROOT, "tools", "ntt_lds_banks.py")).read()
    ns = {}
    exec(compile(src.split('for name, f in')[0], "ntt_lds_banks", "exec"), ns)
    # shapes the pass kernel launches: 1024-element tiles with R = 2^8 (G = 4), 4096-element
    # tiles with R = 2^9..2^12, and the single-tile transforms of 2^10 / 2^11 points
    for (r, G, NT) in [(8, 4, 256), (9, 8, 1024), (10, 4, 1024), (11, 2, 1024), (12, 1, 1024),
                       (11, 1, 256), (10, 1, 256)]:
        worst = max(ns["degree"]([ns["swz_new"](x) for x in sl]) for _, sl in ns["patterns"](r, G, NT))
        assert worst == 1, (r, G, NT, worst)
