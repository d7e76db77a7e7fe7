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


def test_lazy_madd_bounds_bn254():
    spec, mod = _load("lazy_bounds")
    spec.loader.exec_module(mod)
    assert mod.check_bn254()


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
