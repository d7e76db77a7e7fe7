"""The C-ABI library loads and exports every symbol include/*.h declares; its host-side
helpers agree with the oracle.  CPU only: no compute call reaches the GPU here."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = []
    for f in os.listdir(os.path.join(ROOT, "include")):
        if f.endswith(".h"):
            txt = open(os.path.join(ROOT, "include", f)).read()
            syms += re.findall(r"ZKG_API\s+[\w\s\*]+?\b(\w+)\s*\(", txt)
    return syms


def test_header_declares_reference_surface(zk):
    syms = set(declared_symbols())
    assert set(zk.REFERENCE_SYMBOLS) <= syms
    assert set(zk.EXTENSION_SYMBOLS) <= syms


def test_library_exports_every_declared_symbol(zk):
    out = subprocess.check_output(["nm", "-D", "--defined-only", zk.LIB_PATH], text=True)
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    lib = zk.load()
    for s in declared_symbols():
        assert hasattr(lib, s)


def test_library_exports_nothing_else(zk):
    out = subprocess.check_output(["nm", "-D", "--defined-only", zk.LIB_PATH], text=True)
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    extra = exported - set(declared_symbols())
    assert not extra, sorted(extra)[:20]


def test_reference_signatures_match_reference_headers():
    """Our prototypes are textually the reference's (modulo the export macro)."""
    ref = "/root/reference/lib/cbits/curves"
    if not os.path.isdir(ref):
        pytest.skip("reference tree not present")
    ours = open(os.path.join(ROOT, "include", "zkalgebra_gpu.h")).read()

    def norm(s):
        return re.sub(r"\s+", "", s)
    for c in ("bn128", "bls12_381"):
        for hdr, pat in ((f"g1/proj/{c}_G1_proj.h", r"MSM_(mont|std)_coeff_(proj|affine)_out(_variable)?\("),
                         (f"g1/jac/{c}_G1_jac.h", r"MSM_(mont|std)_coeff_(jac|affine)_out\("),
                         (f"poly/mont/{c}_poly_mont.h", r"ntt_(forward|inverse)\(|_by_vanishing\s*\("),
                         (f"array/mont/{c}_arr_mont.h", r"_arr_mont_\w+\s*\("),
                         (f"g1/proj/{c}_G1_proj.h", r"_(batch_(from|to)_affine|fft_(forward|inverse))\s*\("),
                         (f"g1/jac/{c}_G1_jac.h", r"_(batch_(from|to)_affine|fft_(forward|inverse))\s*\("),
                         (f"g2/proj/{c}_G2_proj.h", r"MSM_(mont|std)_coeff_(proj|affine)_out\(")):
            for line in open(os.path.join(ref, hdr)):
                if re.search(pat, line) and "slow_reference" not in line and "noalloc" not in line:
                    proto = line.replace("extern", "").strip().rstrip(";")
                    name = re.search(r"(\w+)\s*\(", proto).group(1)
                    ours_line = [l for l in ours.splitlines() if re.search(r"\b" + name + r"\s*\(", l)]
                    assert ours_line, name
                    # compare parameter types only (names may differ)
                    ptypes = lambda s: [re.sub(r"\w+$", "", a.strip()).replace(" ", "")
                                        for a in s[s.index("(") + 1:s.rindex(")")].split(",")]
                    assert ptypes(proto) == ptypes(ours_line[0]), name


@pytest.mark.parametrize("curve", ["bn128", "bls12_381"])
def test_host_point_helpers_match_oracle(oracle, zk, curve):
    pts = zk.gen_points(curve, 21, 6)
    NP = zk.NLIMBS_P[curve]
    one = {"bn128": None}
    # lift to projective with Z = 1 (Montgomery one taken from a normalised oracle point)
    sc = oracle.to_std(1 if curve == "bn128" else 3, zk.gen_fr(curve, 22, 6))
    for i in range(5):
        a = oracle.msm(curve, sc[i:i + 1], pts[i:i + 1], mont=False, out="proj")
        b = oracle.msm(curve, sc[i + 1:i + 2], pts[i + 1:i + 2], mont=False, out="proj")
        s_o = oracle.normalize(curve, oracle.proj_add(curve, a, b))
        s_z = zk.g1_normalize(curve, zk.g1_add(curve, a, b))
        assert np.array_equal(s_o, s_z)
        assert np.array_equal(zk.g1_to_affine(curve, a), oracle.to_affine(curve, a))
    inf = np.zeros(3 * NP, dtype=np.uint64)
    assert np.all(zk.g1_to_affine(curve, inf) == np.uint64(0xFFFFFFFFFFFFFFFF))
