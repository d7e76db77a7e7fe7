#!/usr/bin/env python3
"""Derive every curve/field constant the kernels need from first principles.

Inputs are only the public curve definitions (primes, curve equation
y^2 = x^3 + B, the standard G1 generator in affine *standard* coordinates and
the FFT-domain generator the reference's Haskell layer uses). Everything else
(Montgomery forms, -p^-1 mod 2^32, R^2, 3B, 1/2, ...) is computed here, and
tests/test_params.py cross-checks the results against the reference's
generated constants (e.g. bls12_381_G1_proj.c:33 gen_G1, :41 const_3B,
bls12_381_poly_mont.c:470 oneHalf) through the compiled oracle.

Writes zikkurat-algebra_amd/csrc/zk_params.inc (checked in).
"""
import os

CURVES = {
    # BN254 (called "bn128" in the reference): Fp/Fr 254-bit, B = 3, G1 generator (1, 2)
    "bn128": dict(
        p=0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47,
        r=0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001,
        B=3,
        gx=1, gy=2,
        # BN128/Fr/Mont.hs:146-148 : generator of the order-2^28 subgroup (standard repr)
        fft_gen=19103219067921713944291392827692070036145651957329286315305642004821462161904,
        fft_log=28,
    ),
    # BLS12-381: Fp 381-bit, Fr 255-bit, B = 4
    "bls12_381": dict(
        p=0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB,
        r=0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
        B=4,
        gx=0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
        gy=0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
        # BLS12_381/Fr/Mont.hs:146-148 : generator of the order-2^32 subgroup (standard repr)
        fft_gen=10238227357739495823651030575849232062558860180284477541189508159991286009131,
        fft_log=32,
    ),
}


def limbs(x, n, bits=64):
    m = (1 << bits) - 1
    return [(x >> (bits * i)) & m for i in range(n)]


def field_block(name, p):
    n64 = (p.bit_length() + 63) // 64
    n32 = 2 * n64
    R = 1 << (64 * n64)
    minv32 = (-pow(p, -1, 1 << 32)) % (1 << 32)
    minv64 = (-pow(p, -1, 1 << 64)) % (1 << 64)
    out = []
    out.append(f"// ---- {name}: {p.bit_length()}-bit prime, {n64} x u64 limbs, R = 2^{64*n64}")
    out.append(f"#define ZK_{name.upper()}_N64 {n64}")
    out.append(f"#define ZK_{name.upper()}_N32 {n32}")
    out.append(f"#define ZK_{name.upper()}_BITS {p.bit_length()}")
    def arr(tag, v, n, bits):
        fmt = "0x%016xull" if bits == 64 else "0x%08xu"
        vals = ", ".join(fmt % w for w in limbs(v, n, bits))
        out.append(f"#define ZK_{name.upper()}_{tag} {{ {vals} }}")
    arr("P64", p, n64, 64)
    arr("P32", p, n32, 32)
    arr("R64", R % p, n64, 64)          # Montgomery one
    arr("R32", R % p, n32, 32)
    arr("R2_64", (R * R) % p, n64, 64)  # for std -> mont
    arr("R2_32", (R * R) % p, n32, 32)
    out.append(f"#define ZK_{name.upper()}_MINV32 0x{minv32:08x}u")
    out.append(f"#define ZK_{name.upper()}_MINV64 0x{minv64:016x}ull")
    return out, R


# unsaturated device representation: limb radix 2^RB, NU limbs, internal Montgomery
# radix R' = 2^(RB*NU).  RB = 28 for the 381-bit field (headroom for one lazy add),
# 29 for the 254/255-bit fields (9 limbs).
UNSAT = {"bn128_fp": (29, 9), "bn128_fr": (29, 9), "bls12_381_fp": (28, 14), "bls12_381_fr": (29, 9)}


def unsat_block(name, p):
    RB, NU = UNSAT[name]
    n64 = (p.bit_length() + 63) // 64
    R = 1 << (64 * n64)          # the reference's Montgomery radix
    Ri = 1 << (RB * NU)          # internal radix
    assert 4 * p < Ri and 16 * p < Ri, name
    mask = (1 << RB) - 1
    # column-sum bound of the product-scanning multiplier for normalized limbs
    assert 2 * NU * (mask * mask) + (1 << (64 - RB + 1)) < (1 << 64), name
    minv = (-pow(p, -1, 1 << RB)) % (1 << RB)
    P = name.upper()
    out = [f"// unsaturated: {NU} limbs x {RB} bits, R' = 2^{RB*NU}"]
    out.append(f"#define ZK_{P}_U_RB {RB}")
    out.append(f"#define ZK_{P}_U_N {NU}")
    out.append(f"#define ZK_{P}_U_MINV 0x{minv:08x}u")
    def arr(tag, v):
        vals = ", ".join("0x%08xu" % w for w in limbs(v, NU, RB))
        out.append(f"#define ZK_{P}_U_{tag} {{ {vals} }}")
    arr("P", p)
    arr("P2", 2 * p)
    arr("ONE", Ri % p)                     # internal one
    arr("KIN", (Ri * Ri * pow(R, -1, p)) % p)   # ref Montgomery -> internal:  mont'(x, KIN)
    arr("KOUT", R % p)                     # internal -> ref Montgomery: mont'(x, KOUT)
    arr("KSTD", (Ri * pow(R, -1, p)) % p)  # ref Montgomery -> standard: mont'(x, KSTD)
    arr("K3", pow(Ri, 3, p))               # (x R')^-1 * R'^3 / R' = x^-1 R' (zk_inv.hpp: after safegcd)
    # safegcd (zk_inv.hpp): p in signed 62-bit limbs, p^-1 mod 2^62, the constant batch count
    # ceil(ceil((49 d + 57) / 17) / 62) of 62 divsteps for a d-bit modulus (Bernstein-Yang, d >= 46)
    nbits = p.bit_length()
    L62 = (nbits + 2 + 61) // 62
    steps = (49 * nbits + 57) // 17 + 1
    vals = ", ".join("%dll" % ((p >> (62 * i)) & ((1 << 62) - 1)) for i in range(L62))
    out.append(f"#define ZK_{P}_S62_L {L62}")
    out.append(f"#define ZK_{P}_S62_P {{ {vals} }}")
    out.append(f"#define ZK_{P}_S62_PINV 0x{pow(p, -1, 1 << 62):016x}ull")
    out.append(f"#define ZK_{P}_S62_BATCHES {-(-steps // 62)}")
    # the same in 60-bit limbs for batches of 2 x 30 divsteps in 32-bit arithmetic (zk_inv.hpp B = 60)
    L60 = (nbits + 2 + 59) // 60
    vals = ", ".join("%dll" % ((p >> (60 * i)) & ((1 << 60) - 1)) for i in range(L60))
    out.append(f"#define ZK_{P}_S60_L {L60}")
    out.append(f"#define ZK_{P}_S60_P {{ {vals} }}")
    out.append(f"#define ZK_{P}_S60_BATCHES {-(-steps // 60)}")
    return out


def main():
    lines = ["// GENERATED by tools/gen_params.py -- do not edit by hand.",
             "// Constants derived from the public curve definitions; cross-checked",
             "// against the reference's generated C in tests/test_params.py.", ""]
    for c, d in CURVES.items():
        p, r = d["p"], d["r"]
        fl, Rp = field_block(f"{c}_fp", p)
        fr, Rr = field_block(f"{c}_fr", r)
        lines += fl + fr
        lines += unsat_block(f"{c}_fp", p) + unsat_block(f"{c}_fr", r)
        C = c.upper()
        n64p = (p.bit_length() + 63) // 64
        n64r = (r.bit_length() + 63) // 64
        def mont(x, R, q):
            return (x * R) % q
        assert (d["gy"] ** 2 - d["gx"] ** 3 - d["B"]) % p == 0, c
        def arr(tag, v, n, bits=64):
            fmt = "0x%016xull" if bits == 64 else "0x%08xu"
            vals = ", ".join(fmt % w for w in limbs(v, n, bits))
            lines.append(f"#define ZK_{C}_{tag} {{ {vals} }}")
        arr("B3_FP64", mont(3 * d["B"], Rp, p), n64p)
        arr("B3_FP32", mont(3 * d["B"], Rp, p), 2 * n64p, 32)
        arr("GX_FP64", mont(d["gx"], Rp, p), n64p)
        arr("GY_FP64", mont(d["gy"], Rp, p), n64p)
        g = d["fft_gen"]
        L = d["fft_log"]
        assert pow(g, 1 << L, r) == 1 and pow(g, 1 << (L - 1), r) != 1, c
        arr("FFT_GEN_FR64", mont(g, Rr, r), n64r)
        lines.append(f"#define ZK_{C}_FFT_LOG {L}")
        arr("HALF_FR64", mont(pow(2, -1, r), Rr, r), n64r)
        lines.append("")
    here = os.path.dirname(os.path.abspath(__file__))
    dst = os.path.join(here, "..", "zikkurat-algebra_amd", "csrc", "zk_params.inc")
    with open(dst, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("wrote", os.path.normpath(dst))


if __name__ == "__main__":
    main()
