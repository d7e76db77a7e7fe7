#!/usr/bin/env python3
"""Bounds of the lazy XYZZ mixed additions in k_accum (zk_curve.hpp), checked with the actual
primes and limb layouts.  CPU only:  python tools/lazy_bounds.py

A device product fe_mul(a, b) (Montgomery w.r.t. R' = 2^(RB N)) returns a value < 2p when
a b < p R'; a lazy difference a + K p - b (fe_sub_lazy<K, BW>) never makes a limb negative
when b's top limb <= the top limb of K p written with borrowed limbs (kp_borrowed)."""
import math

BN254_P = 21888242871839275222246405745257275088696311157297823662689037894645226208583


def kp_borrowed(p, K, BW, RB, N):
    mask = (1 << RB) - 1
    kp = [((K * p) >> (RB * i)) & mask if i < N - 1 else (K * p) >> (RB * i) for i in range(N)]
    out = [kp[0] + (BW << RB)] + [kp[i] + (BW << RB) - BW for i in range(1, N - 1)] + [kp[N - 1] - BW]
    assert sum(v << (RB * i) for i, v in enumerate(out)) == K * p
    return out


def check_bn254():
    p, RB, N = BN254_P, 29, 9
    Rp = 1 << (RB * N)
    ok = True
    # xyzz_add_aff_lazy9: accumulator X, Y, ZZ, ZZZ < 2p; U2, S2, PP, RR, PPP, Q < 2p (products)
    P = 2 + 3   # U2 + 3p - X1
    R = 2 + 3   # S2 + 3p - Y1
    for name, prod in (("P^2", P * P), ("R^2", R * R), ("P PP", P * 2), ("X1 PP", 2 * 2),
                       ("Y3 = R (Q+3p-X3) + (3p-Y1) PPP", R * (2 + 3) + 3 * 2), ("ZZ PP", 4)):
        good = prod * p < Rp
        ok &= good
        print(f"BN254 {name}: {prod} p^2 < p R' ? {good}")
    x3 = 2 + 3 + 5  # RR + 3p - PPP + 5p - 2Q
    good = x3 < 64 and x3 * p < Rp
    ok &= good
    print(f"BN254 X3 lazy < {x3} p (fe_reduce_small needs < 64 p): {good}")
    for K, BW, bmax in ((3, 1, 2 * p), (5, 2, 4 * p)):
        kpb = kp_borrowed(p, K, BW, RB, N)
        good = kpb[-1] >= bmax >> (RB * (N - 1))
        ok &= good
        print(f"BN254 fe_sub_lazy<{K},{BW}> for b < {bmax // p} p: top limb {kpb[-1]} >= {bmax >> (RB * (N - 1))} ? {good}")
    # fe_mul2 column sums with normalised operands (limbs < 2^29): 2 N a*b terms + N m*p terms
    col = 3 * N * (1 << (2 * RB))
    good = col + (1 << 40) < (1 << 64)
    ok &= good
    print(f"BN254 fe_mul2 column sum < 2^{math.log2(col):.2f} < 2^64 ? {good}")
    return ok


if __name__ == "__main__":
    raise SystemExit(0 if check_bn254() else 1)
