"""The Fp2 product of the G2 pipeline (zk_field2.hpp fe_mul on F2<B>, ZK_FP2_LAZY): c0 = REDC(a0 b0 +
a1 (2p - b1)), c1 = REDC(a0 b1 + a1 b0) -- two shared-reduction pairs (fe_mul2 / fe_mul2k) instead of
Karatsuba's three full products.  A bit-level model of the device code (normalised limbs, the u64
column sums of both products, the interleaved REDC of zk_field.hpp redc_cols) against
big-integer Fp2 arithmetic (reference: <C>_Fp2_mont.c, u^2 = -1) on random and extreme operands:
every value < 2p that the G2 formulas feed it, limbs at their maxima.  Checks the outputs are < 2p
(the invariant of every device product) and that no column overflows 64 bits."""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gen_params import CURVES  # noqa: E402

LAYOUT = {"bn128": (29, 9), "bls12_381": (28, 14)}  # (RB, N) of the unsaturated Fp layouts


def to_limbs(x, rb, n):
    return [(x >> (rb * i)) & ((1 << rb) - 1) for i in range(n - 1)] + [x >> (rb * (n - 1))]


def redc_pair(a, b, c, d, p, rb, n):
    """REDC(a b + c d) exactly as fe_mul2 / fe_mul2k form it (column sums, then the m p terms)"""
    A, B, C, D = (to_limbs(x, rb, n) for x in (a, b, c, d))
    T = [sum(A[i] * B[k - i] + C[i] * D[k - i] for i in range(n) if 0 <= k - i < n) for k in range(2 * n - 1)]
    mask = (1 << rb) - 1
    minv = (-pow(p, -1, 1 << rb)) % (1 << rb)
    pl = to_limbs(p, rb, n)
    m, o, acc = [0] * n, [0] * n, 0
    for k in range(2 * n - 1):
        acc += T[k]
        for i in range(max(0, k - n + 1), min(k, n)):
            acc += m[i] * pl[k - i]
        if k < n:
            m[k] = ((acc & 0xFFFFFFFF) * minv) & mask
            acc += m[k] * pl[0]
        assert acc < 1 << 64, "column overflow"
        if k >= n:
            o[k - n] = acc & mask
        acc >>= rb
    o[n - 1] = acc
    return sum(v << (rb * i) for i, v in enumerate(o))


def fp2_mul_model(curve, a0, a1, b0, b1):
    p = CURVES[curve]["p"]
    rb, n = LAYOUT[curve]
    nb1 = 2 * p - b1  # fe_sub_lazy<B, 2, 1>(0, b1) + fe_norm: the value 2p - b1, normalised
    return redc_pair(a0, b0, a1, nb1, p, rb, n), redc_pair(a0, b1, a1, b0, p, rb, n)


@pytest.mark.parametrize("curve", sorted(LAYOUT))
def test_model_vs_bigint(curve):
    p = CURVES[curve]["p"]
    rb, n = LAYOUT[curve]
    assert 8 * p < 1 << (rb * n)  # both pairs < 8p^2 < p R'
    rinv = pow(1 << (rb * n), -1, p)
    rng = random.Random(7)
    top = 2 * p - 1
    extremes = [0, 1, p - 1, p, p + 1, top, top - 1, (1 << (rb * (n - 1))) - 1,
                top & ~((1 << (rb * (n - 1))) - 1)]
    cases = [tuple(rng.choice(extremes) for _ in range(4)) for _ in range(300)]
    cases += [tuple(rng.randrange(2 * p) for _ in range(4)) for _ in range(300)]
    for a0, a1, b0, b1 in cases:
        c0, c1 = fp2_mul_model(curve, a0, a1, b0, b1)
        assert c0 < 2 * p and c1 < 2 * p
        assert c0 % p == (a0 * b0 - a1 * b1) * rinv % p
        assert c1 % p == (a0 * b1 + a1 * b0) * rinv % p
