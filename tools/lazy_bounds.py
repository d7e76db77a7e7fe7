#!/usr/bin/env python3
"""Mechanical bound checks of every lazy-arithmetic path on the device (CPU only):

    python tools/lazy_bounds.py          (exit status 0 = every check holds)

The device field (zikkurat-algebra_amd/csrc/zk_field.hpp) keeps values in unsaturated
RB-bit limbs and skips carries and reductions wherever the headroom allows.  This script is
a small abstract interpreter over that arithmetic: every abstract value carries
  * an upper bound on each limb (the limbs are never negative), and
  * an exclusive upper bound on the integer it represents,
and every device primitive is restated with the conditions its correctness rests on:

  fe_mul / fe_sqr / fe_mul2   every product-scanning column (products + m*p terms + carry-in)
                              < 2^64; squaring's doubled limbs < 2^32; output < A B / R' + p
                              (A, B the operand bounds), limbs normalised
  fe_sub_lazy<K, BW>          r_i = a_i + kpb_i - b_i with kpb = K p in borrowed limbs: needs
                              b_i <= kpb_i (no limb goes negative) and b < K p; r_i < 2^32
  fe_add_lazy, fe_norm        limb sums < 2^32; norm keeps the value, normalises the limbs
  fe_add / fe_sub (exact)     normalised operands; fe_add's result < max(2p, A + B - 2p),
                              fe_sub's (b < 2p) < max(A, 2p)
  fe_reduce_small             v < 64p and the top-limb quotient estimate q_est in {q - 1, q}
                              for EVERY top limb value (interval argument, exact rationals)
  fe_is_zero / fe_canon       operand < 2p
  fe_store_packed             value < 2^256, normalised limbs

The device functions are then replayed on these abstract values, with the representation
invariants they document taken as inputs and re-checked on their outputs:

  * zk_curve.hpp  xyzz_add_aff_lazy   (BLS12-381 Fp, 14 x 28: acc X < 14p, Y < 2p -- the checker
                                       showed the once-documented Y < 6p would break fe_sub_lazy<6,1>'s
                                       top-limb condition; every producer gives Y < 1.06p)
                  xyzz_add_aff_lazy9  (BN254 Fp, 9 x 29: acc < 2p)
                  xyzz_add_lazy       (both fields: the stitch / Y-sum additions)
                  xyzz_add, xyzz_dbl, xyzz_dbl_aff and the quad addition on the lazy forms
                  (the in-wavefront merge, k_ysum, k_jobsum_blk) and the export fe_to_ref
  * zk_ntt.hip    lds_dft for every radix 2^1 .. 2^12 the pass kernel runs (first radix-4
                  round, radix-4 rounds, odd radix-2 stage), the inter-pass twiddle product
                  (table, and the on-the-fly path, whose twiddle is a product < 1.02p), the last pass's closing step
                  (fe_reduce_small, or the product by 1/N), the packed non-canonical store,
                  for BN254 Fr and BLS12-381 Fr
  * zk_msm_impl.hpp  the scalar REDC (fe_ref_to_std of any 256-bit pattern)

Reference semantics these bounds protect: canonical Montgomery results of the reference's
field ops (bls12_381_Fp_mont.c:146-214, bls12_381_Fr_mont.c:84-199), madd / add / dbl
(bls12_381_G1_proj.c:231-374) and the NTT (bls12_381_poly_mont.c:418-522).
"""
import sys
from fractions import Fraction

PRIMES = {
    "bn254_fp": 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47,
    "bn254_fr": 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001,
    "bls12_381_fp": 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB,
    "bls12_381_fr": 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
}
LAYOUT = {"bn254_fp": (29, 9), "bn254_fr": (29, 9), "bls12_381_fp": (28, 14), "bls12_381_fr": (29, 9)}
U32, U64 = 1 << 32, 1 << 64

BN254_P = PRIMES["bn254_fp"]  # kept for older callers


class BoundError(AssertionError):
    pass


class V:
    """abstract value: per-limb maxima `lim`, integer value < `val`"""
    __slots__ = ("lim", "val", "what")

    def __init__(self, lim, val, what=""):
        self.lim, self.val, self.what = list(lim), val, what


class Field:
    def __init__(self, name):
        self.name = name
        self.p = PRIMES[name]
        self.RB, self.N = LAYOUT[name]
        self.MASK = (1 << self.RB) - 1
        self.Rp = 1 << (self.RB * self.N)
        self.pl = self.limbs(self.p)
        self.checks = 0
        self.log = []

    # -- helpers
    def limbs(self, x):
        RB, N = self.RB, self.N
        return [(x >> (RB * i)) & self.MASK if i < N - 1 else x >> (RB * i) for i in range(N)]

    def need(self, cond, msg):
        self.checks += 1
        if not cond:
            raise BoundError(f"{self.name}: {msg}")

    def units(self, v):
        return float(Fraction(v.val, self.p))

    def norm_val(self, bound, what=""):
        """normalised limbs, value < bound"""
        N, RB = self.N, self.RB
        lim = [self.MASK] * (N - 1) + [(bound - 1) >> (RB * (N - 1))]
        return V(lim, bound, what)

    def const(self, x, what=""):
        return V(self.limbs(x), x + 1, what)

    def zero(self):
        return V([0] * self.N, 1, "0")

    def is_norm(self, a):
        return all(l <= self.MASK for l in a.lim[:-1])

    def top_ok(self, a):
        return a.lim[-1] < U32 and all(l < U32 for l in a.lim)

    def kp_borrowed(self, K, BW):
        """zk_field.hpp kp_limb / kp_borrowed: K p with every limb below the top borrowed BW"""
        N, RB = self.N, self.RB
        kp = self.limbs(K * self.p)
        out = [kp[0] + (BW << RB)] + [kp[i] + (BW << RB) - BW for i in range(1, N - 1)] + [kp[N - 1] - BW]
        assert sum(v << (RB * i) for i, v in enumerate(out)) == K * self.p
        return out

    # -- products (fe_mul, fe_sqr, fe_mul2): product scanning with one 64-bit column sum
    def _columns(self, terms, what):
        """terms(k) -> max of the column's limb products (a*b part); adds the m*p part and the
        carry-in and checks every column total < 2^64.  Returns the final carry (o[N-1])."""
        N, RB, M = self.N, self.RB, self.MASK
        carry = 0
        for k in range(2 * N - 1):
            lo, hi = max(0, k - N + 1), min(k, N - 1)
            s = terms(k) + sum(M * self.pl[k - i] for i in range(lo, hi + 1))
            tot = s + carry
            self.need(tot < U64, f"{what}: column {k} sum {tot.bit_length()} bits >= 2^64")
            carry = tot >> RB
        self.need(carry < U32, f"{what}: top limb {carry.bit_length()} bits")
        return carry

    def _prod_out(self, num, what):
        """Montgomery output bound: (num + m p) / R' with m < R'"""
        val = (num - 1) // self.Rp + self.p + 1  # value <= (num-1)/R' + p  (exclusive bound)
        out = self.norm_val(val, what)
        self.need(out.lim[-1] < U32, f"{what}: output top limb")
        return out

    def mul(self, a, b, what="mul"):
        N = self.N
        self.need(self.top_ok(a) and self.top_ok(b), f"{what}: operand limbs >= 2^32")
        self._columns(lambda k: sum(a.lim[i] * b.lim[k - i] for i in range(max(0, k - N + 1), min(k, N - 1) + 1)), what)
        return self._prod_out((a.val - 1) * (b.val - 1) + 1, what)

    def mulk(self, a, b, what="mulk"):
        """fe_mulk (Karatsuba column sums on the 14-limb field, schoolbook otherwise): the columns
        equal the schoolbook ones; the split differences a_lo - a_hi, b_hi - b_lo are int32, so
        every limb must be < 2^31"""
        if self.N == 14:
            self.need(all(l < (1 << 31) for l in a.lim + b.lim), f"{what}: limb >= 2^31 (int32 differences)")
        return self.mul(a, b, what)

    def mul2k(self, a, b, c, d, what="mul2k"):
        if self.N == 14:
            self.need(all(l < (1 << 31) for l in a.lim + b.lim + c.lim + d.lim), f"{what}: limb >= 2^31")
        return self.mul2(a, b, c, d, what)

    def mul2(self, a, b, c, d, what="mul2"):
        N = self.N
        for x in (a, b, c, d):
            self.need(self.top_ok(x), f"{what}: operand limbs >= 2^32")
        self._columns(lambda k: sum(a.lim[i] * b.lim[k - i] + c.lim[i] * d.lim[k - i]
                                    for i in range(max(0, k - N + 1), min(k, N - 1) + 1)), what)
        return self._prod_out((a.val - 1) * (b.val - 1) + (c.val - 1) * (d.val - 1) + 1, what)

    def sqr(self, a, what="sqr"):
        N = self.N
        a2 = [2 * l for l in a.lim]
        self.need(all(l < U32 for l in a2), f"{what}: doubled limbs >= 2^32")

        def terms(k):
            s = sum(a2[i] * a.lim[k - i] for i in range(N) if i < k - i < N)
            if k % 2 == 0 and k // 2 < N:
                s += a.lim[k // 2] ** 2
            return s
        self._columns(terms, what)
        return self._prod_out((a.val - 1) ** 2 + 1, what)

    # -- lazy ops
    def sub_lazy(self, a, b, K, BW, what="sub_lazy"):
        kpb = self.kp_borrowed(K, BW)
        for i in range(self.N):
            self.need(b.lim[i] <= kpb[i], f"{what}<{K},{BW}>: limb {i} of b ({b.lim[i]:#x}) > borrowed K p limb ({kpb[i]:#x})")
        self.need(b.val <= K * self.p, f"{what}<{K},{BW}>: b < {self.units(b):.2f} p not <= {K} p")
        lim = [a.lim[i] + kpb[i] for i in range(self.N)]
        self.need(all(l < U32 for l in lim), f"{what}: limb overflow")
        return V(lim, a.val + K * self.p, what)

    def add_lazy(self, a, b, what="add_lazy"):
        lim = [x + y for x, y in zip(a.lim, b.lim)]
        self.need(all(l < U32 for l in lim), f"{what}: limb overflow")
        return V(lim, a.val + b.val - 1, what)

    def norm(self, a, what="norm"):
        c = 0
        for i in range(self.N - 1):
            c = (a.lim[i] + c) >> self.RB
        top = a.lim[-1] + c
        self.need(top < U32, f"{what}: top limb overflow")
        out = self.norm_val(a.val, what)
        out.lim[-1] = min(out.lim[-1], top)
        return out

    # -- exact ops (fe_add / fe_sub: two int32 carry chains, normalised operands)
    def add(self, a, b, what="add"):
        self.need(self.is_norm(a) and self.is_norm(b), f"{what}: operands not normalised")
        self.need(a.lim[-1] + b.lim[-1] < (1 << 31), f"{what}: int32 top limb")
        return self.norm_val(max(2 * self.p, a.val + b.val - 1 - 2 * self.p), what)

    def sub(self, a, b, what="sub"):
        self.need(self.is_norm(a) and self.is_norm(b), f"{what}: operands not normalised")
        self.need(b.val <= 2 * self.p, f"{what}: subtrahend < {self.units(b):.2f} p not < 2p")
        return self.norm_val(max(a.val, 2 * self.p), what)

    def is_zero_ok(self, a, what):
        self.need(a.val <= 2 * self.p and self.is_norm(a), f"{what}: fe_is_zero needs < 2p (got {self.units(a):.2f} p)")

    def canon(self, a, what="canon"):
        self.need(a.val <= 2 * self.p and self.is_norm(a), f"{what}: fe_canon needs < 2p (got {self.units(a):.2f} p)")
        return self.norm_val(self.p, what)

    def store_packed(self, a, what="store_packed"):
        self.need(self.is_norm(a) and a.val <= 1 << 256, f"{what}: packed store needs normalised limbs, < 2^256")

    def reduce_small(self, a, what="reduce_small"):
        self.need(self.N == 9 and self.RB == 29, f"{what}: derived for 9 x 29 limbs")
        self.need(self.is_norm(a), f"{what}: operand not normalised")
        self.need(a.val <= 64 * self.p, f"{what}: operand {self.units(a):.2f} p not < 64 p")
        self.reduce_small_proof(a.val)
        return self.norm_val(2 * self.p, what)

    def reduce_small_proof(self, vmax):
        """fe_reduce_small: q = (v_top K) >> 32 with v_top = v >> 232 (limb 8) and
        K = floor(2^64 / (floor(p / 2^200) + 1)).  For every v < vmax: q <= floor(v/p) (the
        result stays >= 0) and floor(v/p) - q <= 1 (the result is < 2p).  Per top-limb value
        t, v ranges over [t 2^232, (t+1) 2^232): q_est(t) <= floor(t 2^232 / p) follows from
        K <= 2^64 p' / p ... and the largest quotient in the range exceeds q_est(t) by at most
        1 when t (2^232/p - K/2^32) + 2^232/p < 1 + (the fractional slack), checked exactly
        at the extreme t (the expression is monotone in t)."""
        p = self.p
        Pd = (p >> 200) + 1
        K = (U64 - 1) // Pd  # ~0ull / (...)
        tmax = (vmax - 1) >> 232
        # upper side: q_est(t) = floor(t K / 2^32) <= t 2^232 / p for all t (K / 2^32 <= 2^232 / p)
        self.need(Fraction(K, U32) <= Fraction(1 << 232, p), "reduce_small: reciprocal over-estimates 1/p")
        # lower side: q_max(t) - q_est(t) < (t+1) 2^232 / p - (t K / 2^32 - 1) = t e + 2^232/p + 1,
        # e = 2^232/p - K/2^32 >= 0: increasing in t, so the worst case is t = tmax
        e = Fraction(1 << 232, p) - Fraction(K, U32)
        slack = tmax * e + Fraction(1 << 232, p) + 1
        self.need(slack < 2, f"reduce_small: quotient estimate may be off by 2 (slack {float(slack)})")
        # spot-check the exact claim at both ends of the range and around multiples of p
        for t in (0, 1, tmax // 2, tmax):
            for v in (t << 232, ((t + 1) << 232) - 1):
                if v >= vmax:
                    v = vmax - 1
                q = (t * K) >> 32
                self.need(q <= v // p and v // p - q <= 1, f"reduce_small: spot check at t={t}")
        self.log.append(f"reduce_small: v < {vmax / p:.1f} p, top limb <= {tmax:#x}: q_est in {{q-1, q}} "
                        f"(slack {float(slack):.9f} < 2)")


# --------------------------------------------------------------------------- MSM curve arithmetic

def bucket_form(F):
    """stored accumulator form (k_accum flushes, stitch/Y-sum outputs): see zk_curve.hpp"""
    p = F.p
    if F.N == 14:
        return {"X": F.norm_val(14 * p, "X"), "Y": F.norm_val(2 * p, "Y"), "ZZ": F.norm_val(2 * p, "ZZ"),
                "ZZZ": F.norm_val(2 * p, "ZZZ")}
    return {k: F.norm_val(2 * p, k) for k in ("X", "Y", "ZZ", "ZZZ")}


def in_form(F, pt, what):
    form = bucket_form(F)
    for k in ("X", "Y", "ZZ", "ZZZ"):
        F.need(F.is_norm(pt[k]) and pt[k].val <= form[k].val,
               f"{what}: output {k} < {F.units(pt[k]):.2f} p outside the stored form (< {F.units(form[k]):.0f} p)")


def affine_input(F):
    """internal-form affine point: fe_to_int products (< 2p); a negated y is fe_neg (< 2p)"""
    x = F.norm_val(2 * F.p, "x")
    y = F.sub(F.zero(), F.norm_val(2 * F.p), "fe_neg(y)")
    return x, y


def dbl_aff(F, x, y, tag):
    """xyzz_dbl_aff: exact ops"""
    U = F.add(y, y, tag + " U")
    V_ = F.sqr(U, tag + " V")
    W = F.mul(U, V_, tag + " W")
    S = F.mul(x, V_, tag + " S")
    t = F.sqr(x, tag + " x^2")
    t = F.add(F.add(t, t), t, tag + " M")
    M = t
    t = F.sqr(M, tag + " M^2")
    t = F.sub(t, S, tag)
    X3 = F.sub(t, S, tag + " X3")
    t = F.sub(S, X3, tag)
    t = F.mul(M, t, tag)
    U = F.mul(W, y, tag)
    Y3 = F.sub(t, U, tag + " Y3")
    return {"X": X3, "Y": Y3, "ZZ": V_, "ZZZ": W}


def dbl(F, pt, tag):
    """xyzz_dbl: exact ops on a stored-form point"""
    U = F.add(pt["Y"], pt["Y"], tag + " U")
    V_ = F.sqr(U, tag + " V")
    W = F.mul(U, V_, tag + " W")
    S = F.mul(pt["X"], V_, tag + " S")
    t = F.sqr(pt["X"], tag)
    M = F.add(F.add(t, t), t, tag + " M")
    t = F.sqr(M, tag)
    t = F.sub(t, S, tag)
    X3 = F.sub(t, S, tag + " X3")
    t = F.sub(S, X3, tag)
    t = F.mul(M, t, tag)
    U = F.mul(W, pt["Y"], tag)
    Y3 = F.sub(t, U, tag + " Y3")
    return {"X": X3, "Y": Y3, "ZZ": F.mul(V_, pt["ZZ"], tag), "ZZZ": F.mul(W, pt["ZZZ"], tag)}


def madd_lazy14(F):
    """zk_curve.hpp xyzz_add_aff_lazy (BLS12-381 Fp, 14 x 28; products on Karatsuba column sums)"""
    p, tag = F.p, "xyzz_add_aff_lazy"
    acc = bucket_form(F)
    x, y = affine_input(F)
    t = F.mulk(x, acc["ZZ"], tag + " U2")
    P = F.sub_lazy(t, acc["X"], 16, 1, tag + " P")
    t = F.mulk(y, acc["ZZZ"], tag + " S2")
    R = F.sub_lazy(t, acc["Y"], 8, 1, tag + " R")
    PP = F.sqr(P, tag + " PP")
    RR = F.sqr(R, tag + " RR")
    F.is_zero_ok(PP, tag + " PP")
    F.is_zero_ok(RR, tag + " RR")
    in_form(F, dbl_aff(F, x, y, tag + " (P = R = 0 branch) dbl_aff"), tag + " doubling branch")
    PPP = F.mulk(P, PP, tag + " PPP")
    Q = F.mulk(acc["X"], PP, tag + " Q")
    t = F.sub_lazy(RR, PPP, 4, 1, tag + " RR-PPP")
    q2 = F.add_lazy(Q, Q, tag + " 2Q")
    X3 = F.norm(F.sub_lazy(t, q2, 8, 2, tag + " X3"), tag + " X3")
    t = F.sub_lazy(Q, X3, 16, 1, tag + " Q-X3")
    ny = F.sub_lazy(F.zero(), acc["Y"], 6, 1, tag + " 6p-Y1")
    Y3 = F.mul2k(R, t, ny, PPP, tag + " Y3")
    out = {"X": X3, "Y": Y3, "ZZ": F.mulk(acc["ZZ"], PP, tag + " ZZ3"), "ZZZ": F.mulk(acc["ZZZ"], PPP, tag + " ZZZ3")}
    in_form(F, out, tag)
    F.log.append(f"{tag}: P < {F.units(P):.1f} p, R < {F.units(R):.1f} p, X3 < {F.units(X3):.1f} p, "
                 f"Y3 < {F.units(Y3):.2f} p (R'/p = {F.Rp / p:.0f})")


def madd_lazy9(F):
    """zk_curve.hpp xyzz_add_aff_lazy9 (BN254 Fp, 9 x 29)"""
    tag = "xyzz_add_aff_lazy9"
    acc = bucket_form(F)
    x, y = affine_input(F)
    t = F.mul(x, acc["ZZ"], tag + " U2")
    P = F.norm(F.sub_lazy(t, acc["X"], 3, 1, tag + " P"))
    t = F.mul(y, acc["ZZZ"], tag + " S2")
    R = F.norm(F.sub_lazy(t, acc["Y"], 3, 1, tag + " R"))
    PP, RR = F.sqr(P, tag + " PP"), F.sqr(R, tag + " RR")
    F.is_zero_ok(PP, tag + " PP")
    F.is_zero_ok(RR, tag + " RR")
    in_form(F, dbl_aff(F, x, y, tag + " dbl_aff"), tag + " doubling branch")
    PPP = F.mul(P, PP, tag + " PPP")
    Q = F.mul(acc["X"], PP, tag + " Q")
    t = F.sub_lazy(RR, PPP, 3, 1, tag)
    q2 = F.add_lazy(Q, Q, tag)
    X3 = F.norm(F.sub_lazy(t, q2, 5, 2, tag + " X3"), tag)
    X3r = F.reduce_small(X3, tag + " X3")
    t = F.norm(F.sub_lazy(Q, X3r, 3, 1, tag + " Q-X3"))
    ny = F.norm(F.sub_lazy(F.zero(), acc["Y"], 3, 1, tag + " 3p-Y1"))
    Y3 = F.mul2(R, t, ny, PPP, tag + " Y3")
    out = {"X": X3r, "Y": Y3, "ZZ": F.mul(acc["ZZ"], PP), "ZZZ": F.mul(acc["ZZZ"], PPP)}
    in_form(F, out, tag)
    F.log.append(f"{tag}: P, R < {F.units(P):.1f} p, X3 lazy < {F.units(X3):.1f} p -> < 2p, "
                 f"Y3 < {F.units(Y3):.2f} p (R'/p = {F.Rp / F.p:.0f})")


def add_lazy(F):
    """zk_curve.hpp xyzz_add_lazy (the stitch's and the Y sums' addition), stored forms in and out"""
    tag = "xyzz_add_lazy"
    W9 = F.N == 9
    a, b = bucket_form(F), bucket_form(F)
    U1 = F.mulk(a["X"], b["ZZ"], tag + " U1")
    t = F.mulk(b["X"], a["ZZ"], tag + " U2")
    P = F.norm(F.sub_lazy(t, U1, 3, 1, tag + " P")) if W9 else F.sub_lazy(t, U1, 4, 1, tag + " P")
    S1 = F.mulk(a["Y"], b["ZZZ"], tag + " S1")
    t = F.mulk(b["Y"], a["ZZZ"], tag + " S2")
    R = F.norm(F.sub_lazy(t, S1, 3, 1, tag + " R")) if W9 else F.sub_lazy(t, S1, 4, 1, tag + " R")
    PP, RR = F.sqr(P, tag + " PP"), F.sqr(R, tag + " RR")
    F.is_zero_ok(PP, tag + " PP")
    F.is_zero_ok(RR, tag + " RR")
    in_form(F, dbl(F, b, tag + " dbl"), tag + " doubling branch")
    PPP = F.mulk(P, PP, tag + " PPP")
    Q = F.mulk(U1, PP, tag + " Q")
    q2 = F.add_lazy(Q, Q)
    if W9:
        t = F.sub_lazy(RR, PPP, 3, 1, tag)
        X3 = F.reduce_small(F.norm(F.sub_lazy(t, q2, 5, 2, tag + " X3")), tag + " X3")
        t = F.norm(F.sub_lazy(Q, X3, 3, 1, tag + " Q-X3"))
        ny = F.norm(F.sub_lazy(F.zero(), S1, 3, 1, tag + " 3p-S1"))
    else:
        t = F.sub_lazy(RR, PPP, 4, 1, tag)
        X3 = F.norm(F.sub_lazy(t, q2, 8, 2, tag + " X3"))
        t = F.sub_lazy(Q, X3, 16, 1, tag + " Q-X3")
        ny = F.sub_lazy(F.zero(), S1, 4, 1, tag + " 4p-S1")
    zz = F.mulk(a["ZZ"], b["ZZ"])
    zzz = F.mulk(a["ZZZ"], b["ZZZ"])
    Y3 = F.mul2k(R, t, ny, PPP, tag + " Y3")
    out = {"X": X3, "Y": Y3, "ZZ": F.mulk(zz, PP), "ZZZ": F.mulk(zzz, PPP)}
    in_form(F, out, tag)
    F.log.append(f"{tag}: P, R < {F.units(P):.1f} p, X3 < {F.units(X3):.1f} p, Y3 < {F.units(Y3):.2f} p")


def add_exact_on_stored(F):
    """zk_curve.hpp xyzz_add (k_accum's in-wavefront merge, k_ysum) and xyzz_add_quad (k_jobsum_blk:
    the same products and exact differences, split over a quad) on stored-form inputs; then the
    export fe_to_ref (product by KOUT, fe_canon) of every coordinate"""
    tag = "xyzz_add(stored forms)"
    a, b = bucket_form(F), bucket_form(F)
    U1 = F.mul(a["X"], b["ZZ"], tag + " U1")
    P = F.sub(F.mul(b["X"], a["ZZ"], tag + " U2"), U1, tag + " P")
    S1 = F.mul(a["Y"], b["ZZZ"], tag + " S1")
    R = F.sub(F.mul(b["Y"], a["ZZZ"], tag + " S2"), S1, tag + " R")
    F.is_zero_ok(P, tag + " P")
    F.is_zero_ok(R, tag + " R")
    in_form(F, dbl(F, b, tag + " dbl"), tag + " doubling branch")
    PP = F.sqr(P)
    PPP = F.mul(P, PP)
    Q = F.mul(U1, PP)
    t = F.sub(F.sub(F.sub(F.sqr(R), PPP), Q), Q, tag + " X3")
    X3 = t
    Qm = F.mul(R, F.sub(Q, X3))
    Y3 = F.sub(Qm, F.mul(S1, PPP), tag + " Y3")
    out = {"X": X3, "Y": Y3, "ZZ": F.mul(F.mul(a["ZZ"], b["ZZ"]), PP), "ZZZ": F.mul(F.mul(a["ZZZ"], b["ZZZ"]), PPP)}
    in_form(F, out, tag)
    kout = F.const(pow(2, 64 * ((F.p.bit_length() + 63) // 64), F.p), "KOUT")
    for k, v in bucket_form(F).items():
        F.canon(F.mul(v, kout, "fe_to_ref " + k), "export " + k)


# --------------------------------------------------------------------------- NTT

def ntt_lds_dft(F, r, vin):
    """zk_ntt.hip lds_dft for one R = 2^r point DFT, inputs < vin (normalised limbs); inner
    twiddles are canonical (< p, fe_store_ref'd then loaded).  Returns the output bound."""
    w = F.norm_val(F.p, "itw")
    a = vin
    s = 0
    if r >= 2:  # first radix-4 round
        t = F.mul(F.sub_lazy(a, a, 4, 1, "b3"), w, "first round t")
        b0 = F.add_lazy(a, a)
        b1 = F.sub_lazy(a, a, 4, 1, "b1")
        s23 = F.add_lazy(a, a)
        outs = [F.add_lazy(b0, s23), F.sub_lazy(b0, s23, 4, 2, "a2 = b0 - s23"), F.add_lazy(b1, t),
                F.sub_lazy(b1, t, 4, 1, "a3 = b1 - t")]
        a = max((F.norm(o) for o in outs), key=lambda v: v.val)
        s = 2
    while s + 1 < r:  # radix-4 rounds
        t = F.mul(a, w, f"stage {s} t")
        b0, b1 = F.add_lazy(a, t), F.sub_lazy(a, t, 4, 1, "b1")
        b2, b3 = F.add_lazy(a, t), F.sub_lazy(a, t, 4, 1, "b3")
        t2 = F.mul(b2, w, f"stage {s + 1} t (b2 w2)")
        t3 = F.mul(b3, w, f"stage {s + 1} t (b3 w3)")
        outs = [F.add_lazy(b0, t2), F.sub_lazy(b0, t2, 4, 1, "a2"), F.add_lazy(b1, t3), F.sub_lazy(b1, t3, 4, 1, "a3")]
        a = max((F.norm(o) for o in outs), key=lambda v: v.val)
        s += 2
    if s < r:  # odd r: one radix-2 stage
        t = F.mul(a, w, f"stage {s} t")
        a = max((F.norm(F.add_lazy(a, t)), F.norm(F.sub_lazy(a, t, 4, 1, "y"))), key=lambda v: v.val)
    return a


def ntt_paths(F):
    """every pass shape of zk_ntt.hip: radix 2^r for r = 0..12.  A pass's input is the caller's
    canonical vector (< p, pass 0 and single-pass transforms) or the previous pass's packed
    product (x w with w < p): the bound of the latter is the fixed point of
    V -> max_r (dft_r(V) p / R' + p) over every radix a pass can have.  Closing steps: the
    inter-pass twiddle product (table: canonical; on the fly: tw2's product of two canonical
    table entries, < 1.02p), the last pass's fe_reduce_small, or the product by the 1/N scale
    (fe_to_int of the canonical constant: < 1.02p)."""
    p = F.p
    tw = F.norm_val(p, "canonical twiddle")
    tw_otf = F.mul(F.norm_val(p), F.norm_val(p), "tw2")  # the larger of the two twiddle bounds
    vin = p
    for _ in range(50):  # a bound V with f(V) <= V (f is monotone; V is rounded up to p / 1024 steps)
        nxt = max(p, max(F.mul(ntt_lds_dft(F, r, F.norm_val(vin)), tw_otf, "inter-pass").val for r in range(1, 13)))
        if nxt <= vin:
            break
        vin = -(-nxt // (p // 1024)) * (p // 1024)
    F.need(nxt <= vin, "no inter-pass fixed point")
    F.need(vin <= 2 * p, "inter-pass values not < 2p")
    worst = {}
    for r in range(0, 13):
        for vb in (p, vin):
            a = F.norm_val(vb, "ntt input")
            out = ntt_lds_dft(F, r, a) if r > 0 else a
            worst[r] = max(worst.get(r, 0), out.val)
            for w, name in ((tw, "table"), (tw_otf, "otf")):
                y = F.mul(out, w, f"r={r} inter-pass twiddle ({name})")
                F.need(y.val <= vin, f"r={r}: inter-pass product above the fixed point")
                F.store_packed(y, f"r={r} packed store")
            F.canon(F.reduce_small(out, f"r={r} closing reduce_small"), "fe_store_ref")
            sc = F.mul(F.norm_val(p), F.norm_val(p), "fe_to_int(1/N)")  # canonical 1/N times KIN
            F.canon(F.mul(out, sc, f"r={r} closing product by 1/N"), "fe_store_ref")
    F.log.append(f"ntt inter-pass values < {vin / p:.3f} p; lds_dft output bounds (units of p): " +
                 ", ".join(f"2^{r}: {worst[r] / p:.1f}" for r in range(13)) + f"; R'/p = {F.Rp / p:.1f}")


def scalar_redc(F):
    """zk_msm_impl.hpp DigitStream::load: fe_ref_to_std of any 256-bit pattern (k[8] = 0)"""
    x = V([F.MASK] * 8 + [(1 << 256) - 1 >> 232], 1 << 256, "raw scalar")
    kstd = F.norm_val(F.p, "KSTD")
    F.canon(F.mul(x, kstd, "fe_ref_to_std"), "fe_ref_to_std canon")


JAC_X = 10  # Jacobian accumulator / table-entry invariant of the lazy group-FFT routines: X < 10p


def jac_form(F):
    """zk_g1ext.hip (ZK_FFT_LAZY): X < JAC_X p, Y, Z < 2p, normalised limbs"""
    return {"X": F.norm_val(JAC_X * F.p, "X"), "Y": F.norm_val(2 * F.p, "Y"), "Z": F.norm_val(2 * F.p, "Z")}


def in_jac_form(F, pt, what):
    form = jac_form(F)
    for k in ("X", "Y", "Z"):
        F.need(F.is_norm(pt[k]) and pt[k].val <= form[k].val,
               f"{what}: output {k} < {F.units(pt[k]):.2f} p outside the Jacobian form (< {F.units(form[k]):.0f} p)")


def jac_dbl_lazy(F):
    """zk_g1ext.hip jac_dbl, ZK_FFT_LAZY (both base fields): dbl-2009-l with the multiples folded into
    products and lazy differences; Y3 one shared-reduction pair"""
    tag = "jac_dbl_lazy"
    pt = jac_form(F)
    A = F.sqr(pt["X"], tag + " A")
    B = F.sqr(pt["Y"], tag + " B")
    x4 = F.add_lazy(pt["X"], pt["X"], tag + " 2X")
    x4 = F.add_lazy(x4, x4, tag + " 4X")
    D = F.mulk(x4, B, tag + " D")
    E = F.add_lazy(F.add_lazy(A, A, tag + " 2A"), A, tag + " E")
    if F.N == 9:  # fe_norm on the 29-bit limbs only
        E = F.norm(E, tag + " E")
    F2 = F.sqr(E, tag + " F")
    t = F.add_lazy(D, D, tag + " 2D")
    X3 = F.norm(F.sub_lazy(F2, t, 8, 2, tag + " X3"), tag + " X3")
    y2 = F.add_lazy(pt["Y"], pt["Y"], tag + " 2Y")
    Z3 = F.mulk(y2, pt["Z"], tag + " Z3")
    t = F.norm(F.sub_lazy(D, X3, JAC_X, 1, tag + " D-X3"), tag + " D-X3")
    nb = F.norm(F.sub_lazy(F.zero(), B, 2, 1, tag + " 2p-B"), tag + " 2p-B")
    nb8 = F.add_lazy(nb, nb, tag + " 2nb")
    nb8 = F.add_lazy(nb8, nb8, tag + " 4nb")
    nb8 = F.add_lazy(nb8, nb8, tag + " 8nb")
    if F.N == 9:
        nb8 = F.norm(nb8, tag + " 8nb")
    Y3 = F.mul2k(E, t, nb8, B, tag + " Y3")
    in_jac_form(F, {"X": X3, "Y": Y3, "Z": Z3}, tag)
    F.log.append(f"{tag}: 4X < {F.units(x4):.0f} p, E < {F.units(E):.0f} p, X3 < {F.units(X3):.1f} p, "
                 f"Y3 < {F.units(Y3):.2f} p, Z3 < {F.units(Z3):.2f} p")


def jac_add_cached_lazy(F):
    """zk_g1ext.hip jac_add_cached, ZK_FFT_LAZY: add-1998-cmo-2 with the table entry's Z^2, Z^3
    cached (products), H and r exact (zero-tested), the rest lazy"""
    tag = "jac_add_cached_lazy"
    acc = jac_form(F)
    b = jac_form(F)
    b["ZZ"] = F.sqr(b["Z"], tag + " ZZ")
    b["ZZZ"] = F.mul(b["ZZ"], b["Z"], tag + " ZZZ")
    # lane 1's lookup: X times beta (a product), Y possibly negated (exact fe_neg)
    b["X"] = F.mulk(b["X"], F.norm_val(2 * F.p, "beta"), tag + " beta X")
    b["Y"] = F.sub(F.zero(), b["Y"], tag + " -Y")
    Z1Z1 = F.sqr(acc["Z"], tag + " Z1Z1")
    U1 = F.mulk(acc["X"], b["ZZ"], tag + " U1")
    U2 = F.mulk(b["X"], Z1Z1, tag + " U2")
    S1 = F.mulk(acc["Y"], b["ZZZ"], tag + " S1")
    t = F.mulk(acc["Z"], Z1Z1, tag + " Z1^3")
    S2 = F.mulk(b["Y"], t, tag + " S2")
    H = F.sub(U2, U1, tag + " H")
    r = F.sub(S2, S1, tag + " r")
    F.is_zero_ok(H, tag + " H")
    F.is_zero_ok(r, tag + " r")
    HH = F.sqr(H, tag + " HH")
    HHH = F.mulk(H, HH, tag + " HHH")
    V_ = F.mulk(U1, HH, tag + " V")
    RR = F.sqr(r, tag + " RR")
    t = F.sub_lazy(RR, HHH, 2, 1, tag + " RR-HHH")
    v2 = F.add_lazy(V_, V_, tag + " 2V")
    X3 = F.norm(F.sub_lazy(t, v2, 6, 2, tag + " X3"), tag + " X3")
    t = F.norm(F.sub_lazy(V_, X3, JAC_X + 2, 1, tag + " V-X3"), tag + " V-X3")
    nS1 = F.norm(F.sub_lazy(F.zero(), S1, 2, 1, tag + " 2p-S1"), tag + " 2p-S1")
    Y3 = F.mul2k(r, t, nS1, HHH, tag + " Y3")
    t = F.mulk(acc["Z"], b["Z"], tag + " Z1Z2")
    Z3 = F.mulk(t, H, tag + " Z3")
    in_jac_form(F, {"X": X3, "Y": Y3, "Z": Z3}, tag)
    # the accumulator converted to XYZZ (jac_to_xyzz) keeps X; xyzz_add / the normalisation only
    # multiply it: every product of a value < JAC_X p by one < 2p is in range
    F.mulk(X3, F.norm_val(2 * F.p), tag + " consumers of X")
    F.log.append(f"{tag}: X3 < {F.units(X3):.1f} p, V - X3 < {F.units(t):.1f} p, Y3 < {F.units(Y3):.2f} p")


def radix_conv(F):
    """zk_field.hpp fe_to_int / fe_to_ref on the 9 x 29-bit fields (round 6: R' = 32 R, so the
    conversions are a product by 32 / by 1/32 instead of a Montgomery product by a constant):
      fe_mul32_small: any loaded value < 2^256 (a raw reference word, canonical or not) or any
        product < 2p, shifted by five bits (< 2^261, top limb < 2^29) -> fe_reduce_small, whose
        quotient estimate is proven here over the WHOLE 9-limb range v < 2^261 (not only < 64p)
      fe_div32_small: a < 33p -> (a + k p) / 32 < 2p (k < 32) -> fe_canon"""
    tag = "radix_conv"
    F.need(F.N == 9 and F.RB == 29, f"{tag}: derived for 9 x 29 limbs")
    F.need(F.Rp == 32 * (1 << 256), f"{tag}: R' != 32 R")
    vmax = 1 << 261
    F.reduce_small_proof(vmax)
    F.need(32 * ((1 << 256) - 1) < vmax and 32 * 2 * F.p < vmax, f"{tag}: 32 a exceeds 2^261")
    # to_ref: a < 33 p (every caller passes < 2p: products, the exact 254-bit bucket forms)
    amax = 33 * F.p - 1
    F.need(amax + 31 * F.p < 32 * 2 * F.p, f"{tag}: (a + k p) / 32 not < 2p")
    F.need(amax + 31 * F.p < (1 << 261) * 2 ** 3, f"{tag}: a + k p overflows the 64-bit limb sums")
    F.log.append(f"{tag}: to_int over v < 2^261 = {(1 << 261) / F.p:.0f} p (reduce_small q_est in {{q-1, q}}); "
                 f"to_ref (a + k p)/32 < {(amax + 31 * F.p) / 32 / F.p:.2f} p for a < 33p")


def check_bn254():
    F = Field("bn254_fp")
    madd_lazy9(F)
    add_lazy(F)
    add_exact_on_stored(F)
    return True


def run_all(verbose=True):
    ok = True
    results = []
    plans = [("bls12_381_fp", [madd_lazy14, add_lazy, add_exact_on_stored, jac_dbl_lazy, jac_add_cached_lazy]),
             ("bn254_fp", [madd_lazy9, add_lazy, add_exact_on_stored, jac_dbl_lazy, jac_add_cached_lazy,
                           radix_conv]),
             ("bls12_381_fr", [ntt_paths, scalar_redc, radix_conv]),
             ("bn254_fr", [ntt_paths, scalar_redc, radix_conv])]
    for name, fns in plans:
        F = Field(name)
        for fn in fns:
            try:
                fn(F)
                status = "ok"
            except BoundError as e:
                ok = False
                status = f"FAIL {e}"
            results.append((name, fn.__name__, status))
        if verbose:
            print(f"== {name}: {F.N} x {F.RB}-bit limbs, R'/p = {F.Rp / F.p:.1f}, {F.checks} conditions checked")
            for line in F.log:
                print("   " + line)
    if verbose:
        for name, fn, status in results:
            print(f"{name:14s} {fn:22s} {status}")
    return ok, results


if __name__ == "__main__":
    ok, _ = run_all()
    sys.exit(0 if ok else 1)
