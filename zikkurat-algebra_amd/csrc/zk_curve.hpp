// zk_curve.hpp -- G1 point arithmetic on the device, short Weierstrass a = 0.
//
// The reference accumulates buckets in homogeneous projective coordinates with the
// madd-1998-cmo mixed add (bls12_381_G1_proj.c:334-374, 9M+2S) and the complete
// add-2015-rcb (:273-314, 12M).  On the GPU the bucket accumulators are kept in
// extended Jacobian "XYZZ" coordinates (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2), whose
// mixed add is 8M+2S and whose special cases (P == Q, P == -Q, infinity) are cheap
// to detect.  Only the affine / normalised result leaves the device, and that is
// canonical, so the coordinate system is invisible at the C ABI.
//
// Affine input points use the reference's encoding: Montgomery x || y with the point at
// infinity as all-0xFF bytes (bls12_381_G1_affine.c:1-6, :63-66).
#pragma once
#include "zk_field.hpp"
#include "zk_field2.hpp"

namespace zk {

// curve descriptors: base field, scalar field, and the constants we need
struct BN254 {
  using Fp = BN_Fp;
  using Fr = BN_Fr;
  static constexpr int NP64 = ZK_BN128_FP_N64;
};
struct BLS381 {
  using Fp = BLS_Fp;
  using Fr = BLS_Fr;
  static constexpr int NP64 = ZK_BLS12_381_FP_N64;
};
// G2: the twists over Fp2 (a = 0 as well; the XYZZ formulas never use b)
struct BN254_G2 {
  using Fp = F2<BN_Fp>;
  using Fr = BN_Fr;
  static constexpr int NP64 = 2 * ZK_BN128_FP_N64;
};
struct BLS381_G2 {
  using Fp = F2<BLS_Fp>;
  using Fr = BLS_Fr;
  static constexpr int NP64 = 2 * ZK_BLS12_381_FP_N64;
};

template <class F>
struct Aff {
  Fe<F> x, y;
};
// XYZZ with infinity encoded as ZZ == 0
template <class F>
struct Xyzz {
  Fe<F> X, Y, ZZ, ZZZ;
};

template <class F>
__device__ __forceinline__ void xyzz_set_inf(Xyzz<F> &r) {
  fe_one(r.X);
  fe_one(r.Y);
  fe_zero(r.ZZ);
  fe_zero(r.ZZZ);
}
template <class F>
__device__ __forceinline__ bool xyzz_is_inf(const Xyzz<F> &a) {
  return fe_is_zero(a.ZZ);
}
template <class F>
__device__ __forceinline__ void xyzz_from_aff(Xyzz<F> &r, const Aff<F> &a) {
  r.X = a.x;
  r.Y = a.y;
  fe_one(r.ZZ);
  fe_one(r.ZZZ);
}

// r = 2*(x, y) for an affine point (mdbl-2008-s-1), result XYZZ
template <class F>
__device__ __forceinline__ void xyzz_dbl_aff(Xyzz<F> &r, const Aff<F> &a) {
  Fe<F> U, V, W, S, M, t;
  fe_add(U, a.y, a.y);     // U = 2Y
  fe_sqr(V, U);            // V = U^2
  fe_mul(W, U, V);         // W = U*V
  fe_mul(S, a.x, V);       // S = X*V
  fe_sqr(t, a.x);
  fe_mul3(M, t);           // M = 3X^2
  fe_sqr(t, M);
  fe_sub(t, t, S);
  fe_sub(r.X, t, S);       // X3 = M^2 - 2S
  fe_sub(t, S, r.X);
  fe_mul(t, M, t);
  fe_mul(U, W, a.y);
  fe_sub(r.Y, t, U);       // Y3 = M(S - X3) - W*Y
  r.ZZ = V;
  r.ZZZ = W;
}

// r = 2*p (dbl-2008-s-1), XYZZ
template <class F>
__device__ __forceinline__ void xyzz_dbl(Xyzz<F> &r, const Xyzz<F> &p) {
  if (xyzz_is_inf(p)) { r = p; return; }
  Fe<F> U, V, W, S, M, t;
  fe_add(U, p.Y, p.Y);
  fe_sqr(V, U);
  fe_mul(W, U, V);
  fe_mul(S, p.X, V);
  fe_sqr(t, p.X);
  fe_mul3(M, t);
  fe_sqr(t, M);
  fe_sub(t, t, S);
  Fe<F> X3;
  fe_sub(X3, t, S);
  fe_sub(t, S, X3);
  fe_mul(t, M, t);
  fe_mul(U, W, p.Y);
  fe_sub(r.Y, t, U);
  r.X = X3;
  fe_mul(r.ZZ, V, p.ZZ);
  fe_mul(r.ZZZ, W, p.ZZZ);
}

// acc += a  (mixed add, madd-2008-s), all special cases handled
template <class F>
__device__ __forceinline__ void xyzz_add_aff(Xyzz<F> &acc, const Aff<F> &a) {
  if (xyzz_is_inf(acc)) { xyzz_from_aff(acc, a); return; }
  Fe<F> P, R, t;
  fe_mul(P, a.x, acc.ZZ);      // U2 = X2*ZZ1
  fe_sub(P, P, acc.X);         // P  = U2 - X1
  fe_mul(R, a.y, acc.ZZZ);     // S2 = Y2*ZZZ1
  fe_sub(R, R, acc.Y);         // R  = S2 - Y1
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) { xyzz_dbl_aff(acc, a); }
    else { xyzz_set_inf(acc); }
    return;
  }
  Fe<F> PP, PPP, Q;
  fe_sqr(PP, P);
  fe_mul(PPP, P, PP);
  fe_mul(Q, acc.X, PP);
  fe_sqr(t, R);
  fe_sub(t, t, PPP);
  fe_sub(t, t, Q);
  fe_sub(t, t, Q);             // X3 = R^2 - PPP - 2Q
  fe_sub(Q, Q, t);
  fe_mul(Q, R, Q);             // R*(Q - X3)
  fe_mul(R, acc.Y, PPP);       // Y1*PPP
  fe_sub(acc.Y, Q, R);
  acc.X = t;
  fe_mul(acc.ZZ, acc.ZZ, PP);
  fe_mul(acc.ZZZ, acc.ZZZ, PPP);
}

// Bucket-accumulation mixed add for the 381-bit field, with lazy subtractions.
// Same formula as xyzz_add_aff (madd-2008-s), but every difference is taken lazily
// (a + K p - b, zk_field.hpp "lazy ops"), the P == 0 / R == 0 tests move onto the
// squares PP and RR (products are < 2p and normalised, and PP == 0 <=> P == 0 as p is
// prime), and Y3 = R (Q - X3) - Y1 PPP is one fe_mul2 (shared reduction).
// Representation invariant of acc between calls: X, Y normalised limbs with values
// X < 14p, Y < 2p; ZZ, ZZZ < 2p.  The accumulator is stored in this form: every later
// consumer takes X only into products (which accept it).  Bounds (BLS12-381 Fp: 14 x 28-bit
// limbs, R'/p > 2^11), all checked mechanically by tools/lazy_bounds.py (tests/test_tools_bounds.py):
//   P = U2 + 16p - X1 < 18p, limbs < 2^29.6;  R = S2 + 8p - Y1 < 10p
//   PP, RR, PPP, Q < 2p (products of values < 2^11 p)
//   X3 = RR + 4p - PPP + 8p - 2Q < 14p;  t = Q + 16p - X3 < 18p
//   Y3 = (R t + (6p - Y1) PPP) / R' < 1.06p
// Column sums in fe_mul2 (R t: limbs < 2^29.6 each; (6p - Y1): < 2^29.6) stay < 2^64.  (The
// once-documented Y < 6p would break 6p - Y1's top-limb borrow; every producer gives Y < 1.06p.)
#ifndef ZK_KARA_MADD
#define ZK_KARA_MADD 1  // the madd's products on Karatsuba column sums (fe_mulk); 0: schoolbook
#endif
template <class F>
__device__ __forceinline__ void madd_mul(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  if constexpr (ZK_KARA_MADD) fe_mulk(r, a, b); else fe_mul(r, a, b);
}
template <class F>
__device__ __forceinline__ void xyzz_add_aff_lazy(Xyzz<F> &acc, const Aff<F> &a) {
  static_assert(F::N == 14 && F::RB == 28, "lazy madd bounds are derived for the 14 x 28-bit field");
  if (xyzz_is_inf(acc)) { xyzz_from_aff(acc, a); return; }
  Fe<F> P, R, PP, RR, t;
  madd_mul(t, a.x, acc.ZZ);               // U2
  fe_sub_lazy<F, 16, 1>(P, t, acc.X);     // P = U2 - X1
  madd_mul(t, a.y, acc.ZZZ);              // S2
  fe_sub_lazy<F, 8, 1>(R, t, acc.Y);      // R = S2 - Y1
  fe_sqr(PP, P);
  fe_sqr(RR, R);
  if (fe_is_zero(PP)) {
    if (fe_is_zero(RR)) { xyzz_dbl_aff(acc, a); }
    else { xyzz_set_inf(acc); }
    return;
  }
  Fe<F> PPP, Q, X3, q2;
  madd_mul(PPP, P, PP);
  madd_mul(Q, acc.X, PP);
  fe_sub_lazy<F, 4, 1>(t, RR, PPP);       // RR - PPP
  fe_add_lazy(q2, Q, Q);
  fe_sub_lazy<F, 8, 2>(X3, t, q2);        // - 2Q
  fe_norm(X3);
  fe_sub_lazy<F, 16, 1>(t, Q, X3);        // Q - X3
  Fe<F> ny;
  fe_sub_lazy<F, 6, 1>(ny, Fe<F>{}, acc.Y);  // 6p - Y1 (acc.Y < 2p, normalised)
  if constexpr (ZK_KARA_MADD) fe_mul2k(acc.Y, R, t, ny, PPP);  // Y3 = R (Q - X3) - Y1 PPP
  else fe_mul2(acc.Y, R, t, ny, PPP);
  acc.X = X3;
  madd_mul(acc.ZZ, acc.ZZ, PP);
  madd_mul(acc.ZZZ, acc.ZZZ, PPP);
}
// The same for the 254-bit base field (9 x 29-bit limbs, R'/p ~ 2^7.4: too little headroom to
// keep X lazily, so X3 is brought below 2p by the product-free fe_reduce_small).  The
// accumulator keeps the exact invariant X, Y, ZZ, ZZZ < 2p, normalised.  Bounds (values in
// units of p; checked for BN254 by tools/lazy_bounds.py):
//   P = U2 + 3p - X1 < 5p,  R = S2 + 3p - Y1 < 5p        (normalised before squaring)
//   X3 = RR + 3p - PPP + 5p - 2Q < 10p -> fe_reduce_small -> < 2p
//   Y3 = (R (Q + 3p - X3) + (3p - Y1) PPP) / R' :  (25 + 6) p^2 < p R'  ->  Y3 < 2p
// Limbs: every product operand is normalised (< 2^29; top limbs < 2^25), so fe_mul2's
// column sums stay below 27 * 2^58 < 2^63.
template <class F>
__device__ __forceinline__ void xyzz_add_aff_lazy9(Xyzz<F> &acc, const Aff<F> &a) {
  static_assert(F::N == 9 && F::RB == 29, "bounds derived for the 9 x 29-bit fields");
  if (xyzz_is_inf(acc)) { xyzz_from_aff(acc, a); return; }
  Fe<F> P, R, PP, RR, t;
  fe_mul(t, a.x, acc.ZZ);                 // U2
  fe_sub_lazy<F, 3, 1>(P, t, acc.X);      // P = U2 - X1
  fe_norm(P);
  fe_mul(t, a.y, acc.ZZZ);                // S2
  fe_sub_lazy<F, 3, 1>(R, t, acc.Y);      // R = S2 - Y1
  fe_norm(R);
  fe_sqr(PP, P);
  fe_sqr(RR, R);
  if (fe_is_zero(PP)) {
    if (fe_is_zero(RR)) { xyzz_dbl_aff(acc, a); }
    else { xyzz_set_inf(acc); }
    return;
  }
  Fe<F> PPP, Q, X3, q2;
  fe_mul(PPP, P, PP);
  fe_mul(Q, acc.X, PP);
  fe_sub_lazy<F, 3, 1>(t, RR, PPP);       // RR - PPP
  fe_add_lazy(q2, Q, Q);
  fe_sub_lazy<F, 5, 2>(X3, t, q2);        // - 2Q
  fe_norm(X3);
  fe_reduce_small(X3);                    // < 2p
  fe_sub_lazy<F, 3, 1>(t, Q, X3);         // Q - X3
  fe_norm(t);
  Fe<F> ny;
  fe_sub_lazy<F, 3, 1>(ny, Fe<F>{}, acc.Y);  // 3p - Y1
  fe_norm(ny);
  fe_mul2(acc.Y, R, t, ny, PPP);          // Y3 = R (Q - X3) - Y1 PPP
  acc.X = X3;
  fe_mul(acc.ZZ, acc.ZZ, PP);
  fe_mul(acc.ZZZ, acc.ZZZ, PPP);
}

// dispatch: lazy variants for the 381-bit and the 254-bit base fields, exact otherwise (Fp2)
template <class F>
__device__ __forceinline__ void xyzz_acc_aff(Xyzz<F> &acc, const Aff<F> &a) {
  if constexpr (F::N == 14) xyzz_add_aff_lazy(acc, a);
  else if constexpr (F::N == 9 && F::RB == 29) xyzz_add_aff_lazy9(acc, a);
  else xyzz_add_aff(acc, a);
}

// acc += b  (add-2008-s), all special cases handled
template <class F>
__device__ __forceinline__ void xyzz_add(Xyzz<F> &acc, const Xyzz<F> &b) {
  if (xyzz_is_inf(b)) return;
  if (xyzz_is_inf(acc)) { acc = b; return; }
  Fe<F> U1, S1, P, R, t;
  fe_mul(U1, acc.X, b.ZZ);     // U1 = X1*ZZ2
  fe_mul(P, b.X, acc.ZZ);      // U2 = X2*ZZ1
  fe_sub(P, P, U1);            // P = U2 - U1
  fe_mul(S1, acc.Y, b.ZZZ);    // S1 = Y1*ZZZ2
  fe_mul(R, b.Y, acc.ZZZ);     // S2 = Y2*ZZZ1
  fe_sub(R, R, S1);            // R = S2 - S1
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) { xyzz_dbl(acc, b); }
    else { xyzz_set_inf(acc); }
    return;
  }
  Fe<F> PP, PPP, Q;
  fe_sqr(PP, P);
  fe_mul(PPP, P, PP);
  fe_mul(Q, U1, PP);
  fe_sqr(t, R);
  fe_sub(t, t, PPP);
  fe_sub(t, t, Q);
  fe_sub(t, t, Q);             // X3
  fe_sub(Q, Q, t);
  fe_mul(Q, R, Q);
  fe_mul(S1, S1, PPP);
  fe_sub(acc.Y, Q, S1);
  acc.X = t;
  fe_mul(acc.ZZ, acc.ZZ, b.ZZ);
  fe_mul(acc.ZZ, acc.ZZ, PP);
  fe_mul(acc.ZZZ, acc.ZZZ, b.ZZZ);
  fe_mul(acc.ZZZ, acc.ZZZ, PPP);
}

// acc += b (add-2008-s) for the G1 reductions (Y sums), with lazy differences and the shared-
// reduction Y3 of the lazy mixed adds above.  Inputs in the bucket forms (381-bit: X < 14p,
// Y < 2p; 254-bit: X, Y < 2p), output in the same form.  Bounds (tools/lazy_bounds.py), in units of p:
//   381-bit: P = U2 + 4p - U1 < 6p, R = S2 + 4p - S1 < 6p, X3 < 14p as in the madd,
//            Y3: R (Q + 16p - X3) + (4p - S1) PPP < (6 * 18 + 4 * 2) p^2 < p R' (R'/p > 2^11)
//   254-bit: as xyzz_add_aff_lazy9 with U1, S1 (< 2p) in place of X1, Y1
#ifndef ZK_KARA_ADD
// the 381-bit lazy full add's products on Karatsuba column sums (1) or schoolbook (0): no
// measurable difference in the Y sums / stitch (profiles/r03b_karatsuba_ab.txt), schoolbook kept
#define ZK_KARA_ADD 0
#endif
template <class F>
__device__ __forceinline__ void add_mul(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  if constexpr (ZK_KARA_ADD) fe_mulk(r, a, b); else fe_mul(r, a, b);
}
template <class F>
__device__ __forceinline__ void xyzz_add_lazy(Xyzz<F> &acc, const Xyzz<F> &b) {
  static_assert(F::N == 14 || (F::N == 9 && F::RB == 29), "lazy bounds derived for the G1 base fields");
  constexpr bool W9 = F::N == 9;
  if (xyzz_is_inf(b)) return;
  if (xyzz_is_inf(acc)) { acc = b; return; }
  Fe<F> U1, S1, P, R, PP, RR, t;
  add_mul(U1, acc.X, b.ZZ);
  add_mul(t, b.X, acc.ZZ);                            // U2
  if constexpr (W9) { fe_sub_lazy<F, 3, 1>(P, t, U1); fe_norm(P); }
  else fe_sub_lazy<F, 4, 1>(P, t, U1);                // P = U2 - U1
  add_mul(S1, acc.Y, b.ZZZ);
  add_mul(t, b.Y, acc.ZZZ);                           // S2
  if constexpr (W9) { fe_sub_lazy<F, 3, 1>(R, t, S1); fe_norm(R); }
  else fe_sub_lazy<F, 4, 1>(R, t, S1);                // R = S2 - S1
  fe_sqr(PP, P);
  fe_sqr(RR, R);
  if (fe_is_zero(PP)) {
    if (fe_is_zero(RR)) { xyzz_dbl(acc, b); }
    else { xyzz_set_inf(acc); }
    return;
  }
  Fe<F> PPP, Q, X3, q2, ny;
  add_mul(PPP, P, PP);
  add_mul(Q, U1, PP);
  fe_add_lazy(q2, Q, Q);
  if constexpr (W9) {
    fe_sub_lazy<F, 3, 1>(t, RR, PPP);
    fe_sub_lazy<F, 5, 2>(X3, t, q2);                  // RR - PPP - 2Q < 10p
    fe_norm(X3);
    fe_reduce_small(X3);                              // < 2p
    fe_sub_lazy<F, 3, 1>(t, Q, X3);
    fe_norm(t);
    fe_sub_lazy<F, 3, 1>(ny, Fe<F>{}, S1);
    fe_norm(ny);
  } else {
    fe_sub_lazy<F, 4, 1>(t, RR, PPP);
    fe_sub_lazy<F, 8, 2>(X3, t, q2);                  // RR - PPP - 2Q < 14p
    fe_norm(X3);
    fe_sub_lazy<F, 16, 1>(t, Q, X3);                  // Q - X3 < 18p
    fe_sub_lazy<F, 4, 1>(ny, Fe<F>{}, S1);            // 4p - S1
  }
  Fe<F> zz, zzz;
  add_mul(zz, acc.ZZ, b.ZZ);
  add_mul(zzz, acc.ZZZ, b.ZZZ);
  if constexpr (ZK_KARA_ADD) fe_mul2k(acc.Y, R, t, ny, PPP);  // Y3 = R (Q - X3) - S1 PPP
  else fe_mul2(acc.Y, R, t, ny, PPP);
  acc.X = X3;
  add_mul(acc.ZZ, zz, PP);
  add_mul(acc.ZZZ, zzz, PPP);
}
// the Y sums' addition: lazy for the G1 base fields, exact for Fp2
template <class F>
__device__ __forceinline__ void xyzz_add_red(Xyzz<F> &acc, const Xyzz<F> &b) {
  if constexpr (F::N == 14 || (F::N == 9 && F::RB == 29)) xyzz_add_lazy(acc, b);
  else xyzz_add(acc, b);
}

// XYZZ storage: 4 consecutive field elements, F::SN u32 words each (shared by the MSM and the
// group FFT kernels)
template <class F>
__device__ __forceinline__ void xyzz_store(uint32_t *p, const Xyzz<F> &a) {
  fe_store_u(p + 0 * F::SN, a.X);
  fe_store_u(p + 1 * F::SN, a.Y);
  fe_store_u(p + 2 * F::SN, a.ZZ);
  fe_store_u(p + 3 * F::SN, a.ZZZ);
}
template <class F>
__device__ __forceinline__ void xyzz_load(Xyzz<F> &a, const uint32_t *p) {
  fe_load_u(a.X, p + 0 * F::SN);
  fe_load_u(a.Y, p + 1 * F::SN);
  fe_load_u(a.ZZ, p + 2 * F::SN);
  fe_load_u(a.ZZZ, p + 3 * F::SN);
}
template <class F>
constexpr int xyzz_words() { return 4 * F::SN; }
template <class F>
constexpr int aff_words() { return 2 * F::SN; }

// Affine points on the device are kept in INTERNAL form (converted once per call by
// k_points_int): 2 x SN u32 words; the reference's all-0xFF infinity sentinel becomes a
// first word of 0xFFFFFFFF (never a valid limb).  Returns false for infinity.
template <class F>
__device__ __forceinline__ bool aff_load(Aff<F> &a, const uint32_t *__restrict__ p) {
  fe_load_u(a.x, p);
  fe_load_u(a.y, p + F::SN);
  return a.x.v[0] != 0xffffffffu;
}

// reference-form affine point (x || y, N64 u64 each) -> internal-form storage
template <class F>
__device__ __forceinline__ void aff_ref_to_int(uint32_t *__restrict__ out, const uint64_t *__restrict__ in) {
  uint64_t all = ~0ull;
#pragma unroll
  for (int i = 0; i < 2 * F::N64; i++) all &= in[i];
  if (all == ~0ull) {
    uint4 *o = reinterpret_cast<uint4 *>(out);
#pragma unroll
    for (int i = 0; i < F::SN / 2; i++) o[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
    return;
  }
  Fe<F> x, y, t;
  fe_load_ref(t, in);
  fe_to_int(x, t);
  fe_load_ref(t, in + F::N64);
  fe_to_int(y, t);
  fe_store_u(out, x);
  fe_store_u(out + F::SN, y);
}

}  // namespace zk
