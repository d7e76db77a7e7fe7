// zk_field2.hpp -- the quadratic extension Fp2 = Fp[u]/(u^2 + 1) on the device.
//
// Replaces, on the GPU, <C>_Fp2_mont_{add,sub,neg,mul,sqr} (lib/cbits/curves/fields/mont/
// bls12_381_Fp2_mont.c:150-215; bn128_Fp2_mont.c same layout): both BN128 and BLS12-381
// use u^2 = -1, c0 = a0 b0 - a1 b1, c1 = a0 b1 + a1 b0 (Karatsuba, 3 base products).
// An element is stored as the base field's limbs of c0 followed by those of c1
// (Fe<F2<B>>::v[0..N) = c0, v[N..2N) = c1); the reference layout (c0 || c1, N64 u64 each)
// is kept at every HBM boundary.  The generic curve / MSM templates (zk_curve.hpp,
// zk_msm.hip) instantiate unchanged on F2<B>: every field primitive they call has an
// overload here, picked by partial ordering.
#pragma once
#include "zk_field.hpp"

namespace zk {

template <class B>
struct F2 {
  using Base = B;
  static constexpr int N = 2 * B::N;
  static constexpr int SN = 2 * B::SN;
  static constexpr int N64 = 2 * B::N64;
  static constexpr int NW = 2 * B::NW;
  static constexpr int RB = B::RB;
};

// G1 (base field) or G2 (Fp2) point coordinates: the paths tuned and measured on G1 only (the
// curve-aware window table, the quad-cooperative stitch and Y-sum fold) gate on this
template <class F>
struct IsF2 {
  static constexpr bool value = false;
};
template <class B>
struct IsF2<F2<B>> {
  static constexpr bool value = true;
};
template <class F>
constexpr bool is_base_field() { return !IsF2<F>::value; }

template <class B>
__device__ __forceinline__ void f2_split(Fe<B> &c0, Fe<B> &c1, const Fe<F2<B>> &a) {
#pragma unroll
  for (int i = 0; i < B::N; i++) {
    c0.v[i] = a.v[i];
    c1.v[i] = a.v[B::N + i];
  }
}
template <class B>
__device__ __forceinline__ void f2_join(Fe<F2<B>> &r, const Fe<B> &c0, const Fe<B> &c1) {
#pragma unroll
  for (int i = 0; i < B::N; i++) {
    r.v[i] = c0.v[i];
    r.v[B::N + i] = c1.v[i];
  }
}

template <class B>
__device__ __forceinline__ void fe_zero(Fe<F2<B>> &r) {
#pragma unroll
  for (int i = 0; i < 2 * B::N; i++) r.v[i] = 0;
}
template <class B>
__device__ __forceinline__ void fe_one(Fe<F2<B>> &r) {
  Fe<B> o, z;
  fe_one(o);
  fe_zero(z);
  f2_join(r, o, z);
}
template <class B>
__device__ __forceinline__ bool fe_is_zero(const Fe<F2<B>> &a) {
  Fe<B> a0, a1;
  f2_split(a0, a1, a);
  return fe_is_zero(a0) && fe_is_zero(a1);
}
template <class B>
__device__ __forceinline__ void fe_add(Fe<F2<B>> &r, const Fe<F2<B>> &a, const Fe<F2<B>> &b) {
  Fe<B> a0, a1, b0, b1, r0, r1;
  f2_split(a0, a1, a);
  f2_split(b0, b1, b);
  fe_add(r0, a0, b0);
  fe_add(r1, a1, b1);
  f2_join(r, r0, r1);
}
template <class B>
__device__ __forceinline__ void fe_sub(Fe<F2<B>> &r, const Fe<F2<B>> &a, const Fe<F2<B>> &b) {
  Fe<B> a0, a1, b0, b1, r0, r1;
  f2_split(a0, a1, a);
  f2_split(b0, b1, b);
  fe_sub(r0, a0, b0);
  fe_sub(r1, a1, b1);
  f2_join(r, r0, r1);
}
template <class B>
__device__ __forceinline__ void fe_neg(Fe<F2<B>> &r, const Fe<F2<B>> &a) {
  Fe<F2<B>> z;
  fe_zero(z);
  fe_sub(r, z, a);
}
template <class B>
__device__ __forceinline__ void fe_mul3(Fe<F2<B>> &r, const Fe<F2<B>> &a) {
  Fe<F2<B>> t;
  fe_add(t, a, a);
  fe_add(r, t, a);
}
#ifndef ZK_FP2_LAZY
#define ZK_FP2_LAZY 1  // 0: three full Montgomery products (A/B hook)
#endif
// c0 = a0 b0 - a1 b1, c1 = a0 b1 + a1 b0 as two shared-reduction pairs (fe_mul2: the column sums of
// two products, one Montgomery reduction): c0 = REDC(a0 b0 + a1 (2p - b1)), c1 = REDC(a0 b1 + a1 b0).
// Four limb products and two reductions instead of Karatsuba's three products and three
// reductions, and none of its five exact additions / subtractions (each two carry chains).
// Operands < 2p with normalised limbs (what every G2 producer -- the exact add / sub / mul --
// gives) -> both pairs < 8p^2 < p R' (R'/p = 2^11 on BLS12-381, 2^7.4 on BN254), outputs < 2p,
// columns as fe_mul2's (zk_params.inc asserts their bound).  tests/test_fp2_lazy.py runs a
// bit-level model of it against big-integer Fp2 arithmetic on extreme operands.
template <class B>
__device__ __forceinline__ void fe_mul(Fe<F2<B>> &r, const Fe<F2<B>> &a, const Fe<F2<B>> &b) {
  Fe<B> a0, a1, b0, b1, r0, r1;
  f2_split(a0, a1, a);
  f2_split(b0, b1, b);
#if ZK_FP2_LAZY
  Fe<B> nb1;
  fe_sub_lazy<B, 2, 1>(nb1, Fe<B>{}, b1);  // 2p - b1, in (0, 2p]
  fe_norm(nb1);
  fe_mul2(r0, a0, b0, a1, nb1);  // schoolbook streaming pairs: the Karatsuba-column form (fe_mul2k)
  fe_mul2(r1, a0, b1, a1, b0);   // held two column arrays and spilled ~360 VGPRs in the G2 madd
#else
  Fe<B> t0, t1, s, u, m;
  fe_mul(t0, a0, b0);
  fe_mul(t1, a1, b1);
  fe_add(s, a0, a1);
  fe_add(u, b0, b1);
  fe_mul(m, s, u);
  fe_sub(r0, t0, t1);
  fe_sub(m, m, t0);
  fe_sub(r1, m, t1);
#endif
  f2_join(r, r0, r1);
}
// (a0 + a1 u)^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u
template <class B>
__device__ __forceinline__ void fe_sqr(Fe<F2<B>> &r, const Fe<F2<B>> &a) {
  Fe<B> a0, a1, s, d, r0, r1, t;
  f2_split(a0, a1, a);
  fe_add(s, a0, a1);
  fe_sub(d, a0, a1);
  fe_mul(r0, s, d);
  fe_mul(t, a0, a1);
  fe_add(r1, t, t);
  f2_join(r, r0, r1);
}
template <class B>
__device__ __forceinline__ void fe_canon(Fe<F2<B>> &a) {
  Fe<B> a0, a1;
  f2_split(a0, a1, a);
  fe_canon(a0);
  fe_canon(a1);
  f2_join(a, a0, a1);
}
// radix conversions are linear: component-wise
template <class B>
__device__ __forceinline__ void fe_to_int(Fe<F2<B>> &r, const Fe<F2<B>> &a) {
  Fe<B> a0, a1, r0, r1;
  f2_split(a0, a1, a);
  fe_to_int(r0, a0);
  fe_to_int(r1, a1);
  f2_join(r, r0, r1);
}
template <class B>
__device__ __forceinline__ void fe_to_ref(Fe<F2<B>> &r, const Fe<F2<B>> &a) {
  Fe<B> a0, a1, r0, r1;
  f2_split(a0, a1, a);
  fe_to_ref(r0, a0);
  fe_to_ref(r1, a1);
  f2_join(r, r0, r1);
}
template <class B>
__device__ __forceinline__ void fe_load_ref(Fe<F2<B>> &r, const uint64_t *__restrict__ p) {
  Fe<B> r0, r1;
  fe_load_ref(r0, p);
  fe_load_ref(r1, p + B::N64);
  f2_join(r, r0, r1);
}
template <class B>
__device__ __forceinline__ void fe_store_ref(uint64_t *__restrict__ p, const Fe<F2<B>> &a) {
  Fe<B> a0, a1;
  f2_split(a0, a1, a);
  fe_store_ref(p, a0);
  fe_store_ref(p + B::N64, a1);
}

}  // namespace zk
