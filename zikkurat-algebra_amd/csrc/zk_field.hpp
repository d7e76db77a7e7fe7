// zk_field.hpp -- prime-field arithmetic in Montgomery form for gfx950 (device)
//
// Replaces, on the GPU, the reference's generated per-field C:
//   <C>_Fp_mont_{add,sub,neg,mul,sqr} / <C>_Fr_mont_*  (lib/cbits/curves/fields/mont/
//   bls12_381_Fp_mont.c:44-215, bls12_381_Fr_mont.c:44-199, bn128_*_mont.c same lines)
//   and the bigint256/384 limb kernels under them (lib/cbits/bigint/bigint256.c:108-356).
//
// Representation: the SAME Montgomery representation as the reference (R = 2^(64*n64):
// 2^256 for BN128 Fp/Fr and BLS12-381 Fr, 2^384 for BLS12-381 Fp), stored as 2*n64
// little-endian 32-bit limbs in registers -- the natural VALU word on CDNA4
// (v_mad_u64_u32 gives a 32x32+64 -> 64 product-accumulate in one instruction).
// Every operation returns the canonical representative (< p) for canonical inputs,
// exactly like the reference (sub_prime_if_above / add-prime-on-borrow, Fr_mont.c:72-116),
// so results are bit-identical regardless of the algorithm that produced them.
//
// Multiplication is the "no-carry" CIOS variant: valid because every one of the four
// primes leaves its top 32-bit limb below (2^32-1)/2 (spare bits: BN 2, BLS-Fr 1, BLS-Fp 3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zk_params.inc"

namespace zk {

// ---------------------------------------------------------------------------
// Field descriptors (compile-time constants; indices are always unrolled so the
// limbs of p become scalar operands / inline constants, never memory loads).

#define ZK_DEFINE_FIELD(NAME, PFX)                                                  \
  struct NAME {                                                                     \
    static constexpr int N = PFX##_N32;     /* 32-bit limbs */                      \
    static constexpr int N64 = PFX##_N64;                                           \
    static constexpr int BITS = PFX##_BITS;                                         \
    static constexpr uint32_t MINV = PFX##_MINV32;                                  \
    __host__ __device__ static constexpr uint32_t p(int i) {                        \
      constexpr uint32_t P_[] = PFX##_P32; return P_[i]; }                          \
    __host__ __device__ static constexpr uint32_t one(int i) {                      \
      constexpr uint32_t R_[] = PFX##_R32; return R_[i]; }                          \
    __host__ __device__ static constexpr uint32_t r2(int i) {                       \
      constexpr uint32_t R2_[] = PFX##_R2_32; return R2_[i]; }                      \
  };

ZK_DEFINE_FIELD(BN_Fp,  ZK_BN128_FP)
ZK_DEFINE_FIELD(BN_Fr,  ZK_BN128_FR)
ZK_DEFINE_FIELD(BLS_Fp, ZK_BLS12_381_FP)
ZK_DEFINE_FIELD(BLS_Fr, ZK_BLS12_381_FR)

template <class F>
struct Fe {
  uint32_t v[F::N];
};

// ---------------------------------------------------------------------------
// limb-level helpers

__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t &cout) {
  uint32_t c;
  uint32_t r = __builtin_addc(a, b, cin, &c);
  cout = c;
  return r;
}
__device__ __forceinline__ uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t &bout) {
  uint32_t c;
  uint32_t r = __builtin_subc(a, b, bin, &c);
  bout = c;
  return r;
}

template <class F>
__device__ __forceinline__ void fe_zero(Fe<F> &r) {
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = 0;
}
template <class F>
__device__ __forceinline__ void fe_one(Fe<F> &r) {
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = F::one(i);
}
template <class F>
__device__ __forceinline__ bool fe_is_zero(const Fe<F> &a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) acc |= a.v[i];
  return acc == 0;
}
template <class F>
__device__ __forceinline__ bool fe_eq(const Fe<F> &a, const Fe<F> &b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) acc |= (a.v[i] ^ b.v[i]);
  return acc == 0;
}

// r = (a >= p) ? a - p : a      (a < 2p assumed)
template <class F>
__device__ __forceinline__ void fe_reduce_once(Fe<F> &a) {
  uint32_t t[F::N];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) t[i] = subb(a.v[i], F::p(i), br, br);
  // br == 1  <=> a < p  -> keep a
#pragma unroll
  for (int i = 0; i < F::N; i++) a.v[i] = br ? a.v[i] : t[i];
}

template <class F>
__device__ __forceinline__ void fe_add(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = addc(a.v[i], b.v[i], c, c);
  // spare top bit => no carry out of the top limb
  fe_reduce_once(r);
}

template <class F>
__device__ __forceinline__ void fe_sub(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = subb(a.v[i], b.v[i], br, br);
  const uint32_t mask = 0u - br;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = addc(r.v[i], F::p(i) & mask, c, c);
}

template <class F>
__device__ __forceinline__ void fe_neg(Fe<F> &r, const Fe<F> &a) {
  // p - a, and 0 -> 0 (reference: Fr_mont.c:44-58)
  const uint32_t nz = fe_is_zero(a) ? 0u : 0xffffffffu;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = subb(F::p(i) & nz, a.v[i], br, br);
}

template <class F>
__device__ __forceinline__ void fe_dbl(Fe<F> &r, const Fe<F> &a) { fe_add(r, a, a); }

// Montgomery product, "no-carry" CIOS with 32-bit limbs.
//   t = a*b*2^(-32N) mod p, canonical.
template <class F>
__device__ __forceinline__ void fe_mul(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  constexpr int N = F::N;
  uint32_t t[N];
#pragma unroll
  for (int j = 0; j < N; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint32_t bi = b.v[i];
    uint64_t x = (uint64_t)a.v[0] * bi + t[0];
    uint32_t A = (uint32_t)(x >> 32);
    const uint32_t t0 = (uint32_t)x;
    const uint32_t m = t0 * F::MINV;
    uint64_t y = (uint64_t)m * F::p(0) + t0;
    uint32_t C = (uint32_t)(y >> 32);
#pragma unroll
    for (int j = 1; j < N; j++) {
      x = (uint64_t)a.v[j] * bi + t[j];
      x += A;
      A = (uint32_t)(x >> 32);
      y = (uint64_t)m * F::p(j) + (uint32_t)x;
      y += C;
      C = (uint32_t)(y >> 32);
      t[j - 1] = (uint32_t)y;
    }
    t[N - 1] = C + A;
  }
#pragma unroll
  for (int j = 0; j < N; j++) r.v[j] = t[j];
  fe_reduce_once(r);
}

template <class F>
__device__ __forceinline__ void fe_sqr(Fe<F> &r, const Fe<F> &a) { fe_mul(r, a, a); }

// REDC of a single-width value: a * R^-1 mod p  (the reference's `to_std`,
// Fr_mont.c:330-335: REDC of [a, 0]; canonical for every a < 2^(32N)).
template <class F>
__device__ __forceinline__ void fe_from_mont(Fe<F> &r, const Fe<F> &a) {
  Fe<F> one;
#pragma unroll
  for (int i = 0; i < F::N; i++) one.v[i] = (i == 0) ? 1u : 0u;
  fe_mul(r, a, one);
}

// small-integer multiples used by the curve formulas
template <class F>
__device__ __forceinline__ void fe_mul3(Fe<F> &r, const Fe<F> &a) {
  Fe<F> t;
  fe_add(t, a, a);
  fe_add(r, t, a);
}

// ---------------------------------------------------------------------------
// memory helpers: limbs are stored in HBM as little-endian u64 words, which is
// byte-identical to little-endian u32 limbs.

template <class F>
__device__ __forceinline__ void fe_load(Fe<F> &r, const uint64_t *__restrict__ p) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
  for (int i = 0; i < F::N / 4; i++) {
    uint4 w = q[i];
    r.v[4 * i + 0] = w.x;
    r.v[4 * i + 1] = w.y;
    r.v[4 * i + 2] = w.z;
    r.v[4 * i + 3] = w.w;
  }
}
template <class F>
__device__ __forceinline__ void fe_store(uint64_t *__restrict__ p, const Fe<F> &a) {
  uint4 *q = reinterpret_cast<uint4 *>(p);
#pragma unroll
  for (int i = 0; i < F::N / 4; i++) {
    q[i] = make_uint4(a.v[4 * i + 0], a.v[4 * i + 1], a.v[4 * i + 2], a.v[4 * i + 3]);
  }
}

}  // namespace zk
