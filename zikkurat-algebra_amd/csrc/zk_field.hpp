// zk_field.hpp -- prime-field arithmetic for gfx950 (device), unsaturated limbs.
//
// Replaces, on the GPU, the reference's generated per-field C:
//   <C>_Fp_mont_{add,sub,neg,mul,sqr} / <C>_Fr_mont_*  (lib/cbits/curves/fields/mont/
//   bls12_381_Fp_mont.c:44-215, bls12_381_Fr_mont.c:44-199, bn128_*_mont.c same lines)
//   and the bigint256/384 limb kernels under them (lib/cbits/bigint/bigint256.c:108-356).
//
// Why unsaturated: on CDNA4 `v_mad_u64_u32` (32x32 + 64 -> 64) issues at close to the
// plain-add rate (tools/microbench/field_rates.hip: 25 Tops/s vs 32), so the cheapest
// multiprecision product is one mad per limb product with NO carry handling.  With limbs
// of RB = 28/29 bits a whole product-scanning column (<= 2N products of < 2^(2RB)) fits
// in one 64-bit accumulator.  Measured: 70 vs 39 G mul/s (381-bit) over 32-bit CIOS.
//
//   field          limbs x bits   internal Montgomery radix R'
//   BN128 Fp, Fr    9 x 29        2^261
//   BLS12-381 Fr    9 x 29        2^261
//   BLS12-381 Fp   14 x 28        2^392
//
// Values: normalized limbs (< 2^RB), integer value < 2p, Montgomery form w.r.t. R'.
// The reference's representation (R = 2^256 / 2^384, u64 limbs, canonical) is used
// at every HBM boundary: fe_load_ref/fe_store_ref repack the bits, fe_to_int /
// fe_to_ref convert between R and R' with one product by a constant (KIN, KOUT).
// For linear maps (the NTT) no radix conversion is needed at all: a reference-form
// value x*R multiplied by an internal-form twiddle w*R' yields (x w)*R.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zk_inv.hpp"
#include "zk_params.inc"

namespace zk {

#define ZK_DEFINE_FIELD(NAME, PFX)                                                      \
  struct NAME {                                                                         \
    static constexpr int N = PFX##_U_N;      /* limbs */                                \
    static constexpr int RB = PFX##_U_RB;    /* bits per limb */                        \
    static constexpr uint32_t MASK = (1u << PFX##_U_RB) - 1;                            \
    static constexpr uint32_t MINV = PFX##_U_MINV;                                      \
    static constexpr int N64 = PFX##_N64;    /* reference u64 limbs */                  \
    static constexpr int NW = 2 * PFX##_N64; /* reference u32 words */                  \
    static constexpr int SN = (PFX##_U_N + 3) & ~3; /* storage stride (u32) */          \
    __host__ __device__ static constexpr uint32_t p(int i) {                            \
      constexpr uint32_t v_[] = PFX##_U_P; return v_[i]; }                              \
    __host__ __device__ static constexpr uint32_t p2(int i) {                           \
      constexpr uint32_t v_[] = PFX##_U_P2; return v_[i]; }                             \
    __host__ __device__ static constexpr uint32_t one(int i) {                          \
      constexpr uint32_t v_[] = PFX##_U_ONE; return v_[i]; }                            \
    __host__ __device__ static constexpr uint32_t kin(int i) {                          \
      constexpr uint32_t v_[] = PFX##_U_KIN; return v_[i]; }                            \
    __host__ __device__ static constexpr uint32_t kout(int i) {                         \
      constexpr uint32_t v_[] = PFX##_U_KOUT; return v_[i]; }                           \
    __host__ __device__ static constexpr uint32_t kstd(int i) {                         \
      constexpr uint32_t v_[] = PFX##_U_KSTD; return v_[i]; }                           \
    __host__ __device__ static constexpr uint32_t k3(int i) {                           \
      constexpr uint32_t v_[] = PFX##_U_K3; return v_[i]; }                             \
    static constexpr int S62_L = PFX##_S62_L;           /* safegcd limbs (zk_inv.hpp) */ \
    static constexpr int S62_NB = PFX##_S62_BATCHES;    /* 62-divstep batches */       \
    static constexpr uint64_t S62_PINV = PFX##_S62_PINV;                              \
    __host__ __device__ static constexpr int64_t s62p(int i) {                          \
      constexpr int64_t v_[] = PFX##_S62_P; return v_[i]; }                           \
    static constexpr int S60_L = PFX##_S60_L;           /* 60-bit limbs, 2 x 30 steps */ \
    static constexpr int S60_NB = PFX##_S60_BATCHES;                                   \
    __host__ __device__ static constexpr int64_t s60p(int i) {                          \
      constexpr int64_t v_[] = PFX##_S60_P; return v_[i]; }                           \
  };

ZK_DEFINE_FIELD(BN_Fp, ZK_BN128_FP)
ZK_DEFINE_FIELD(BN_Fr, ZK_BN128_FR)
ZK_DEFINE_FIELD(BLS_Fp, ZK_BLS12_381_FP)
ZK_DEFINE_FIELD(BLS_Fr, ZK_BLS12_381_FR)

template <class F>
struct Fe {
  uint32_t v[F::N];
};

// ---------------------------------------------------------------------------- basics

template <class F>
__device__ __forceinline__ void fe_zero(Fe<F> &r) {
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = 0;
}
template <class F>
__device__ __forceinline__ void fe_one(Fe<F> &r) {  // internal-form 1 (R' mod p)
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = F::one(i);
}
template <class F>
__device__ __forceinline__ void fe_const_kin(Fe<F> &r) {
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = F::kin(i);
}
// value == 0 (mod p), for values < 2p
template <class F>
__device__ __forceinline__ bool fe_is_zero(const Fe<F> &a) {
  uint32_t z = 0, q = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    z |= a.v[i];
    q |= a.v[i] ^ F::p(i);
  }
  return z == 0 || q == 0;
}

// r = a + b  (mod 2p representative: result < 2p).  Two carry chains (a+b and
// a+b-2p) run interleaved; the sign of the second selects.
template <class F>
__device__ __forceinline__ void fe_add(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  int32_t c0 = 0, c1 = 0;
  uint32_t s0[F::N], s1[F::N];
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    const int32_t t = (int32_t)(a.v[i] + b.v[i]);
    const int32_t v0 = t + c0;
    const int32_t v1 = t - (int32_t)F::p2(i) + c1;
    s0[i] = (uint32_t)v0 & F::MASK;
    s1[i] = (uint32_t)v1 & F::MASK;
    c0 = v0 >> F::RB;
    c1 = v1 >> F::RB;
  }
  const bool ge = c1 >= 0;  // a + b >= 2p
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = ge ? s1[i] : s0[i];
}

// r = a - b  (result < 2p): a-b if >= 0 else a-b+2p
template <class F>
__device__ __forceinline__ void fe_sub(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  int32_t c0 = 0, c1 = 0;
  uint32_t s0[F::N], s1[F::N];
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    const int32_t t = (int32_t)a.v[i] - (int32_t)b.v[i];
    const int32_t v0 = t + c0;
    const int32_t v1 = t + (int32_t)F::p2(i) + c1;
    s0[i] = (uint32_t)v0 & F::MASK;
    s1[i] = (uint32_t)v1 & F::MASK;
    c0 = v0 >> F::RB;
    c1 = v1 >> F::RB;
  }
  const bool neg = c0 < 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = neg ? s1[i] : s0[i];
}

template <class F>
__device__ __forceinline__ void fe_neg(Fe<F> &r, const Fe<F> &a) {
  Fe<F> z;
  fe_zero(z);
  fe_sub(r, z, a);
}

template <class F>
__device__ __forceinline__ void fe_dbl(Fe<F> &r, const Fe<F> &a) { fe_add(r, a, a); }

template <class F>
__device__ __forceinline__ void fe_mul3(Fe<F> &r, const Fe<F> &a) {
  Fe<F> t;
  fe_add(t, a, a);
  fe_add(r, t, a);
}

// Montgomery product w.r.t. R' = 2^(RB*N): product scanning (FIPS) with one 64-bit
// column accumulator; every limb product is a single v_mad_u64_u32.
// Inputs < 2p (normalized limbs) -> output < 2p (normalized), since 4p < R'.
template <class F>
__device__ __forceinline__ void fe_mul(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  constexpr int N = F::N;
  uint32_t m[N];
  uint32_t o[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < N; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)m[i] * F::p(k - i);
    }
    acc += (uint64_t)a.v[k] * b.v[0];
    m[k] = ((uint32_t)acc * F::MINV) & F::MASK;
    acc += (uint64_t)m[k] * F::p(0);
    acc >>= F::RB;
  }
#pragma unroll
  for (int k = N; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = k - N + 1; i < N; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)m[i] * F::p(k - i);
    }
    o[k - N] = (uint32_t)acc & F::MASK;
    acc >>= F::RB;
  }
  o[N - 1] = (uint32_t)acc;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = o[i];
}

// r = (a*b + c*d) / R'  -- two products sharing ONE Montgomery reduction (lazy
// reduction): 2N^2 + N^2 mads instead of 4N^2.  Column sums hold 2N products of each
// kind, so the operand limbs must be small enough (see callers); inputs whose
// a*b + c*d < p*R' give an output < 2p.
template <class F>
__device__ __forceinline__ void fe_mul2(Fe<F> &r, const Fe<F> &a, const Fe<F> &b, const Fe<F> &c,
                                        const Fe<F> &d) {
  constexpr int N = F::N;
  uint32_t m[N];
  uint32_t o[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < N; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)c.v[i] * d.v[k - i];
      acc += (uint64_t)m[i] * F::p(k - i);
    }
    acc += (uint64_t)a.v[k] * b.v[0];
    acc += (uint64_t)c.v[k] * d.v[0];
    m[k] = ((uint32_t)acc * F::MINV) & F::MASK;
    acc += (uint64_t)m[k] * F::p(0);
    acc >>= F::RB;
  }
#pragma unroll
  for (int k = N; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = k - N + 1; i < N; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)c.v[i] * d.v[k - i];
      acc += (uint64_t)m[i] * F::p(k - i);
    }
    o[k - N] = (uint32_t)acc & F::MASK;
    acc >>= F::RB;
  }
  o[N - 1] = (uint32_t)acc;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = o[i];
}

// ---- one Karatsuba level on the a*b part (even N; used for the 14-limb 381-bit field):
//   a b = z0 + (z0 + z2 + z1') 2^(H RB) + z2 2^(2 H RB),  H = N/2,
//   z0 = a_lo b_lo, z2 = a_hi b_hi, z1' = (a_lo - a_hi)(b_hi - b_lo)  (signed 32-bit differences,
//   v_mad_i64_i32), so 3 H^2 limb products instead of N^2.  Column k of a b (kara_cols) equals
// the schoolbook column sum exactly, so the interleaved REDC (redc_cols) sees the same column
// values and bounds as fe_mul (tools/lazy_bounds.py); the middle columns are formed in
// wrapping u64 arithmetic (the true value, a_lo b_hi + a_hi b_lo, is >= 0 and < 2^64).
// Static A/B (tools/experiments/kara_isa.hip): 436 vs 472 issue slots per 381-bit product.
template <class F>
__device__ __forceinline__ void kara_cols(uint64_t (&T)[2 * F::N - 1], const Fe<F> &a, const Fe<F> &b,
                                          bool accumulate) {
  constexpr int N = F::N, H = N / 2;
  static_assert(N % 2 == 0, "Karatsuba split needs an even limb count");
  int32_t da[H], db[H];
#pragma unroll
  for (int i = 0; i < H; i++) {
    da[i] = (int32_t)a.v[i] - (int32_t)a.v[i + H];
    db[i] = (int32_t)b.v[i + H] - (int32_t)b.v[i];
  }
  uint64_t z0[2 * H - 1], z2[2 * H - 1], mid[2 * H - 1];
#pragma unroll
  for (int k = 0; k < 2 * H - 1; k++) {
    uint64_t s0 = 0, s2 = 0;
#pragma unroll
    for (int i = 0; i < H; i++) {
      const int j = k - i;
      if (j < 0 || j >= H) continue;
      s0 += (uint64_t)a.v[i] * b.v[j];
      s2 += (uint64_t)a.v[i + H] * b.v[j + H];
    }
    z0[k] = s0;
    z2[k] = s2;
    uint64_t s1 = s0 + s2;
#pragma unroll
    for (int i = 0; i < H; i++) {
      const int j = k - i;
      if (j < 0 || j >= H) continue;
      s1 += (uint64_t)((int64_t)da[i] * (int64_t)db[j]);
    }
    mid[k] = s1;
  }
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint64_t t = accumulate ? T[k] : 0;
    if (k < 2 * H - 1) t += z0[k];
    if (k >= H && k - H < 2 * H - 1) t += mid[k - H];
    if (k >= 2 * H && k - 2 * H < 2 * H - 1) t += z2[k - 2 * H];
    T[k] = t;
  }
}
// Montgomery reduction of product-scanning column sums T (the m*p part interleaved as in fe_mul)
template <class F>
__device__ __forceinline__ void redc_cols(Fe<F> &r, const uint64_t (&T)[2 * F::N - 1]) {
  constexpr int N = F::N;
  uint32_t m[N], o[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < N; k++) {
    acc += T[k];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * F::p(k - i);
    m[k] = ((uint32_t)acc * F::MINV) & F::MASK;
    acc += (uint64_t)m[k] * F::p(0);
    acc >>= F::RB;
  }
#pragma unroll
  for (int k = N; k < 2 * N - 1; k++) {
    acc += T[k];
#pragma unroll
    for (int i = k - N + 1; i < N; i++) acc += (uint64_t)m[i] * F::p(k - i);
    o[k - N] = (uint32_t)acc & F::MASK;
    acc >>= F::RB;
  }
  o[N - 1] = (uint32_t)acc;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = o[i];
}
// The same reduction in operand-scanning order: digit m_k is formed as soon as column k holds
// its carry, and its row m_k p_j is added to the 14 later columns at once (independent
// v_mad_u64_u32, no chain through one accumulator); only mul_lo -> mad -> shift -> add per digit
// is serial.  Every column ends with the same sum as in redc_cols (the terms are added in another
// order, all non-negative), so tools/lazy_bounds.py's column bounds hold unchanged.
template <class F>
__device__ __forceinline__ void redc_rows(Fe<F> &r, uint64_t (&T)[2 * F::N - 1]) {
  constexpr int N = F::N;
#pragma unroll
  for (int k = 0; k < N; k++) {
    const uint32_t m = ((uint32_t)T[k] * F::MINV) & F::MASK;
#pragma unroll
    for (int j = 0; j < N; j++) T[k + j] += (uint64_t)m * F::p(j);
    T[k + 1] += T[k] >> F::RB;  // the low RB bits of T[k] are now zero
  }
  uint64_t acc = 0;
#pragma unroll
  for (int k = N; k < 2 * N - 1; k++) {
    acc += T[k];
    r.v[k - N] = (uint32_t)acc & F::MASK;
    acc >>= F::RB;
  }
  r.v[N - 1] = (uint32_t)acc;
}
#ifndef ZK_REDC_ROWS
#define ZK_REDC_ROWS 0  // A/B: 1 = redc_rows in the Karatsuba products below
#endif
template <class F>
__device__ __forceinline__ void redc_k(Fe<F> &r, uint64_t (&T)[2 * F::N - 1]) {
  if constexpr (ZK_REDC_ROWS) redc_rows(r, T); else redc_cols(r, T);
}
// the product / shared-reduction pair with the Karatsuba column sums (14-limb field), the
// schoolbook ones otherwise
template <class F>
__device__ __forceinline__ void fe_mulk(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  if constexpr (F::N == 14) {
    uint64_t T[2 * F::N - 1];
    kara_cols(T, a, b, false);
    redc_k(r, T);
  } else {
    fe_mul(r, a, b);
  }
}
template <class F>
__device__ __forceinline__ void fe_mul2k(Fe<F> &r, const Fe<F> &a, const Fe<F> &b, const Fe<F> &c, const Fe<F> &d) {
  if constexpr (F::N == 14) {
    uint64_t T[2 * F::N - 1];
    kara_cols(T, a, b, false);
    kara_cols(T, c, d, true);
    redc_k(r, T);
  } else {
    fe_mul2(r, a, b, c, d);
  }
}

// squaring: off-diagonal products once, doubled (saves ~N^2/2 mads)
template <class F>
__device__ __forceinline__ void fe_sqr(Fe<F> &r, const Fe<F> &a) {
  constexpr int N = F::N;
  uint32_t a2[N];
#pragma unroll
  for (int i = 0; i < N; i++) a2[i] = a.v[i] << 1;
  uint32_t m[N];
  uint32_t o[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    // a-part of column k: sum_{i<j, i+j=k} 2 a_i a_j  +  a_{k/2}^2
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j > i && j < N) acc += (uint64_t)a2[i] * a.v[j];
    }
    if ((k & 1) == 0 && (k >> 1) < N) acc += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
    // m-part
    if (k < N) {
#pragma unroll
      for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * F::p(k - i);
      m[k] = ((uint32_t)acc * F::MINV) & F::MASK;
      acc += (uint64_t)m[k] * F::p(0);
      acc >>= F::RB;
    } else {
#pragma unroll
      for (int i = k - N + 1; i < N; i++) acc += (uint64_t)m[i] * F::p(k - i);
      o[k - N] = (uint32_t)acc & F::MASK;
      acc >>= F::RB;
    }
  }
  o[N - 1] = (uint32_t)acc;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = o[i];
}

// x^e for a kernel-uniform exponent of nw 64-bit words (Fermat inversions): left-to-right
// sliding window of width 3 over the odd powers x, x^3, x^5, x^7, i.e. ~bits squarings plus one
// product per window.  For the BLS12-381 base prime (p - 2: 381 bits, 229 ones) ~485 products
// instead of square-and-multiply's 610; for its scalar field (r - 2: 255 bits, 164 ones) ~330
// instead of 419.  Every branch depends on the exponent only, so the lanes never diverge.
template <class F>
__device__ __forceinline__ void fe_pow_sw(Fe<F> &r, const Fe<F> &x, const uint64_t *e, int nw) {
  auto bit = [&](int i) -> uint32_t { return (uint32_t)(e[i >> 6] >> (i & 63)) & 1u; };
  Fe<F> x2, x3, x5, x7, t;
  fe_sqr(x2, x);
  fe_mul(x3, x, x2);
  fe_mul(x5, x3, x2);
  fe_mul(x7, x5, x2);
  int i = nw * 64 - 1;
  while (i >= 0 && !bit(i)) i--;
  fe_one(r);
  bool started = false;
  while (i >= 0) {
    if (!bit(i)) {
      fe_sqr(t, r);
      r = t;
      i--;
      continue;
    }
    int j = i >= 2 ? i - 2 : 0;  // window [i .. j], ending in a set bit
    while (!bit(j)) j++;
    uint32_t val = 0;
    for (int k = i; k >= j; k--) val = (val << 1) | bit(k);
    if (started)
      for (int k = i; k >= j; k--) {
        fe_sqr(t, r);
        r = t;
      }
    if (!started) r = val == 1 ? x : (val == 3 ? x3 : (val == 5 ? x5 : x7));
    else if (val == 1) { fe_mul(t, r, x); r = t; }
    else if (val == 3) { fe_mul(t, r, x3); r = t; }
    else if (val == 5) { fe_mul(t, r, x5); r = t; }
    else { fe_mul(t, r, x7); r = t; }
    started = true;
    i = j - 1;
  }
}

// ---------------------------------------------------------------------------- lazy ops
// Redundant arithmetic for chains of additions (NTT butterflies).  The unsaturated
// limbs leave 32 - RB bits of headroom per limb and R'/p >= 2^(RB*N)/p spare value
// range, so sums need no carry handling and no reduction:
//   fe_add_lazy  r_i = a_i + b_i
//   fe_sub_lazy  r_i = a_i + kp_i - b_i, kp = K*p written with "borrowed" limbs
//                (every limb below the top >= BW*(2^RB - 1)), so no limb goes negative
//                as long as b's limbs are <= BW*(2^RB - 1) and b's top limb fits.
//   fe_norm      carry-propagate back to RB-bit limbs (value unchanged)
// fe_mul accepts one operand with limbs < 2^31 (the column sums stay < 2^64) and maps
// any value < (R'/p) * p to < 2p when the other operand is < p, which is how the NTT
// brings lazily-grown values back into range.
template <class F, int K>
__host__ __device__ constexpr uint32_t kp_limb(int i) {  // limb i of K*p, RB-bit limbs
  uint64_t carry = 0;
  uint32_t out = 0;
  for (int j = 0; j <= i; j++) {
    const uint64_t v = (uint64_t)F::p(j) * K + carry;
    out = (j == F::N - 1) ? (uint32_t)v : (uint32_t)(v & F::MASK);
    carry = v >> F::RB;
  }
  return out;
}
template <class F, int K, int BW>
__host__ __device__ constexpr uint32_t kp_borrowed(int i) {
  return i == 0 ? kp_limb<F, K>(0) + ((uint32_t)BW << F::RB)
                : (i < F::N - 1 ? kp_limb<F, K>(i) + ((uint32_t)BW << F::RB) - BW : kp_limb<F, K>(i) - BW);
}
template <class F>
__device__ __forceinline__ void fe_add_lazy(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = a.v[i] + b.v[i];
}
template <class F, int K = 4, int BW = 1>
__device__ __forceinline__ void fe_sub_lazy(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = a.v[i] + kp_borrowed<F, K, BW>(i) - b.v[i];
}
template <class F>
__device__ __forceinline__ void fe_norm(Fe<F> &a) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::N - 1; i++) {
    const uint32_t v = a.v[i] + c;
    a.v[i] = v & F::MASK;
    c = v >> F::RB;
  }
  a.v[F::N - 1] += c;
}

// canonical representative (< p) of a value < 2p
template <class F>
__device__ __forceinline__ void fe_canon(Fe<F> &a) {
  int32_t c = 0;
  uint32_t d[F::N];
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    const int32_t v = (int32_t)a.v[i] - (int32_t)F::p(i) + c;
    d[i] = (uint32_t)v & F::MASK;
    c = v >> F::RB;
  }
  const bool lt = c < 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) a.v[i] = lt ? a.v[i] : d[i];
}

// normalised limbs holding a value v < 64p (< 2^261 for the 9 x 29-bit fields) -> same
// residue, < 2p, without a product: q = floor(v / p) is estimated from the top limb with a
// reciprocal of p's top 64 bits (q_est = q or q - 1), then v - q_est p.  ~40 VALU ops
// instead of a Montgomery product by one (the NTT's last-pass closing step).
template <class F>
__host__ __device__ constexpr uint64_t fe_qk() {  // floor(2^64 / (floor(p / 2^(RB (N-1) - 32)) + 1))
  static_assert(F::N == 9 && F::RB == 29, "derived for the 9 x 29-bit fields");
  // p / 2^200 from limbs 6 (bits 174..202), 7 (203..231), 8 (232..260)
  return ~0ull / ((((uint64_t)F::p(8) << 32) | ((uint64_t)F::p(7) << 3) | (F::p(6) >> 26)) + 1);
}
template <class F>
__device__ __forceinline__ void fe_reduce_small(Fe<F> &v) {
  constexpr uint64_t K = fe_qk<F>();
  const uint32_t q = (uint32_t)(((uint64_t)v.v[F::N - 1] * K) >> 32);
  int64_t carry = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    const int64_t t = (int64_t)v.v[i] - (int64_t)((uint64_t)q * F::p(i)) + carry;
    v.v[i] = (i < F::N - 1) ? ((uint32_t)t & F::MASK) : (uint32_t)t;
    carry = t >> F::RB;
  }
}

// any value < (R'/2) (normalised or lazily grown limbs < 2^31) -> same residue, < 2p
template <class F>
__device__ __forceinline__ void fe_reduce(Fe<F> &a) {
  Fe<F> one, t;
  fe_one(one);
  fe_mul(t, a, one);
  a = t;
}

// ---------------------------------------------------------------------------- radix conversion

// Round 6: on the 9 x 29-bit fields R' = 2^261 = 32 R, so the radix conversions are a product by
// 32 or by 1/32 mod p -- no full Montgomery product (162 mads + bookkeeping) is needed:
//   to_int  x R -> x R' = 32 (x R):  five-bit limb shift (value < 64p < 2^261 for inputs < 2p),
//                                    then fe_reduce_small (q estimated from the top limb) -> < 2p;
//   to_ref  x R' -> x R = (x R' + k p) / 32 with k = -(x R') p^-1 mod 32 (the low five bits of one
//                                    REDC digit): nine small products and a five-bit shift -> < 1.05p.
// tools/lazy_bounds.py (radix_conv) checks both on the fields' bounds.
template <class F>
__device__ __forceinline__ void fe_mul32_small(Fe<F> &r, const Fe<F> &a) {  // a < 2p normalised -> 32a mod p, < 2p
  static_assert(F::N == 9 && F::RB == 29, "9 x 29-bit fields only");
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::N - 1; i++) {
    const uint32_t v = a.v[i];
    r.v[i] = ((v << 5) & F::MASK) | c;
    c = v >> (F::RB - 5);
  }
  r.v[F::N - 1] = (a.v[F::N - 1] << 5) | c;  // 32a < 64p < 2^261: the top limb stays < 2^29
  fe_reduce_small(r);
}
template <class F>
__device__ __forceinline__ void fe_div32_small(Fe<F> &r, const Fe<F> &a) {  // a < 2p normalised -> a / 32 mod p, < 1.05p
  static_assert(F::N == 9 && F::RB == 29, "9 x 29-bit fields only");
  const uint32_t k = (a.v[0] * F::MINV) & 31u;  // a + k p = 0 mod 32
  uint64_t t[F::N];
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) {  // a + k p, normalised to 29-bit limbs (top limb unbounded)
    const uint64_t v = (uint64_t)a.v[i] + (uint64_t)k * F::p(i) + carry;
    t[i] = (i < F::N - 1) ? (v & F::MASK) : v;
    carry = v >> F::RB;
  }
#pragma unroll
  for (int i = 0; i < F::N - 1; i++) r.v[i] = (uint32_t)((t[i] >> 5) | ((t[i + 1] << (F::RB - 5)) & F::MASK));
  r.v[F::N - 1] = (uint32_t)(t[F::N - 1] >> 5);
}
// reference Montgomery (R) -> internal (R'):  x*R  ->  x*R'
template <class F>
__device__ __forceinline__ void fe_to_int(Fe<F> &r, const Fe<F> &a) {
  if constexpr (F::N == 9 && F::RB == 29) {
    fe_mul32_small(r, a);
  } else {
    Fe<F> k;
#pragma unroll
    for (int i = 0; i < F::N; i++) k.v[i] = F::kin(i);
    fe_mul(r, a, k);
  }
}
// internal (R') -> reference Montgomery (R), canonical
template <class F>
__device__ __forceinline__ void fe_to_ref(Fe<F> &r, const Fe<F> &a) {
  if constexpr (F::N == 9 && F::RB == 29) {
    fe_div32_small(r, a);
  } else {
    Fe<F> k;
#pragma unroll
    for (int i = 0; i < F::N; i++) k.v[i] = F::kout(i);
    fe_mul(r, a, k);
  }
  fe_canon(r);
}
// reference Montgomery -> standard integer (the reference's `to_std` = REDC(x, 0),
// Fr_mont.c:330-335), canonical; valid for every 256-bit input x (a raw bit pattern).
template <class F>
__device__ __forceinline__ void fe_ref_to_std(Fe<F> &r, const Fe<F> &a) {
  Fe<F> k;
#pragma unroll
  for (int i = 0; i < F::N; i++) k.v[i] = F::kstd(i);
  fe_mul(r, a, k);
  fe_canon(r);
}

// ---------------------------------------------------------------------------- packing

// NW little-endian u32 words (any integer < 2^(32 NW)) -> RB-bit limbs
template <class F>
__device__ __forceinline__ void fe_unpack(Fe<F> &r, const uint32_t *w) {
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    const int bit = i * F::RB;
    const int wi = bit >> 5, sh = bit & 31;
    uint32_t lo = (wi < F::NW) ? w[wi] : 0u;
    uint32_t hi = (wi + 1 < F::NW) ? w[wi + 1] : 0u;
    uint32_t x = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
    r.v[i] = x & F::MASK;
  }
}
// RB-bit limbs (value < 2^(32 NW)) -> NW u32 words
template <class F>
__device__ __forceinline__ void fe_pack(uint32_t *w, const Fe<F> &a) {
#pragma unroll
  for (int j = 0; j < F::NW; j++) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < F::N; i++) {
      const int lo = i * F::RB;           // limb i covers bits [lo, lo+RB)
      const int wlo = j * 32;             // word j covers bits [wlo, wlo+32)
      if (lo + F::RB <= wlo || lo >= wlo + 32) continue;
      const int sh = lo - wlo;
      x |= sh >= 0 ? (a.v[i] << sh) : (a.v[i] >> (-sh));
    }
    w[j] = x;
  }
}

// load / store a reference-form element (N64 u64 words in HBM)
template <class F>
__device__ __forceinline__ void fe_load_ref(Fe<F> &r, const uint64_t *__restrict__ p) {
  uint32_t w[F::NW];
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
  for (int i = 0; i < F::NW / 4; i++) {
    uint4 x = q[i];
    w[4 * i] = x.x; w[4 * i + 1] = x.y; w[4 * i + 2] = x.z; w[4 * i + 3] = x.w;
  }
  fe_unpack(r, w);
}
// stores the canonical representative
template <class F>
__device__ __forceinline__ void fe_store_ref(uint64_t *__restrict__ p, const Fe<F> &a) {
  Fe<F> c = a;
  fe_canon(c);
  uint32_t w[F::NW];
  fe_pack(w, c);
  uint4 *q = reinterpret_cast<uint4 *>(p);
#pragma unroll
  for (int i = 0; i < F::NW / 4; i++) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

// Inverse in internal form by safegcd (zk_inv.hpp): a = x R' (any value < 2p, normalised limbs) ->
// x^-1 R' (< 2p).  canon(a) = x R' mod p as an integer; b = (x R')^-1 mod p by divsteps; one product
// by R'^3 gives x^-1 R'.  a = 0 gives 0.  ~18 / 12 batches of 62 divsteps (381- / 255-bit fields)
// instead of a 489 / 323-product Fermat chain (round 6).
#ifndef ZK_INV_DS30
#define ZK_INV_DS30 1  // 60-bit limbs, batches of 2 x 30 divsteps in 32-bit arithmetic; 0: 62 in 64-bit
#endif
template <class F>
__device__ __forceinline__ void fe_inv_sg(Fe<F> &r, const Fe<F> &a) {
  Fe<F> c = a;
  fe_canon(c);
  uint32_t w[F::NW];
  fe_pack(w, c);
  uint64_t x[F::N64], y[F::N64];
#pragma unroll
  for (int i = 0; i < F::N64; i++) x[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
#if ZK_INV_DS30
  int64_t P[F::S60_L];
#pragma unroll
  for (int i = 0; i < F::S60_L; i++) P[i] = F::s60p(i);
  sg_inverse_words<F::S60_L, F::S60_NB, 60>(y, x, F::N64, P, F::S62_PINV);
#else
  int64_t P[F::S62_L];
#pragma unroll
  for (int i = 0; i < F::S62_L; i++) P[i] = F::s62p(i);
  sg_inverse_words<F::S62_L, F::S62_NB>(y, x, F::N64, P, F::S62_PINV);
#endif
#pragma unroll
  for (int i = 0; i < F::N64; i++) {
    w[2 * i] = (uint32_t)y[i];
    w[2 * i + 1] = (uint32_t)(y[i] >> 32);
  }
  Fe<F> b, k;
  fe_unpack(b, w);
#pragma unroll
  for (int i = 0; i < F::N; i++) k.v[i] = F::k3(i);
  fe_mul(r, b, k);
}

// internal-form storage: SN u32 words (limbs, zero padded), 16-B aligned
template <class F>
__device__ __forceinline__ void fe_load_u(Fe<F> &r, const uint32_t *__restrict__ p) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  uint32_t w[F::SN];
#pragma unroll
  for (int i = 0; i < F::SN / 4; i++) {
    uint4 x = q[i];
    w[4 * i] = x.x; w[4 * i + 1] = x.y; w[4 * i + 2] = x.z; w[4 * i + 3] = x.w;
  }
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = w[i];
}
template <class F>
__device__ __forceinline__ void fe_store_u(uint32_t *__restrict__ p, const Fe<F> &a) {
  uint32_t w[F::SN];
#pragma unroll
  for (int i = 0; i < F::SN; i++) w[i] = i < F::N ? a.v[i] : 0u;
  uint4 *q = reinterpret_cast<uint4 *>(p);
#pragma unroll
  for (int i = 0; i < F::SN / 4; i++) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

}  // namespace zk
