// zk_g1ext.hip -- G1 batch affine conversion and the group (curve) FFT on gfx950.
//
// Replaces:
//   <C>_G1_proj_batch_from_affine / _batch_to_affine  bls12_381_G1_proj.c:147-167
//        (Haskell batchFromAffine / batchToAffine, G1/Proj.hs:409-430; msmProj, :222-223)
//   <C>_G1_proj_fft_forward / _fft_inverse            bls12_381_G1_proj.c:679-790
//        (Haskell forwardFFT / inverseFFT = curveFFT / curveIFFT, G1/Proj.hs:270-294)
// and their Jacobian twins (round 6), bound by the Jacobian G1 instance (G1/Jac.hs:188-196, 264-265,
// 374-389; msmJac = msm . batchToAffine, Jac.hs:220):
//   <C>_G1_jac_batch_from_affine / _batch_to_affine   bls12_381_G1_jac.c:139-158
//   <C>_G1_jac_fft_forward / _fft_inverse             bls12_381_G1_jac.c:727-838
// The Jacobian FFT is the projective one's text with jac_add / jac_scl (the same per-level scalars,
// the same group elements), so both run the same stages; only the load (x = X/Z^2, y = Y/Z^3) and the
// infinity conventions differ: affine infinity -> (1 : 1 : 0) (jac set_infinity, :183-187), Z = 0 ->
// all-0xFF (to_affine, :120-125), normalised output infinity (0 : 1 : 0) as the projective normalise
// (jac normalize, :62-67).  An input row with Z = 0 is infinity (the reference's is_infinity also
// wants Y^2 = X^3, X, Y != 0, :164-180; rows failing that are not curve points and the reference's
// add takes them as finite, so they are outside the contract).
//
// batch_to_affine: the reference inverts every Z separately (Fp_mont_inv per point,
// G1_proj.c:133-145); here CHK consecutive points per lane share ONE Fermat inversion
// (Montgomery's trick), points at infinity (Z = 0) are skipped in the product and come
// out as the all-0xFF affine sentinel, exactly like the reference.
//
// Group FFT: the reference recursion (radix-2 DIT forward; DIF with a factor 1/2 per
// level inverse) multiplies points by canonical Fr scalars at every level:
//   forward level s: t = w_s^j * v,  (u + t, u - t)
//   inverse level s: ((u + v) * 1/2,  (u - v) * (w_s^-j / 2))
// Scalar multiplication is by the INTEGER value of the canonical scalar, so for points
// outside the order-r subgroup (BLS12-381 G1 has a cofactor) the result depends on the
// exact per-level scalars, not only on their product mod r.  This implementation applies
// the same per-level scalars at the same positions (iterative DIT / DIF over HBM,
// ping-pong buffers), so its output is bit-identical for every on-curve input.
// Scalar multiplication (xyzz_scl): Jacobian accumulator, signed 5-bit windows MSB first, a
// 16-entry table per lane in global scratch (no lane divergence on the digit: every window does
// one table add).
// Outputs are normalised (Z = 1, infinity = (0:1:0)) as the reference does (:719, :785).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
#include "zk_curve.hpp"
#include "zk_host.hpp"
#include "zk_msm.hpp"
#include "zk_runtime.hpp"
#include "zk_g1ext.hpp"

namespace zk {

struct W6 {
  uint64_t w[6];
};

template <class F>
constexpr int xw() { return xyzz_words<F>(); }  // u32 words per stored XYZZ point

// x^e for an NW-word exponent (sliding window, zk_field.hpp fe_pow_sw; uniform across lanes)
template <class F, int NW>
__device__ __forceinline__ void fe_pow_words(Fe<F> &r, const Fe<F> &x, const W6 &e) {
  fe_pow_sw(r, x, e.w, NW);
}

template <class F>
__device__ __forceinline__ void ld_int(Fe<F> &r, const uint64_t *p) {  // reference form -> internal
  Fe<F> t;
  fe_load_ref(t, p);
  fe_to_int(r, t);
}
template <class F>
__device__ __forceinline__ void st_ref(uint64_t *p, const Fe<F> &a) {  // internal -> canonical reference form
  Fe<F> t;
  fe_to_ref(t, a);
  fe_store_ref(p, t);
}
template <class F>
__device__ __forceinline__ bool ref_all_ones(const uint64_t *p, int words) {
  uint64_t a = ~0ull;
  for (int i = 0; i < words; i++) a &= p[i];
  return a == ~0ull;
}

// ---------------------------------------------------------------------------- batch_from_affine

template <class C, bool JAC>
__global__ void __launch_bounds__(256) k_from_affine(int n, const uint64_t *__restrict__ src,
                                                     uint64_t *__restrict__ tgt, W6 one_ref) {
  constexpr int NP = C::NP64;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)n) return;
  const uint64_t *a = src + i * 2 * NP;
  uint64_t *o = tgt + i * 3 * NP;
  if (ref_all_ones<typename C::Fp>(a, 2 * NP)) {  // affine infinity -> (0 : 1 : 0), G1_proj.c:121-129;
    // Jacobian: (1 : 1 : 0), G1_jac.c:108-116, 183-187
    for (int k = 0; k < NP; k++) { o[k] = JAC ? one_ref.w[k] : 0; o[NP + k] = one_ref.w[k]; o[2 * NP + k] = 0; }
  } else {
    for (int k = 0; k < 2 * NP; k++) o[k] = a[k];
    for (int k = 0; k < NP; k++) o[2 * NP + k] = one_ref.w[k];
  }
}

// ---------------------------------------------------------------------------- chunked inversion
// MODE_PROJ_TO_AFF : src = reference projective (X:Y:Z), tgt = affine (X/Z, Y/Z) / 0xFF..
// MODE_XYZZ_TO_PROJ: src = device XYZZ, tgt = normalised reference projective, written at
//                    index bitrev_m(i) when m >= 0 (inverse FFT output order)
// MODE_JAC_TO_AFF  : src = reference Jacobian (X:Y:Z), tgt = affine (X/Z^2, Y/Z^3) / 0xFF..
enum { MODE_PROJ_TO_AFF = 0, MODE_XYZZ_TO_PROJ = 1, MODE_JAC_TO_AFF = 2 };

// Round 6: the chunk of lane t is the strided set {t, t + T, ...} (T = lanes, as k_inv_chunks):
// neighbouring lanes touch neighbouring point rows.  STRIDED = false: CHK consecutive points.
// canonical reference-form words of a (internal form), or `alt` where !keep, stored as 16-B runs
template <class F>
__device__ __forceinline__ void st_ref_or(uint64_t *p, const Fe<F> &a, bool keep, const uint32_t (&alt)[F::NW]) {
  Fe<F> t;
  fe_to_ref(t, a);
  fe_canon(t);
  uint32_t w[F::NW];
  fe_pack(w, t);
#pragma unroll
  for (int i = 0; i < F::NW; i++) w[i] = keep ? w[i] : alt[i];
  uint4 *q = reinterpret_cast<uint4 *>(p);
#pragma unroll
  for (int i = 0; i < F::NW / 4; i++) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}
// BF (round 6, default; ZK_NORM_BF=0 restores the branches): every step branch-free -- the points at
// infinity take the factor 1 and have their output rows selected word by word, and every load and
// store is unconditional, so no path merge inside the loop makes the compiler wait for all
// outstanding memory (the Fr inversion measured the same effect, profiles/r06v_inv_ilp_ab.txt).
template <class C, int MODE, bool SG = true, bool STRIDED = true, bool BF = true>
__global__ void __launch_bounds__(256) k_norm_chunks(int n, int CHK, const void *__restrict__ srcv,
                                                     uint64_t *__restrict__ scratch, uint64_t *__restrict__ tgt,
                                                     W6 pm2, int bitrev_m, int lanes) {
  using F = typename C::Fp;
  constexpr int NP = C::NP64;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t T = STRIDED ? (size_t)lanes : 1;
  const size_t i0 = STRIDED ? t : t * CHK;
  if ((STRIDED && t >= T) || i0 >= (size_t)n) return;
  const size_t left = ((size_t)n - i0 + T - 1) / T;
  const size_t cnt = left < (size_t)CHK ? left : (size_t)CHK;
  const uint64_t *srcp = reinterpret_cast<const uint64_t *>(srcv);
  const uint32_t *srcx = reinterpret_cast<const uint32_t *>(srcv);
  auto den = [&](size_t i, Fe<F> &d) -> bool {  // denominator (internal); false = infinity
    if (MODE != MODE_XYZZ_TO_PROJ) {
      ld_int(d, srcp + i * 3 * NP + 2 * NP);
    } else {
      fe_load_u(d, srcx + i * xw<F>() + 3 * F::SN);  // ZZZ
    }
    return !fe_is_zero(d);
  };
  Fe<F> P, one_int;
  fe_one(P);
  fe_one(one_int);
  for (size_t k = 0; k < cnt; k++) {
    const size_t i = i0 + k * T;
    Fe<F> d, q;
    if constexpr (BF) {
      const bool fin = den(i, d);
      Fe<F> f;
#pragma unroll
      for (int l = 0; l < F::N; l++) f.v[l] = fin ? d.v[l] : one_int.v[l];
      fe_mul(q, P, f);
      P = q;
    } else if (den(i, d)) {
      fe_mul(q, P, d);
      P = q;
    }
    fe_store_ref(scratch + i * NP, P);  // running product (internal form, packed)
  }
  Fe<F> inv;
  if (SG) fe_inv_sg(inv, P);  // divsteps (zk_inv.hpp); Fermat with ZK_INV_SG=0
  else fe_pow_words<F, NP>(inv, P, pm2);
  if constexpr (BF) {
    uint32_t ones[F::NW], zeros[F::NW], oneref[F::NW];
    {
      Fe<F> t;
      fe_to_ref(t, one_int);
      fe_canon(t);
      fe_pack(oneref, t);
    }
#pragma unroll
    for (int l = 0; l < F::NW; l++) { ones[l] = ~0u; zeros[l] = 0; }
    for (size_t kk = cnt; kk-- > 0;) {
      const size_t i = i0 + kk * T;
      Fe<F> d, e, prev, f, dinv, q;
      const bool fin = den(i, d);
      size_t o = i;
      if (MODE == MODE_XYZZ_TO_PROJ && bitrev_m > 0)
        o = (size_t)(__builtin_bitreverse32((uint32_t)i) >> (32 - bitrev_m));
      fe_load_ref(e, scratch + (kk > 0 ? i - T : i) * NP);
#pragma unroll
      for (int l = 0; l < F::N; l++) {
        prev.v[l] = kk > 0 ? e.v[l] : one_int.v[l];
        f.v[l] = fin ? d.v[l] : one_int.v[l];
      }
      fe_mul(dinv, inv, prev);  // 1 / d_i
      fe_mul(q, inv, f);
      inv = q;
      if (MODE == MODE_PROJ_TO_AFF || MODE == MODE_JAC_TO_AFF) {
        Fe<F> X, Y, x, y;
        ld_int(X, srcp + i * 3 * NP);
        ld_int(Y, srcp + i * 3 * NP + NP);
        if (MODE == MODE_PROJ_TO_AFF) {
          fe_mul(x, X, dinv);
          fe_mul(y, Y, dinv);
        } else {
          Fe<F> d2, d3;
          fe_sqr(d2, dinv);
          fe_mul(d3, d2, dinv);
          fe_mul(x, X, d2);
          fe_mul(y, Y, d3);
        }
        st_ref_or(tgt + o * 2 * NP, x, fin, ones);  // infinity: all-ones row, G1_proj.c:134-138
        st_ref_or(tgt + o * 2 * NP + NP, y, fin, ones);
      } else {
        Xyzz<F> p;
        xyzz_load(p, srcx + i * xw<F>());
        Fe<F> iz, iz2, x, y;
        fe_mul(iz, p.ZZ, dinv);  // ZZ / ZZZ = 1/Z
        fe_sqr(iz2, iz);         // 1/ZZ
        fe_mul(x, p.X, iz2);
        fe_mul(y, p.Y, dinv);
        uint64_t *qo = tgt + o * 3 * NP;
        st_ref_or(qo, x, fin, zeros);  // infinity: (0 : 1 : 0)
        st_ref_or(qo + NP, y, fin, oneref);
        st_ref_or(qo + 2 * NP, one_int, fin, zeros);
      }
    }
    return;
  }
  for (size_t kk = cnt; kk-- > 0;) {
    const size_t i = i0 + kk * T;
    Fe<F> d;
    const bool fin = den(i, d);
    size_t o = i;
    if (MODE == MODE_XYZZ_TO_PROJ && bitrev_m > 0)
      o = (size_t)(__builtin_bitreverse32((uint32_t)i) >> (32 - bitrev_m));
    if (!fin) {
      if (MODE != MODE_XYZZ_TO_PROJ) {
        for (int k = 0; k < 2 * NP; k++) tgt[o * 2 * NP + k] = ~0ull;  // G1_proj.c:134-138
      } else {
        uint64_t *q = tgt + o * 3 * NP;
        for (int k = 0; k < NP; k++) q[k] = 0;
        st_ref(q + NP, one_int);
        for (int k = 0; k < NP; k++) q[2 * NP + k] = 0;
      }
      continue;
    }
    Fe<F> prev, dinv, q;
    if (kk > 0) fe_load_ref(prev, scratch + (i - T) * NP); else prev = one_int;
    fe_mul(dinv, inv, prev);  // 1 / d_i
    fe_mul(q, inv, d);
    inv = q;
    if (MODE == MODE_PROJ_TO_AFF) {
      Fe<F> X, Y, x, y;
      ld_int(X, srcp + i * 3 * NP);
      ld_int(Y, srcp + i * 3 * NP + NP);
      fe_mul(x, X, dinv);
      fe_mul(y, Y, dinv);
      st_ref(tgt + o * 2 * NP, x);
      st_ref(tgt + o * 2 * NP + NP, y);
    } else if (MODE == MODE_JAC_TO_AFF) {
      Fe<F> X, Y, x, y, d2, d3;
      ld_int(X, srcp + i * 3 * NP);
      ld_int(Y, srcp + i * 3 * NP + NP);
      fe_sqr(d2, dinv);
      fe_mul(d3, d2, dinv);
      fe_mul(x, X, d2);
      fe_mul(y, Y, d3);
      st_ref(tgt + o * 2 * NP, x);
      st_ref(tgt + o * 2 * NP + NP, y);
    } else {
      Xyzz<F> p;
      xyzz_load(p, srcx + i * xw<F>());
      Fe<F> iz, iz2, x, y;
      fe_mul(iz, p.ZZ, dinv);  // ZZ / ZZZ = 1/Z
      fe_sqr(iz2, iz);         // 1/ZZ
      fe_mul(x, p.X, iz2);
      fe_mul(y, p.Y, dinv);
      uint64_t *qo = tgt + o * 3 * NP;
      st_ref(qo, x);
      st_ref(qo + NP, y);
      st_ref(qo + 2 * NP, one_int);
    }
  }
}

// ---------------------------------------------------------------------------- group FFT

// reference projective -> device XYZZ (x = X/Z -> X' = X Z, ZZ = Z^2; y = Y/Z -> Y' = Y Z^2,
// ZZZ = Z^3), stored at bitrev_m(i) when m > 0 (forward FFT input order); Jacobian (x = X/Z^2,
// y = Y/Z^3) -> X' = X, Y' = Y, ZZ = Z^2, ZZZ = Z^3
template <class C, bool JAC>
__global__ void __launch_bounds__(256) k_fft_load(int n, int bitrev_m, const uint64_t *__restrict__ src,
                                                  uint32_t *__restrict__ dst) {
  using F = typename C::Fp;
  constexpr int NP = C::NP64;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)n) return;
  Fe<F> X, Y, Z;
  ld_int(X, src + i * 3 * NP);
  ld_int(Y, src + i * 3 * NP + NP);
  ld_int(Z, src + i * 3 * NP + 2 * NP);
  Xyzz<F> p;
  if (fe_is_zero(Z)) {
    xyzz_set_inf(p);
  } else {
    fe_sqr(p.ZZ, Z);
    fe_mul(p.ZZZ, p.ZZ, Z);
    if (JAC) {
      p.X = X;
      p.Y = Y;
    } else {
      fe_mul(p.X, X, Z);
      fe_mul(p.Y, Y, p.ZZ);
    }
  }
  const size_t o = bitrev_m > 0 ? (size_t)(__builtin_bitreverse32((uint32_t)i) >> (32 - bitrev_m)) : i;
  xyzz_store(dst + o * xw<F>(), p);
}

template <class F>
__device__ __forceinline__ void xyzz_neg(Xyzz<F> &r, const Xyzz<F> &a) {
  r = a;
  fe_neg(r.Y, a.Y);
}

// Scalar multiplication r = k P for the group FFT (k a 256-bit integer, 4 u64), computed with
// the accumulator in JACOBIAN coordinates: the chain is 255 doublings, and a Jacobian doubling
// (dbl-2009-l, a = 0) is 7 products against XYZZ's 9; additions take the table entry with its
// Z^2, Z^3 cached (add-1998-cmo-2: 14 products, as XYZZ's).  Digits: signed 5-bit windows
// (K = k + sum_i 16 * 32^i, digit i = bits [5i, 5i + 5) of K minus 16, in [-16, 15]; K < 2^260
// as k < 2^256 - 2^255), so at most 52 additions instead of 64 with a 16-point table.
// 255 x 7 + 52 x 14 + table 241 = ~2750 products per multiplication (was ~3350).
template <class F>
struct Jac {
  Fe<F> X, Y, Z;  // x = X / Z^2, y = Y / Z^3; Z = 0: infinity
};
// Round 5 form (ZK_FFT_DBL2, default): D = 4 X B as one product instead of 2((X + B)^2 - A - C),
// and Y3 = E (D - X3) + (-8B) B as ONE shared-reduction pair (fe_mul2k: Karatsuba columns of both
// products, one Montgomery reduction), so C = B^2 is never reduced on its own: 4 products + 1
// pair, 6 reductions instead of 7, and three exact additions fewer.  Bounds: every operand < 2p,
// E (D - X3) + (-8B) B < 8 p^2 < p R' (R' / p = 2^11), so the pair's output is < 2p like fe_mul's.
#ifndef ZK_FFT_DBL2
#define ZK_FFT_DBL2 1
#endif
// the point routines' products: Karatsuba columns (fe_mulk, 436 vs 472 issue slots per 381-bit
// product) with ZK_FFT_DBL2, the schoolbook fe_mul of round 4 otherwise (A/B)
template <class F>
__device__ __forceinline__ void fft_mul(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
#if ZK_FFT_DBL2
  fe_mulk(r, a, b);
#else
  fe_mul(r, a, b);
#endif
}
// Lazy form (ZK_FFT_LAZY, default, both base fields): the doubling and the cached addition take no
// exact addition / subtraction (each two carry chains, ~56 issue slots) except the two whose
// results are tested for zero (the addition's H and r): multiples are folded into products (4X B,
// (2Y) Z), differences are a + K p - b (fe_sub_lazy) re-normalised where a product takes them.
// Invariant of a Jacobian accumulator / table entry: X < 10p, Y, Z < 2p, normalised limbs (every
// consumer of X multiplies it: the XYZZ it is converted to keeps X < 10p, which xyzz_add and the
// normalisation only multiply).  tools/lazy_bounds.py (jac_dbl_lazy, jac_add_cached_lazy) replays
// both routines on that invariant for each field: outputs X < 9p, every column < 2^64, and Y, Z < 1.02p
// on BLS12-381 (R'/p ~ 2520) but Y < 1.41p, Z < 1.05p on BN254 (R'/p ~ 169: the Y3 pair's larger
// quotient) -- still inside the < 2p invariant; `python tools/lazy_bounds.py` prints these per field.
#ifndef ZK_FFT_LAZY
#define ZK_FFT_LAZY 1
#endif
template <class F>
__device__ __forceinline__ void jac_dbl(Jac<F> &p) {  // in place; infinity stays infinity
#if ZK_FFT_LAZY
  if constexpr (F::N == 14 || (F::N == 9 && F::RB == 29)) {
    Fe<F> A, B, D, E, F2, X3, t, x4, y2, nb, nb8;
    fe_sqr(A, p.X);                        // X < 10p
    fe_sqr(B, p.Y);
    fe_add_lazy(x4, p.X, p.X);
    fe_add_lazy(x4, x4, x4);               // 4X < 40p, limbs < 2^30
    fe_mulk(D, x4, B);                     // D = 4 X B
    fe_add_lazy(E, A, A);
    fe_add_lazy(E, E, A);                  // E = 3A < 6p
    if constexpr (F::N == 9) fe_norm(E);  // 29-bit limbs: the doubled limbs of the square
    fe_sqr(F2, E);                         // F = E^2
    fe_add_lazy(t, D, D);                  // 2D < 4p
    fe_sub_lazy<F, 8, 2>(X3, F2, t);       // X3 = F - 2D < 9p
    fe_norm(X3);
    fe_add_lazy(y2, p.Y, p.Y);
    fe_mulk(p.Z, y2, p.Z);                 // Z3 = (2Y) Z
    fe_sub_lazy<F, 10, 1>(t, D, X3);       // D - X3 < 12p
    fe_norm(t);
    fe_sub_lazy<F, 2, 1>(nb, Fe<F>{}, B);  // 2p - B
    fe_norm(nb);
    fe_add_lazy(nb8, nb, nb);
    fe_add_lazy(nb8, nb8, nb8);
    fe_add_lazy(nb8, nb8, nb8);            // 8 (2p - B) < 16p
    if constexpr (F::N == 9) fe_norm(nb8);  // 29-bit limbs: 8x would reach 2^32
    fe_mul2k(p.Y, E, t, nb8, B);           // Y3 = E (D - X3) - 8 B^2
    p.X = X3;
    return;
  }
#endif
#if ZK_FFT_DBL2
  Fe<F> A, B, D, E, F2, X3, t, u;
  fe_sqr(A, p.X);
  fe_sqr(B, p.Y);
  fe_mulk(t, p.X, B);
  fe_add(t, t, t);
  fe_add(D, t, t);          // D = 4 X B  (= 2((X + B)^2 - A - C))
  fe_mul3(E, A);            // E = 3A
  fe_sqr(F2, E);            // F = E^2
  fe_sub(t, F2, D);
  fe_sub(X3, t, D);         // X3 = F - 2D
  fe_mulk(u, p.Y, p.Z);
  fe_add(p.Z, u, u);        // Z3 = 2 Y Z
  fe_sub(t, D, X3);
  Fe<F> b8, nb8;
  fe_add(b8, B, B);
  fe_add(b8, b8, b8);
  fe_add(b8, b8, b8);       // 8B
  fe_neg(nb8, b8);
  fe_mul2k(p.Y, E, t, nb8, B);  // Y3 = E (D - X3) - 8 B^2
  p.X = X3;
#else
  Fe<F> A, B, C, D, E, t, u;
  fe_sqr(A, p.X);
  fe_sqr(B, p.Y);
  fe_sqr(C, B);
  fe_add(t, p.X, B);
  fe_sqr(u, t);
  fe_sub(u, u, A);
  fe_sub(u, u, C);
  fe_add(D, u, u);          // D = 2((X + B)^2 - A - C)
  fe_mul3(E, A);            // E = 3A
  fe_sqr(t, E);             // F = E^2
  fe_sub(t, t, D);
  Fe<F> X3;
  fe_sub(X3, t, D);         // X3 = F - 2D
  fe_mul(u, p.Y, p.Z);
  fe_add(p.Z, u, u);        // Z3 = 2 Y Z
  fe_sub(t, D, X3);
  fe_mul(u, E, t);          // E (D - X3)
  fe_add(C, C, C);
  fe_add(C, C, C);
  fe_add(C, C, C);          // 8C
  fe_sub(p.Y, u, C);
  p.X = X3;
#endif
}
// table entry: the point and its Z^2, Z^3
template <class F>
struct JacC {
  Fe<F> X, Y, Z, ZZ, ZZZ;
};
template <class F>
__device__ __forceinline__ void jac_cache(JacC<F> &c, const Jac<F> &p) {
  c.X = p.X;
  c.Y = p.Y;
  c.Z = p.Z;
  fe_sqr(c.ZZ, p.Z);
  fe_mul(c.ZZZ, c.ZZ, p.Z);
}
template <class F>
__device__ __forceinline__ bool jac_is_inf(const Jac<F> &p) { return fe_is_zero(p.Z); }
// acc += b (b cached, b not infinity); all special cases handled
template <class F>
__device__ __forceinline__ void jac_add_cached(Jac<F> &acc, const JacC<F> &b) {
  if (jac_is_inf(acc)) {
    acc.X = b.X;
    acc.Y = b.Y;
    acc.Z = b.Z;
    return;
  }
  Fe<F> Z1Z1, U1, U2, S1, S2, H, r, t;
  fe_sqr(Z1Z1, acc.Z);
  fft_mul(U1, acc.X, b.ZZ);
  fft_mul(U2, b.X, Z1Z1);
  fft_mul(S1, acc.Y, b.ZZZ);
  fft_mul(t, acc.Z, Z1Z1);
  fft_mul(S2, b.Y, t);
  fe_sub(H, U2, U1);
  fe_sub(r, S2, S1);
  if (fe_is_zero(H)) {
    if (fe_is_zero(r)) jac_dbl(acc);  // acc == b
    else fe_zero(acc.Z);              // acc == -b
    return;
  }
  Fe<F> HH, HHH, V, X3;
  fe_sqr(HH, H);
  fft_mul(HHH, H, HH);
  fft_mul(V, U1, HH);
#if ZK_FFT_LAZY
  if constexpr (F::N == 14 || (F::N == 9 && F::RB == 29)) {
    Fe<F> RR, v2, nS1;
    fe_sqr(RR, r);
    fe_sub_lazy<F, 2, 1>(t, RR, HHH);      // RR - HHH < 4p
    fe_add_lazy(v2, V, V);
    fe_sub_lazy<F, 6, 2>(X3, t, v2);       // X3 = r^2 - HHH - 2V < 9p
    fe_norm(X3);
    fe_sub_lazy<F, 12, 1>(t, V, X3);       // V - X3 < 14p
    fe_norm(t);
    fe_sub_lazy<F, 2, 1>(nS1, Fe<F>{}, S1);
    fe_norm(nS1);
    fe_mul2k(acc.Y, r, t, nS1, HHH);       // Y3 = r (V - X3) - S1 HHH
    fft_mul(t, acc.Z, b.Z);
    fft_mul(acc.Z, t, H);                  // Z3 = Z1 Z2 H
    acc.X = X3;
    return;
  }
#endif
  fe_sqr(t, r);
  fe_sub(t, t, HHH);
  fe_sub(t, t, V);
  fe_sub(X3, t, V);         // X3 = r^2 - HHH - 2V
  fe_sub(t, V, X3);
#if ZK_FFT_DBL2
  Fe<F> nS1;
  fe_neg(nS1, S1);
  fe_mul2k(acc.Y, r, t, nS1, HHH);  // Y3 = r (V - X3) - S1 HHH, one shared reduction (< 8 p^2 < p R')
#else
  fe_mul(V, r, t);          // r (V - X3)
  fe_mul(t, S1, HHH);
  fe_sub(acc.Y, V, t);
#endif
  fft_mul(t, acc.Z, b.Z);
  fft_mul(acc.Z, t, H);     // Z3 = Z1 Z2 H
  acc.X = X3;
}
template <class F>
__device__ __forceinline__ void jacc_store(uint32_t *p, const JacC<F> &c) {
  fe_store_u(p + 0 * F::SN, c.X);
  fe_store_u(p + 1 * F::SN, c.Y);
  fe_store_u(p + 2 * F::SN, c.Z);
  fe_store_u(p + 3 * F::SN, c.ZZ);
  fe_store_u(p + 4 * F::SN, c.ZZZ);
}
template <class F>
__device__ __forceinline__ void jacc_load(JacC<F> &c, const uint32_t *p) {
  fe_load_u(c.X, p + 0 * F::SN);
  fe_load_u(c.Y, p + 1 * F::SN);
  fe_load_u(c.Z, p + 2 * F::SN);
  fe_load_u(c.ZZ, p + 3 * F::SN);
  fe_load_u(c.ZZZ, p + 4 * F::SN);
}
constexpr int SCL_TAB = 16;                                  // table entries d P, d = 1..16
template <class F>
constexpr int scl_tab_words() { return SCL_TAB * 5 * F::SN; }  // u32 words of one lane's table
// window i (5 bits) of the 261-bit K held in 5 u64 words
__device__ __forceinline__ uint32_t win5(const uint64_t *K, int i) {
  const int b = 5 * i, w = b >> 6, o = b & 63;
  uint64_t v = K[w] >> o;
  if (o > 59 && w < 4) v |= K[w + 1] << (64 - o);
  return (uint32_t)v & 31u;
}
// Every point routine of the group FFT is inlined into its kernel.  Round 4's first Jacobian
// build left xyzz_scl outlined (a real call: s_swappc_b64 into it, s_setpc_b64 s[30:31] back), and
// LLVM's branch relaxation of a long branch inside the callee took s[30:31] -- the return address
// -- as its scratch pair without saving it, so the return jumped into the callee's own body and
// the kernel never finished (profiles/r05*_fft_outlined_scl.txt holds the disassembly of that
// variant, built with -DZK_FFT_SCL_ATTR=__noinline__).  tests/test_isa_guard.py checks the
// shipped code object: no group-FFT kernel may contain a call.
#ifndef ZK_FFT_SCL_ATTR
#define ZK_FFT_SCL_ATTR __forceinline__
#endif
template <class F>
__device__ ZK_FFT_SCL_ATTR void xyzz_scl(Xyzz<F> &r, const Xyzz<F> &P, const uint64_t *k, uint32_t *__restrict__ tab) {
  if (xyzz_is_inf(P)) {
    r = P;
    return;
  }
  {  // P in Jacobian form: Z' = ZZ ZZZ, X' = X ZZ ZZZ^2, Y' = Y ZZZ^4 (valid XYZZ has ZZ^3 = ZZZ^2)
    Jac<F> p, acc;
    Fe<F> z2, z4, t;
    fe_sqr(z2, P.ZZZ);
    fe_mul(t, P.X, P.ZZ);
    fe_mul(p.X, t, z2);
    fe_sqr(z4, z2);
    fe_mul(p.Y, P.Y, z4);
    fe_mul(p.Z, P.ZZ, P.ZZZ);
    JacC<F> pc, c;
    jac_cache(pc, p);
    jacc_store(tab, pc);
    acc = p;
    jac_dbl(acc);
    jac_cache(c, acc);
    jacc_store(tab + 1 * 5 * F::SN, c);
    for (int d = 3; d <= SCL_TAB; d++) {
      jac_add_cached(acc, pc);
      jac_cache(c, acc);
      jacc_store(tab + (size_t)(d - 1) * 5 * F::SN, c);
    }
  }
  uint64_t K[5];
  {
    const uint64_t H[5] = {0x0842108421084210ull, 0x1084210842108421ull, 0x2108421084210842ull,
                           0x4210842108421084ull, 0x8ull};
    uint64_t cy = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) {
      const uint64_t a = j < 4 ? k[j] : 0, s1 = a + H[j];
      const uint64_t c1 = s1 < a ? 1 : 0, s2 = s1 + cy;
      K[j] = s2;
      cy = c1 | (s2 < s1 ? 1 : 0);
    }
  }
  Jac<F> acc;
  fe_one(acc.X);
  fe_one(acc.Y);
  fe_zero(acc.Z);
  for (int i = 51; i >= 0; i--) {
    if (i != 51)
      for (int z = 0; z < 5; z++) jac_dbl(acc);
    const int d = (int)win5(K, i) - 16;
    if (d) {
      JacC<F> e;
      jacc_load(e, tab + (size_t)((d < 0 ? -d : d) - 1) * 5 * F::SN);
      if (d < 0) {
        Fe<F> ny;
        fe_neg(ny, e.Y);
        e.Y = ny;
      }
      jac_add_cached(acc, e);
    }
  }
  if (jac_is_inf(acc)) {
    xyzz_set_inf(r);
    return;
  }
  r.X = acc.X;
  r.Y = acc.Y;
  fe_sqr(r.ZZ, acc.Z);
  fe_mul(r.ZZZ, r.ZZ, acc.Z);
}

// ---------------------------------------------------------------------------- GLV stages
// On the order-r subgroup phi(x, y) = (beta x, y) is [lambda], so k P = k1 P + k2 phi(P) with
// |k1|, |k2| < 2^130 (k = k1 + k2 lambda mod r; constants: zk_glv.inc, tools/gen_glv.py).  A
// butterfly's multiplication then runs on a PAIR of lanes -- lane 0: k1 P, lane 1: k2 phi(P), 27
// signed 5-bit windows (130 doublings) each -- and the pair swaps results (DPP) and adds them.
// The chain per lane is ~half of the 255-doubling one, and the stage has twice the lanes (2^16
// points: 2^16 lanes instead of 2^15, so every SIMD holds a wavefront).  Valid only on the
// subgroup (for other points k P depends on the integer k, not on k mod r, and the reference
// multiplies by the integer): BN254 G1 has cofactor 1; BLS12-381 inputs are checked first
// (k_subgroup_check) and the call falls back to the integer stages when any point fails.
#include "zk_glv.inc"
// Waves per SIMD the GLV stage and membership kernels are compiled for (2 caps them at 256 VGPRs
// so two wavefronts share a SIMD).  BN254 fits 256 with a few spilled registers and gains 8% at
// 2^18 (57.2 -> 52.7 ms forward, profiles/r05s_fft_two_waves.txt); BLS12-381's kernels hold 445-503
// VGPRs and spilled 290-420 of them when capped (2^16 forward 25.7 -> 27.6 ms), so they stay at one.
#ifndef ZK_FFT_WAVES_BN
#define ZK_FFT_WAVES_BN 2
#endif
#ifndef ZK_FFT_WAVES_BLS
#define ZK_FFT_WAVES_BLS 1
#endif
template <class C>
constexpr int fft_waves() { return C::NP64 == 4 ? ZK_FFT_WAVES_BN : ZK_FFT_WAVES_BLS; }

struct GlvParams {  // decomposition constants of one curve (kernel argument)
  uint64_t g1[4], g2[4], a1[3], b1[3], a2[3], b2[3];
  int s1, s2;
};
template <class C>
static GlvParams glv_params() {
  GlvParams p;
  auto cp = [](uint64_t *d, const uint64_t *s, int n) { for (int i = 0; i < n; i++) d[i] = s[i]; };
  if constexpr (C::NP64 == 4) {
    cp(p.g1, GLV_BN254_G1, 4); cp(p.g2, GLV_BN254_G2, 4);
    cp(p.a1, GLV_BN254_A1, 3); cp(p.b1, GLV_BN254_B1, 3); cp(p.a2, GLV_BN254_A2, 3); cp(p.b2, GLV_BN254_B2, 3);
    p.s1 = GLV_BN254_SGN1; p.s2 = GLV_BN254_SGN2;
  } else {
    cp(p.g1, GLV_BLS381_G1, 4); cp(p.g2, GLV_BLS381_G2, 4);
    cp(p.a1, GLV_BLS381_A1, 3); cp(p.b1, GLV_BLS381_B1, 3); cp(p.a2, GLV_BLS381_A2, 3); cp(p.b2, GLV_BLS381_B2, 3);
    p.s1 = GLV_BLS381_SGN1; p.s2 = GLV_BLS381_SGN2;
  }
  return p;
}
template <class C>
static W6 glv_beta_ref() {
  W6 b = {{0, 0, 0, 0, 0, 0}};
  const uint64_t *s = C::NP64 == 4 ? GLV_BN254_BETA_REF : GLV_BLS381_BETA_REF;
  for (int i = 0; i < C::NP64; i++) b.w[i] = s[i];
  return b;
}

// 192-bit two's complement helpers (values of the decomposition are < 2^131 in magnitude)
__device__ __forceinline__ void u192_mul(uint64_t r[3], const uint64_t a[3], const uint64_t b[3]) {
  const uint64_t lo00 = a[0] * b[0], hi00 = __umul64hi(a[0], b[0]);
  const uint64_t lo01 = a[0] * b[1], hi01 = __umul64hi(a[0], b[1]);
  const uint64_t lo10 = a[1] * b[0], hi10 = __umul64hi(a[1], b[0]);
  r[0] = lo00;
  const uint64_t s1 = hi00 + lo01, c1 = s1 < hi00 ? 1 : 0;
  const uint64_t s2 = s1 + lo10, c2 = s2 < s1 ? 1 : 0;
  r[1] = s2;
  r[2] = hi01 + hi10 + c1 + c2 + a[0] * b[2] + a[1] * b[1] + a[2] * b[0];
}
__device__ __forceinline__ void u192_sub(uint64_t r[3], const uint64_t a[3], const uint64_t b[3]) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const uint64_t d = a[i] - b[i], b1 = a[i] < b[i] ? 1 : 0, d2 = d - br, b2 = d < br ? 1 : 0;
    r[i] = d2;
    br = b1 | b2;
  }
}
__device__ __forceinline__ void u192_neg(uint64_t r[3], const uint64_t a[3]) {
  const uint64_t z[3] = {0, 0, 0};
  u192_sub(r, z, a);
}
// c = floor(k g / 2^382) (k, g < 2^256; c < 2^130)
__device__ __forceinline__ void glv_round(uint64_t c[3], const uint64_t k[4], const uint64_t g[4]) {
  uint64_t p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint64_t lo = k[i] * g[j], hi = __umul64hi(k[i], g[j]);
      const uint64_t s = p[i + j] + lo, c1 = s < lo ? 1 : 0;
      const uint64_t s2 = s + carry, c2 = s2 < s ? 1 : 0;
      p[i + j] = s2;
      carry = hi + c1 + c2;
    }
    p[i + 4] = carry;
  }
  c[0] = (p[5] >> 62) | (p[6] << 2);
  c[1] = (p[6] >> 62) | (p[7] << 2);
  c[2] = p[7] >> 62;
}
// k (standard form, < r) -> |k1|, |k2| (3 words each) and their signs (bit 0: k1 < 0, bit 1: k2 < 0)
__device__ __forceinline__ void glv_decompose(uint64_t out[8], const uint64_t k[4], const GlvParams &P) {
  uint64_t c1[3], c2[3], t[3], k1[3], k2[3];
  glv_round(c1, k, P.g1);
  glv_round(c2, k, P.g2);
  if (P.s1 < 0) u192_neg(c1, c1);
  if (P.s2 < 0) u192_neg(c2, c2);
  const uint64_t kk[3] = {k[0], k[1], k[2]};
  u192_mul(t, c1, P.a1);
  u192_sub(k1, kk, t);
  u192_mul(t, c2, P.a2);
  u192_sub(k1, k1, t);  // k1 = k - c1 a1 - c2 a2
  u192_mul(t, c1, P.b1);
  u192_neg(k2, t);
  u192_mul(t, c2, P.b2);
  u192_sub(k2, k2, t);  // k2 = -c1 b1 - c2 b2
  uint32_t sg = 0;
  if (k1[2] >> 63) { u192_neg(k1, k1); sg |= 1; }
  if (k2[2] >> 63) { u192_neg(k2, k2); sg |= 2; }
  out[0] = k1[0]; out[1] = k1[1]; out[2] = k1[2];
  out[3] = k2[0]; out[4] = k2[1]; out[5] = k2[2];
  out[6] = sg;
  out[7] = 0;
}

// twg[e] = GLV decomposition of std(scale * base^e) (8 u64 per entry), e < cnt
template <class Fr>
__global__ void __launch_bounds__(256) k_fft_tw_glv(int cnt, W6 base, W6 scale, GlvParams gp,
                                                    uint64_t *__restrict__ twg) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cnt) return;
  Fe<Fr> b, acc, t;
  ld_int(b, base.w);
  fe_load_ref(acc, scale.w);
  Fe<Fr> p = b;
  for (int x = e; x; x >>= 1) {
    if (x & 1) { fe_mul(t, acc, p); acc = t; }
    fe_sqr(t, p);
    p = t;
  }
  Fe<Fr> sd;
  fe_ref_to_std(sd, acc);
  uint64_t k[4], o[8];
  fe_store_ref(k, sd);
  glv_decompose(o, k, gp);
#pragma unroll
  for (int i = 0; i < 8; i++) twg[(size_t)e * 8 + i] = o[i];
}

// point-pair swap inside a lane pair (DPP quad_perm [1, 0, 3, 2])
template <class F>
__device__ __forceinline__ void fe_pair_swap(Fe<F> &r, const Fe<F> &v) {
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.v[i], 0xB1, 0xf, 0xf, false);
}
template <class F>
__device__ __forceinline__ void xyzz_to_jac(Jac<F> &p, const Xyzz<F> &P) {  // P not infinity
  Fe<F> z2, z4, t;
  fe_sqr(z2, P.ZZZ);
  fe_mul(t, P.X, P.ZZ);
  fe_mul(p.X, t, z2);
  fe_sqr(z4, z2);
  fe_mul(p.Y, P.Y, z4);
  fe_mul(p.Z, P.ZZ, P.ZZZ);
}
template <class F>
__device__ __forceinline__ void jac_to_xyzz(Xyzz<F> &r, const Jac<F> &a) {
  if (jac_is_inf(a)) {
    xyzz_set_inf(r);
    return;
  }
  r.X = a.X;
  r.Y = a.Y;
  fe_sqr(r.ZZ, a.Z);
  fe_mul(r.ZZZ, r.ZZ, a.Z);
}
// acc += b, either may be infinity
template <class F>
__device__ __forceinline__ void jac_add_any(Jac<F> &acc, const Jac<F> &b) {
  if (jac_is_inf(b)) return;
  if (jac_is_inf(acc)) {
    acc = b;
    return;
  }
  JacC<F> c;
  jac_cache(c, b);
  jac_add_cached(acc, c);
}
// window i (5 bits) of a 3-word K
__device__ __forceinline__ uint32_t win5_3(const uint64_t *K, int i) {
  const int b = 5 * i, w = b >> 6, o = b & 63;
  uint64_t v = K[w] >> o;
  if (o > 59 && w < 2) v |= K[w + 1] << (64 - o);
  return (uint32_t)v & 31u;
}
// The pair's shared table: d P for d = 1..16 built by both lanes (lane 0 the odd d, lane 1 the
// even d, stepping by 2P: one doubling and 7 additions each instead of 15 additions per lane),
// stored at the pair's slot; lane 1 uses phi(d P) = (beta X, Y, Z) at lookup (one product per
// window).  The halves are read back by the other lane of the wavefront: the stores are
// released and the CU's L1 invalidated (agent-scope fences) before the lookups.
// r = k (phi^q P) for k < 2^130, signs applied at lookup (neg: the half's scalar is negative)
template <class F>
__device__ __forceinline__ void jac_scl130_pair(Jac<F> &acc, const Jac<F> &p, const uint64_t *k, bool neg,
                                                const Fe<F> &mulx, uint32_t *__restrict__ tab) {
  const int q = (int)(threadIdx.x & 1);
  {
    Jac<F> two = p, a;
    jac_dbl(two);
    JacC<F> c2, c;
    jac_cache(c2, two);
    a = q ? two : p;
    for (int i = 0; i < SCL_TAB / 2; i++) {
      if (i) jac_add_cached(a, c2);
      jac_cache(c, a);
      jacc_store(tab + (size_t)(q + 2 * i) * 5 * F::SN, c);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  uint64_t K[3];
  {
    const uint64_t H[3] = {0x0842108421084210ull, 0x1084210842108421ull, 0x0000000000000042ull};
    uint64_t cy = 0;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const uint64_t a = k[j], s1 = a + H[j];
      const uint64_t c1 = s1 < a ? 1 : 0, s2 = s1 + cy;
      K[j] = s2;
      cy = c1 | (s2 < s1 ? 1 : 0);
    }
  }
  fe_one(acc.X);
  fe_one(acc.Y);
  fe_zero(acc.Z);
  for (int i = 26; i >= 0; i--) {
    if (i != 26)
      for (int z = 0; z < 5; z++) jac_dbl(acc);
    const int d = (int)win5_3(K, i) - 16;
    if (d) {
      JacC<F> e;
      jacc_load(e, tab + (size_t)((d < 0 ? -d : d) - 1) * 5 * F::SN);
      Fe<F> x;
      fe_mul(x, e.X, mulx);  // lane 1: phi
      e.X = x;
      if ((d < 0) != neg) {
        Fe<F> ny;
        fe_neg(ny, e.Y);
        e.Y = ny;
      }
      jac_add_cached(acc, e);
    }
  }
}
// pair-cooperative t = k v (k decomposed: dk = |k1|, |k2|, signs): lane q of the pair computes
// its half, the pair swaps and adds (both lanes end with t)
template <class F>
__device__ __forceinline__ void glv_scl_pair(Xyzz<F> &t, const Xyzz<F> &v, const uint64_t *__restrict__ dk,
                                             const Fe<F> &beta, uint32_t *__restrict__ tab) {
  const int q = (int)(threadIdx.x & 1);
  Jac<F> r;
  if (xyzz_is_inf(v)) {
    fe_one(r.X);
    fe_one(r.Y);
    fe_zero(r.Z);
  } else {
    Jac<F> p;
    xyzz_to_jac(p, v);
    Fe<F> mulx;
    if (q) mulx = beta;
    else fe_one(mulx);
    // the pair's table lives in lane 0's scratch slot
    jac_scl130_pair(r, p, dk + 3 * q, ((dk[6] >> q) & 1) != 0, mulx, tab - (size_t)q * scl_tab_words<F>());
  }
  Jac<F> o;
  fe_pair_swap(o.X, r.X);
  fe_pair_swap(o.Y, r.Y);
  fe_pair_swap(o.Z, r.Z);
  jac_add_any(r, o);
  jac_to_xyzz(t, r);
}

// forward DIT stage on lane pairs: pair = butterfly; lane 0 writes u + t, lane 1 u - t
template <class C>
__global__ void __launch_bounds__(256, fft_waves<C>()) k_fft_fwd_stage_glv(int m, int s, const uint32_t *__restrict__ A,
                                                           uint32_t *__restrict__ B, const uint64_t *__restrict__ twg,
                                                           W6 beta_ref, uint32_t *__restrict__ scratch, int lanes) {
  using F = typename C::Fp;
  const int half = 1 << (s - 1);
  const size_t nl = (size_t)1 << m;  // two lanes per butterfly
  Fe<F> beta, t0;
  fe_load_ref(t0, beta_ref.w);
  fe_to_int(beta, t0);
  uint32_t *tab = scratch + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * scl_tab_words<F>();
  for (size_t L = (size_t)blockIdx.x * blockDim.x + threadIdx.x; L < nl; L += (size_t)lanes) {
    const size_t b = L >> 1;
    const int q = (int)(L & 1);
    const size_t blk = b >> (s - 1), j = b & (half - 1);
    const size_t k0 = (blk << s) + j;
    Xyzz<F> u, v, t;
    xyzz_load(v, A + (k0 + half) * xw<F>());
    if (j == 0) t = v;
    else glv_scl_pair(t, v, twg + (j << (m - s)) * 8, beta, tab);
    if (q) {
      Xyzz<F> nt;
      xyzz_neg(nt, t);
      t = nt;
    }
    xyzz_load(u, A + k0 * xw<F>());  // read after the multiplication: not live across its chain
    xyzz_add(u, t);
    xyzz_store(B + (k0 + (q ? half : 0)) * xw<F>(), u);
  }
}

// inverse DIF stage on lane pairs, factor 1/2 per level deferred (k_fft_inv_first_glv applies N^-1
// once): lane 0 writes u + v, lane 1 (u - v) w^-j
template <class C>
__global__ void __launch_bounds__(256, fft_waves<C>()) k_fft_inv_stage_glv(int m, int s, const uint32_t *__restrict__ A,
                                                           uint32_t *__restrict__ B, const uint64_t *__restrict__ twg,
                                                           W6 beta_ref, uint32_t *__restrict__ scratch, int lanes) {
  using F = typename C::Fp;
  const int half = 1 << (s - 1);
  const size_t nl = (size_t)1 << m;
  Fe<F> beta, t0;
  fe_load_ref(t0, beta_ref.w);
  fe_to_int(beta, t0);
  uint32_t *tab = scratch + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * scl_tab_words<F>();
  for (size_t L = (size_t)blockIdx.x * blockDim.x + threadIdx.x; L < nl; L += (size_t)lanes) {
    const size_t b = L >> 1;
    const int q = (int)(L & 1);
    const size_t blk = b >> (s - 1), j = b & (half - 1);
    const size_t k0 = (blk << s) + j;
    Xyzz<F> u, v, d;
    xyzz_load(u, A + k0 * xw<F>());
    xyzz_load(v, A + (k0 + half) * xw<F>());
    if (q == 0) {  // lane 0's output u + v is written first: u, v are not live across the chain
      Xyzz<F> w = u;
      xyzz_add(w, v);
      xyzz_store(B + k0 * xw<F>(), w);
    }
    d = u;
    {
      Xyzz<F> nv;
      xyzz_neg(nv, v);
      xyzz_add(d, nv);
    }
    Xyzz<F> t = d;
    if (j != 0) glv_scl_pair(t, d, twg + (j << (m - s)) * 8, beta, tab);
    if (q) xyzz_store(B + (k0 + half) * xw<F>(), t);
  }
}

// the inverse's FIRST stage (s = m) with the deferred N^-1 applied to both outputs: four lanes
// per butterfly, pair 0 -> (u + v) N^-1 (dkn), pair 1 -> (u - v) w^-j N^-1 (twn[j], the twiddle
// with N^-1 folded in) -- one doubled stage instead of a stage plus a scaling pass over N points
template <class C>
__global__ void __launch_bounds__(256, fft_waves<C>()) k_fft_inv_first_glv(int m, const uint32_t *__restrict__ A,
                                                           uint32_t *__restrict__ B, const uint64_t *__restrict__ twn,
                                                           const uint64_t *__restrict__ dkn, W6 beta_ref,
                                                           uint32_t *__restrict__ scratch, int lanes) {
  using F = typename C::Fp;
  const size_t half = (size_t)1 << (m - 1);
  const size_t nl = (size_t)1 << (m + 1);  // 4 lanes x N / 2 butterflies
  Fe<F> beta, t0;
  fe_load_ref(t0, beta_ref.w);
  fe_to_int(beta, t0);
  uint32_t *tab = scratch + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * scl_tab_words<F>();
  for (size_t L = (size_t)blockIdx.x * blockDim.x + threadIdx.x; L < nl; L += (size_t)lanes) {
    const size_t j = L >> 2;  // s = m: one block, k0 = j
    const int pr = (int)((L >> 1) & 1);
    Xyzz<F> u, v, d, t;
    xyzz_load(u, A + j * xw<F>());
    xyzz_load(v, A + (j + half) * xw<F>());
    d = u;
    if (pr) {
      Xyzz<F> nv;
      xyzz_neg(nv, v);
      xyzz_add(d, nv);
    } else {
      xyzz_add(d, v);
    }
    glv_scl_pair(t, d, pr ? twn + j * 8 : dkn, beta, tab);
    if ((L & 1) == 0) xyzz_store(B + (j + (pr ? half : 0)) * xw<F>(), t);
  }
}

// ---------------------------------------------------------------------------- radix-2^b GLV stages
// (round 6) At KZG SRS sizes (2^12 - 2^14 points, examples/KZG.hs:55) a radix-2 stage holds N lanes
// (two per butterfly) = 64 - 256 wavefronts for 1024 SIMDs, and every stage is one lane's ~1250-
// product chain: the transform costs m chains.  On the order-r subgroup the per-level scalars may be
// combined mod r, so a stage can take b bits at once: a Stockham radix-r step (r = 2^b, natural
// order in and out) with the r-point DFT's roots folded into the twiddles.  With L the transform
// length done so far, L' = r L and G = N / L' classes, the data holds at index c + (N / L) k the
// length-L DFT of x[c + (N / L) n]; a step computes, for each class c' < G and k0 < L,
//   X[c' + G (k0 + q L)] = sum_{m < r} w_N^(G m k0 + m q N / r) A[c' + G (m + r k0)],   q < r,
// whose scalar is w_N^(G m k0 + delta N / r) times (-1)^sigma for m q mod r = delta + sigma r / 2: the
// products are (m, delta) pairs -- 1 / 5 / 21 / 85 per group for r = 2 / 4 / 8 / 16 -- every one an
// independent GLV lane pair (k_fft_radix_prod), then each output adds its r terms (k_fft_radix_sum).
// A stage is then ONE multiplication chain for b bits; the work per point-bit grows (1/2, 5/8, 7/8,
// 4/3 products), so the planner (radix_plan) takes b > 1 only while the stage's lanes fit about one
// wavefront per SIMD.  The inverse is the same DIT with w^-1 and N^-1 folded into the first stage's
// scalars (the m = 0 term becomes a product too).
struct RadixPlan {
  int b, D;              // radix 2^b; products per group
  uint8_t pm[96], pd[96];  // product p -> (m, delta)
  uint8_t qmap[16][16];  // (q, m) -> product index (255: the unscaled m = 0 input itself)
  uint8_t qsgn[16][16];  // (q, m) -> negate
};

template <class C>
__global__ void __launch_bounds__(256, fft_waves<C>()) k_fft_radix_prod(int m, int lgG, const uint32_t *__restrict__ A,
                                                         uint32_t *__restrict__ P, const uint64_t *__restrict__ twg,
                                                         int scaled, W6 beta_ref, uint32_t *__restrict__ scratch,
                                                         int lanes, RadixPlan plan) {
  using F = typename C::Fp;
  const int b = plan.b;
  const size_t N = (size_t)1 << m, NG = N >> b, G = (size_t)1 << lgG;
  const size_t nl = 2 * NG * (size_t)plan.D;  // two lanes per product
  Fe<F> beta, t0;
  fe_load_ref(t0, beta_ref.w);
  fe_to_int(beta, t0);
  uint32_t *tab = scratch + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * scl_tab_words<F>();
  for (size_t L = (size_t)blockIdx.x * blockDim.x + threadIdx.x; L < nl; L += (size_t)lanes) {
    const size_t pair = L >> 1;
    const int q = (int)(L & 1);
    const size_t pidx = pair >> (m - b), g = pair & (NG - 1);  // product-major: neighbours share (m, delta)
    const size_t mm = plan.pm[pidx], dl = plan.pd[pidx];
    const size_t c = g & (G - 1), k0 = g >> lgG;
    Xyzz<F> v, t;
    xyzz_load(v, A + (c + G * (mm + (k0 << b))) * xw<F>());
    size_t e = (G * mm * k0 + dl * NG) & (N - 1);
    const bool neg = e >= N / 2;
    e &= N / 2 - 1;
    if (e == 0 && !scaled) t = v;  // w^0 = 1 (the pair is uniform: both lanes take this branch)
    else glv_scl_pair(t, v, twg + e * 8, beta, tab);
    if (neg) {
      Xyzz<F> nt;
      xyzz_neg(nt, t);
      t = nt;
    }
    if (q == 0) xyzz_store(P + (pidx * NG + g) * xw<F>(), t);
  }
}

// The r terms of an output are summed by S = min(r, 4) lanes (each adds every S-th term), then the
// S partial sums are combined across the lanes by shuffles: log2 S + r / S - 1 additions deep
// instead of r - 1 (radix 16: 5 instead of 15).  S consecutive lanes per output.
template <class F>
__device__ __forceinline__ void xyzz_shfl_xor(Xyzz<F> &r, const Xyzz<F> &a, int mask) {
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    r.X.v[i] = (uint32_t)__shfl_xor((int)a.X.v[i], mask);
    r.Y.v[i] = (uint32_t)__shfl_xor((int)a.Y.v[i], mask);
    r.ZZ.v[i] = (uint32_t)__shfl_xor((int)a.ZZ.v[i], mask);
    r.ZZZ.v[i] = (uint32_t)__shfl_xor((int)a.ZZZ.v[i], mask);
  }
}
template <class C>
__global__ void __launch_bounds__(256) k_fft_radix_sum(int m, int lgG, const uint32_t *__restrict__ A,
                                                       const uint32_t *__restrict__ P, uint32_t *__restrict__ B,
                                                       RadixPlan plan) {
  using F = typename C::Fp;
  const int b = plan.b, r = 1 << b;
  const int lgS = b < 2 ? b : 2, S = 1 << lgS;
  const size_t N = (size_t)1 << m, NG = N >> b, G = (size_t)1 << lgG;
  const size_t gt = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t o = gt >> lgS;
  const int j = (int)(gt & (S - 1));
  if (o >= N) return;  // N S is a multiple of 64 (N >= 16) or the grid's lanes of one output stay together
  const size_t g = o & (NG - 1);
  const int q = (int)(o >> (m - b));
  const size_t c = g & (G - 1), k0 = g >> lgG;
  Xyzz<F> acc, t;
  xyzz_set_inf(acc);
  for (int mm = j; mm < r; mm += S) {
    if (mm == 0) {
      const int p0 = plan.qmap[q][0];
      if (p0 == 255) xyzz_load(t, A + (c + G * (k0 << b)) * xw<F>());
      else xyzz_load(t, P + ((size_t)p0 * NG + g) * xw<F>());
    } else {
      xyzz_load(t, P + ((size_t)plan.qmap[q][mm] * NG + g) * xw<F>());
      if (plan.qsgn[q][mm]) {
        Xyzz<F> nt;
        xyzz_neg(nt, t);
        t = nt;
      }
    }
    xyzz_add(acc, t);
  }
  for (int d = 1; d < S; d <<= 1) {
    Xyzz<F> other;
    xyzz_shfl_xor(other, acc, d);
    xyzz_add(acc, other);
  }
  if (j == 0) xyzz_store(B + o * xw<F>(), acc);  // = c' + G (k0 + q L)
}

// r = [|z|] p for BLS12-381's z = -0xd201000000010000 (bits 63, 62, 60, 57, 48, 16): 63 doublings
// and 5 additions, the membership test's chain (k_subgroup_check)
template <class F>
__device__ __forceinline__ void jac_mul_absz(Jac<F> &r, const Jac<F> &p) {
  JacC<F> pc;
  jac_cache(pc, p);
  r = p;
  // runs of doublings between the set bits, each a rolled loop: the fully unrolled chain (63
  // inlined doublings) held 512 VGPRs and spilled 230 of them to scratch
  constexpr int kRun[6] = {1, 2, 3, 9, 32, 16};  // doublings before the additions at bits 62, 60, 57, 48, 16; tail
  for (int s = 0; s < 6; s++) {
#pragma unroll 1
    for (int i = 0; i < kRun[s]; i++) jac_dbl(r);
    if (s < 5 && !jac_is_inf(p)) jac_add_cached(r, pc);
  }
}

// subgroup membership (curves with a cofactor): phi(P) == [lambda] P for every point (lambda
// 128 bits on BLS12-381; tools/gen_glv.py checks the test on subgroup and non-subgroup points).
// bad[block] = 1 when some point of the block fails.
template <class C>
__global__ void __launch_bounds__(256, fft_waves<C>()) k_subgroup_check(int n, const uint32_t *__restrict__ A, W6 beta_ref, int lanes,
                                                        uint32_t *__restrict__ bad) {
  using F = typename C::Fp;
  Fe<F> beta, t0;
  fe_load_ref(t0, beta_ref.w);
  fe_to_int(beta, t0);
  int fail = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)n; i += (size_t)lanes) {
    Xyzz<F> v;
    xyzz_load(v, A + i * xw<F>());
    if (xyzz_is_inf(v)) continue;
    Jac<F> p, r;
    {  // [lambda] P = [|z|]([|z|] P) - P (lambda = z^2 - 1; |z| = 0xd201000000010000 has 6 bits set).
      // The two [|z|] chains run as ONE rolled loop body and P is re-read from A afterwards
      // instead of staying live across them: kept live and inlined twice, the kernel held 512
      // VGPRs and spilled ~260 to scratch inside the doubling chains.
      xyzz_to_jac(r, v);
#pragma unroll 1
      for (int rep = 0; rep < 2; rep++) {
        Jac<F> t;
        jac_mul_absz(t, r);
        r = t;
      }
      xyzz_load(v, A + i * xw<F>());
      xyzz_to_jac(p, v);
      Jac<F> np = p;
      fe_neg(np.Y, p.Y);
      JacC<F> nc;
      jac_cache(nc, np);
      jac_add_cached(r, nc);
    }
    if (jac_is_inf(r)) {
      fail = 1;
      continue;
    }
    // (beta Xp : Yp : Zp) == (Xr : Yr : Zr): Xr Zp^2 == beta Xp Zr^2 and Yr Zp^3 == Yp Zr^3
    Fe<F> zp2, zr2, zp3, zr3, a, b, c;
    fe_sqr(zp2, p.Z);
    fe_sqr(zr2, r.Z);
    fe_mul(zp3, zp2, p.Z);
    fe_mul(zr3, zr2, r.Z);
    fe_mul(a, r.X, zp2);
    fe_mul(c, p.X, beta);
    fe_mul(b, c, zr2);
    fe_sub(c, a, b);
    if (!fe_is_zero(c)) fail = 1;
    fe_mul(a, r.Y, zp3);
    fe_mul(b, p.Y, zr3);
    fe_sub(c, a, b);
    if (!fe_is_zero(c)) fail = 1;
  }
  const int any = __syncthreads_or(fail);
  if (threadIdx.x == 0) bad[blockIdx.x] = any ? 1u : 0u;
}

// forward DIT stage s (block 2^s): lane = butterfly (blk, j); t = w_s^j v (w_s^j = tw[j 2^(m-s)],
// canonical Fr in standard form, = 1 for j = 0); out = (u + t, u - t)
template <class C>
__global__ void __launch_bounds__(256) k_fft_fwd_stage(int m, int s, const uint32_t *__restrict__ A,
                                                       uint32_t *__restrict__ B, const uint64_t *__restrict__ tw,
                                                       uint32_t *__restrict__ scratch, int lanes) {
  using F = typename C::Fp;
  const int half = 1 << (s - 1);
  const size_t nb = (size_t)1 << (m - 1);
  for (size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (size_t)lanes) {
    const size_t blk = b >> (s - 1), j = b & (half - 1);
    const size_t k0 = (blk << s) + j;
    Xyzz<F> u, v, t;
    xyzz_load(u, A + k0 * xw<F>());
    xyzz_load(v, A + (k0 + half) * xw<F>());
    if (j == 0) {
      t = v;
    } else {
      const uint64_t *k = tw + (j << (m - s)) * 4;
      xyzz_scl(t, v, k, scratch + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * scl_tab_words<F>());
    }
    Xyzz<F> x = u, nt;
    xyzz_add(x, t);
    xyzz_neg(nt, t);
    xyzz_add(u, nt);
    xyzz_store(B + k0 * xw<F>(), x);
    xyzz_store(B + (k0 + half) * xw<F>(), u);
  }
}

// inverse DIF stage s: lane = output (butterfly, which): which 0 -> (u + v) * 1/2,
// which 1 -> (u - v) * (w_s^-j / 2) (tw[e] = inv(w)^e / 2, standard form); half = std(1/2)
template <class C>
__global__ void __launch_bounds__(256) k_fft_inv_stage(int m, int s, const uint32_t *__restrict__ A,
                                                       uint32_t *__restrict__ B, const uint64_t *__restrict__ tw,
                                                       uint32_t *__restrict__ scratch, int lanes) {
  using F = typename C::Fp;
  const int half = 1 << (s - 1);
  const size_t no = (size_t)1 << m;
  for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o < no; o += (size_t)lanes) {
    const size_t b = o >> 1;
    const int which = (int)(o & 1);
    const size_t blk = b >> (s - 1), j = b & (half - 1);
    const size_t k0 = (blk << s) + j;
    Xyzz<F> u, v, t;
    xyzz_load(u, A + k0 * xw<F>());
    xyzz_load(v, A + (k0 + half) * xw<F>());
    if (which == 0) {
      xyzz_add(u, v);
    } else {
      Xyzz<F> nv;
      xyzz_neg(nv, v);
      xyzz_add(u, nv);
    }
    const uint64_t *k = tw + (which ? (j << (m - s)) : 0) * 4;  // tw[0] = 1/2
    xyzz_scl(t, u, k, scratch + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * scl_tab_words<F>());
    xyzz_store(B + (k0 + (which ? half : 0)) * xw<F>(), t);
  }
}

// tw[e] = std(scale * base^e) for e < cnt (base, scale: Fr reference Montgomery form)
template <class Fr>
__global__ void __launch_bounds__(256) k_fft_tw(int cnt, W6 base, W6 scale, uint64_t *__restrict__ tw) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cnt) return;
  Fe<Fr> b, acc, t;
  ld_int(b, base.w);
  fe_load_ref(acc, scale.w);  // reference form
  Fe<Fr> p = b;
  for (int x = e; x; x >>= 1) {
    if (x & 1) { fe_mul(t, acc, p); acc = t; }
    fe_sqr(t, p);
    p = t;
  }
  Fe<Fr> sd;
  fe_ref_to_std(sd, acc);
  fe_store_ref(tw + (size_t)e * 4, sd);
}

// ---------------------------------------------------------------------------- host side

template <class HF>
static W6 exp_p_minus_2() {
  W6 e = {{0, 0, 0, 0, 0, 0}};
  for (int j = 0; j < HF::N; j++) e.w[j] = HF::P[j];
  uint64_t br = 2;
  for (int j = 0; j < HF::N && br; j++) {
    const uint64_t o = e.w[j];
    e.w[j] = o - br;
    br = o < br ? 1 : 0;
  }
  return e;
}
template <class HF>
static W6 one_ref() {
  W6 o = {{0, 0, 0, 0, 0, 0}};
  for (int j = 0; j < HF::N; j++) o.w[j] = HF::ONE[j];
  return o;
}

template <class C>
static void batch_from_affine_t(Device &dev, int n, const uint64_t *src, uint64_t *tgt, bool host_io, bool jac) {
  using HF = typename HostOf<C>::Fp;
  constexpr int NP = C::NP64;
  if (n <= 0) return;
  hipStream_t st = dev.stream;
  const size_t N = (size_t)n;
  dev.arena.reserve(N * 5 * NP * 8 + (1 << 20));
  dev.arena.reset();
  const uint64_t *ds = src;
  uint64_t *dt = tgt;
  if (host_io) {
    uint64_t *a = dev.arena.take<uint64_t>(N * 2 * NP);
    ZK_CHECK(hipMemcpyAsync(a, src, N * 2 * NP * 8, hipMemcpyHostToDevice, st));
    ds = a;
    dt = dev.arena.take<uint64_t>(N * 3 * NP);
  }
  if (jac) hipLaunchKernelGGL((k_from_affine<C, true>), dim3(div_up(N, 256)), dim3(256), 0, st, n, ds, dt, one_ref<HF>());
  else hipLaunchKernelGGL((k_from_affine<C, false>), dim3(div_up(N, 256)), dim3(256), 0, st, n, ds, dt, one_ref<HF>());
  ZK_CHECK(hipGetLastError());
  if (host_io) copy_to_host(dev, st, tgt, dt, N * 3 * NP * 8);  // fresh caller arrays: zk_runtime.hpp
  ZK_CHECK(hipStreamSynchronize(st));
}

// points per Fermat inversion in k_norm_chunks: each lane's chain is CHK prefix products, one
// inversion (~490 products) and ~5 products per point on the way back, and the lanes are N / CHK.
// The kernel is latency-bound on that chain (one wavefront per SIMD at 248-254 VGPRs already
// issues most of what a SIMD can), so CHK keeps ~one wavefront per SIMD busy: N / ZK_NORM_LANES
// (default 65536) within [2, 32] -- 2^16 points: 2 (the group FFT), 2^20: 16.  Measured
// (profiles/r05u_inversion_chunks.txt): 2^20 0.95 ms at 32, 0.81 at 16, 1.16 at 8; 2^16 0.541 at
// 4, 0.528 at 2, 0.553 at 1.
// ZK_INV_SG=0: Fermat inversions in k_norm_chunks (A/B hook, read once; default: safegcd)
static bool inv_sg() {
  static const bool on = [] {
    const char *e = getenv("ZK_INV_SG");
    return !(e && e[0] == '0');
  }();
  return on;
}
// ZK_INV_STRIDE=0: consecutive-point chunks (A/B hook, read once; default strided)
static bool inv_strided() {
  static const bool on = [] {
    const char *e = getenv("ZK_INV_STRIDE");
    return !(e && e[0] == '0');
  }();
  return on;
}
// ZK_NORM_BF=0: k_norm_chunks with the round-6 branches (A/B hook, read once; default branch-free)
static bool norm_bf() {
  static const bool on = [] {
    const char *e = getenv("ZK_NORM_BF");
    return !(e && e[0] == '0');
  }();
  return on;
}
template <class C, int MODE>
static void launch_norm(hipStream_t st, int n, int chk, const void *src, uint64_t *scratch, uint64_t *tgt, W6 pm2,
                        int bitrev_m) {
  const size_t lanes = ((size_t)n + chk - 1) / chk;
  const dim3 grid(div_up(lanes, 256));
  if (inv_sg() && inv_strided() && norm_bf())
    hipLaunchKernelGGL((k_norm_chunks<C, MODE, true, true, true>), grid, dim3(256), 0, st, n, chk, src, scratch, tgt, pm2,
                       bitrev_m, (int)lanes);
  else if (inv_sg() && inv_strided())
    hipLaunchKernelGGL((k_norm_chunks<C, MODE, true, true, false>), grid, dim3(256), 0, st, n, chk, src, scratch, tgt,
                       pm2, bitrev_m, (int)lanes);
  else if (inv_sg())
    hipLaunchKernelGGL((k_norm_chunks<C, MODE, true, false, false>), grid, dim3(256), 0, st, n, chk, src, scratch, tgt,
                       pm2, bitrev_m, (int)lanes);
  else
    hipLaunchKernelGGL((k_norm_chunks<C, MODE, false, false, false>), grid, dim3(256), 0, st, n, chk, src, scratch, tgt,
                       pm2, bitrev_m, (int)lanes);
  ZK_CHECK(hipGetLastError());
}
static int norm_chk(size_t N) {
  static const size_t target = [] {
    const char *e = getenv("ZK_NORM_LANES");
    const long v = e ? atol(e) : 0;
    return v > 0 ? (size_t)v : (size_t)65536;
  }();
  const size_t c = N / target;
  return c < 2 ? 2 : (c > 32 ? 32 : (int)c);
}

template <class C>
static void batch_to_affine_t(Device &dev, int n, const uint64_t *src, uint64_t *tgt, bool host_io, bool jac) {
  using HF = typename HostOf<C>::Fp;
  constexpr int NP = C::NP64;
  if (n <= 0) return;
  hipStream_t st = dev.stream;
  const size_t N = (size_t)n;
  dev.arena.reserve(N * 6 * NP * 8 + (1 << 20));
  dev.arena.reset();
  const uint64_t *ds = src;
  uint64_t *dt = tgt;
  if (host_io) {
    uint64_t *a = dev.arena.take<uint64_t>(N * 3 * NP);
    ZK_CHECK(hipMemcpyAsync(a, src, N * 3 * NP * 8, hipMemcpyHostToDevice, st));
    ds = a;
    dt = dev.arena.take<uint64_t>(N * 2 * NP);
  }
  uint64_t *scratch = dev.arena.take<uint64_t>(N * NP);
  const int chk = norm_chk(N);
  if (jac)
    launch_norm<C, MODE_JAC_TO_AFF>(st, n, chk, ds, scratch, dt, exp_p_minus_2<HF>(), 0);
  else
    launch_norm<C, MODE_PROJ_TO_AFF>(st, n, chk, ds, scratch, dt, exp_p_minus_2<HF>(), 0);
  ZK_CHECK(hipGetLastError());
  if (host_io) copy_to_host(dev, st, tgt, dt, N * 2 * NP * 8);
  ZK_CHECK(hipStreamSynchronize(st));
}

static RadixPlan make_radix_plan(int b, bool scaled) {
  RadixPlan pl;
  memset(&pl, 0, sizeof pl);
  const int r = 1 << b, h = r > 2 ? r / 2 : 1;
  int idx[16][16];
  for (auto &row : idx)
    for (int &x : row) x = -1;
  pl.b = b;
  pl.D = 0;
  auto add = [&](int mm, int dl) {
    idx[mm][dl] = pl.D;
    pl.pm[pl.D] = (uint8_t)mm;
    pl.pd[pl.D] = (uint8_t)dl;
    pl.D++;
  };
  if (scaled) add(0, 0);
  for (int mm = 1; mm < r; mm++)
    for (int q = 0; q < r; q++) {
      const int dl = (mm * q % r) % h;
      if (idx[mm][dl] < 0) add(mm, dl);
    }
  for (int q = 0; q < r; q++)
    for (int mm = 0; mm < r; mm++) {
      if (mm == 0) {
        pl.qmap[q][0] = scaled ? (uint8_t)idx[0][0] : 255;
        continue;
      }
      const int t = mm * q % r;
      pl.qmap[q][mm] = (uint8_t)idx[mm][t % h];
      pl.qsgn[q][mm] = (uint8_t)(r > 2 ? t >= h : t == 1);
    }
  return pl;
}
// products per group of a radix-2^b stage (unscaled): r = 2, 4, 8, 16 -> 1, 5, 21, 85
static int radix_products(int b) { return make_radix_plan(b, false).D; }

// Bits per stage for a 2^m GLV transform, or {} for the fused radix-2 stages.  A stage costs its
// multiplication chain times the rounds its wavefronts take: on BLS12-381 (stages at 445-503
// VGPRs, one wavefront per SIMD) ceil(waves / 1024) chains; on BN254 (two per SIMD) one chain up to
// 1024 waves and 1.75 per 2048 beyond (measured: a 2^15 radix-4 stage of 1280 waves took 1.75x a
// 512-wave radix-2 stage, profiles/r06a_fft_radix_ab.txt).  A radix-2^b stage adds its sum kernel,
// r - 1 XYZZ additions per output (~1/90 chain each) and ~0.02 chain of launches and product
// traffic.  The fused radix-2 stages cost their rounds only; the radix plan (dynamic programming
// over b = 1..4) is taken when it is at least 3 % cheaper.  ZK_FFT_RADIX=1 forces the fused stages,
// 2..4 that radix for every stage (the last one takes the remainder) -- A/B hooks.
static double stage_rounds(double waves, int waves_per_simd) {
  if (waves_per_simd <= 1) return std::ceil(waves / 1024.0);
  return waves <= 1024.0 ? 1.0 : 1.75 * std::ceil(waves / 2048.0);
}
static std::vector<int> radix_plan(int m, int waves_per_simd) {
  static const int forced = [] {
    const char *e = getenv("ZK_FFT_RADIX");
    return e ? atoi(e) : 0;
  }();
  std::vector<int> bits;
  if (forced == 1) return bits;
  if (forced >= 2 && forced <= 4) {
    int left = m;
    while (left > 0) {
      const int b = std::min(forced, left);
      bits.push_back(b);
      left -= b;
    }
    return bits;
  }
  const double N = std::ldexp(1.0, m);
  const double glanes = std::min(N, 131072.0);  // the fused stages' lanes (grid-strided beyond)
  const double fused = m * stage_rounds(glanes / 64.0, waves_per_simd) * std::ceil(N / glanes);
  std::vector<double> best(m + 1, 1e30);
  std::vector<int> how(m + 1, 0);
  best[0] = 0;
  for (int k = 1; k <= m; k++)
    for (int b = 1; b <= 4 && b <= k; b++) {
      const double waves = std::ceil(2.0 * radix_products(b) * (N / (1 << b)) / 64.0);
      const double c = best[k - b] + stage_rounds(waves, waves_per_simd) + ((1 << b) - 1) / 90.0 + 0.02;
      if (c < best[k]) {
        best[k] = c;
        how[k] = b;
      }
    }
  if (!(best[m] < 0.97 * fused)) return bits;
  for (int k = m; k > 0; k -= how[k]) bits.push_back(how[k]);
  return bits;  // any order: every stage is the same Stockham step
}

template <class C>
static void g1_fft_t(Device &dev, int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt, bool host_io,
                     bool inverse, bool jac) {
  using F = typename C::Fp;
  using HF = typename HostOf<C>::Fp;
  using HR = typename HostOf<C>::Fr;
  using Fr = typename C::Fr;
  constexpr int NP = C::NP64;
  ZK_REQUIRE(m >= 0 && m <= 26, "G1 fft: log2 size out of range (0..26)");
  hipStream_t st = dev.stream;
  const size_t N = (size_t)1 << m;
  // scalar-multiplication lanes are grid-strided so the per-lane table scratch stays bounded.
  // (Round 4 measured quad-cooperative stages -- 4 lanes per multiplication, signed 5-bit
  // windows, xyzz_dbl_quad / xyzz_add_quad: BLS12-381 2^16 forward 50 vs 55 ms, inverse 102 vs
  // 61 ms; at 1-2 waves per SIMD the quads' 4x lanes take extra rounds, profiles/r04g_*.)
  const size_t work = inverse ? N : N / 2;
  size_t lanes = work < (1u << 17) ? work : (1u << 17);
  lanes = (lanes + 255) & ~(size_t)255;
  if (lanes == 0) lanes = 256;
  const size_t tw_cnt = N > 1 ? N / 2 : 1;
  // GLV stages: two lanes per multiplication (forward N / 2 butterflies, inverse N / 2 plus the
  // final N^-1 scaling of N points)
  size_t glanes = N < (1u << 17) ? N : (1u << 17);
  glanes = (glanes + 255) & ~(size_t)255;
  // radix-2^b stages (GLV path only, m > 0)
  const std::vector<int> rbits = m > 0 ? radix_plan(m, fft_waves<C>()) : std::vector<int>();
  const bool radix = !rbits.empty();
  size_t rlanes = 0, pbuf = 0;
  if (radix)
    for (int b : rbits) {
      const size_t np = (size_t)(make_radix_plan(b, true).D) * (N >> b);
      rlanes = std::max(rlanes, std::min(2 * np, (size_t)1 << 17));
      pbuf = std::max(pbuf, np);
    }
  rlanes = (rlanes + 255) & ~(size_t)255;
  const size_t tlanes = std::max(std::max(lanes, glanes), rlanes);
  const size_t nbad = div_up(N, 256);
  dev.arena.reserve(N * 3 * NP * 8 * (host_io ? 2 : 0) + 3 * N * xw<F>() * 4 + tlanes * scl_tab_words<F>() * 4 +
                    tw_cnt * 32 + 2 * tw_cnt * 64 + 64 + nbad * 4 + N * NP * 8 + pbuf * xw<F>() * 4 + (1 << 20));
  dev.arena.reset();
  const uint64_t *ds = src;
  uint64_t *dt = tgt;
  if (host_io) {
    uint64_t *a = dev.arena.take<uint64_t>(N * 3 * NP);
    ZK_CHECK(hipMemcpyAsync(a, src, N * 3 * NP * 8, hipMemcpyHostToDevice, st));
    ds = a;
    dt = dev.arena.take<uint64_t>(N * 3 * NP);
  }
  uint32_t *A = dev.arena.take<uint32_t>(N * xw<F>());
  uint32_t *B = dev.arena.take<uint32_t>(N * xw<F>());
  uint32_t *scratch = dev.arena.take<uint32_t>(tlanes * scl_tab_words<F>());
  uint64_t *tw = dev.arena.take<uint64_t>(tw_cnt * 4);
  uint64_t *twg = dev.arena.take<uint64_t>(2 * tw_cnt * 8 + 8);  // w^e, then (w^-1)^e N^-1, then N^-1
  uint32_t *bad = dev.arena.take<uint32_t>(nbad);
  uint64_t *nscratch = dev.arena.take<uint64_t>(N * NP);
  uint32_t *Pb = radix ? dev.arena.take<uint32_t>(pbuf * xw<F>()) : nullptr;

  // input order: bit-reversed for the radix-2 forward stages, natural for the inverse (DIF) and the
  // Stockham radix-2^b stages
  auto load_points = [&](bool natural) {
    const int br = (inverse || natural) ? 0 : m;
    if (jac)
      hipLaunchKernelGGL((k_fft_load<C, true>), dim3(div_up(N, 256)), dim3(256), 0, st, (int)N, br, ds, A);
    else
      hipLaunchKernelGGL((k_fft_load<C, false>), dim3(div_up(N, 256)), dim3(256), 0, st, (int)N, br, ds, A);
    ZK_CHECK(hipGetLastError());
  };
  static const bool glv_on0 = [] {
    const char *e = getenv("ZK_FFT_GLV");
    return !(e && e[0] == '0');
  }();
  const bool use_radix = radix && glv_on0;
  load_points(use_radix);
  // GLV stages when every point is in the order-r subgroup (always on BN254, cofactor 1; checked
  // on BLS12-381).  ZK_FFT_GLV=0: the integer stages always (A/B hook, read once).
  static const bool glv_on = [] {
    const char *e = getenv("ZK_FFT_GLV");
    return !(e && e[0] == '0');
  }();
  bool glv = glv_on && m > 0;
  const GlvParams gp = glv_params<C>();
  const W6 beta = glv_beta_ref<C>();
  // BLS12-381: the membership test runs on the context's side stream, on a copy of the loaded
  // points, BESIDE the GLV stages (speculative: both are one chain per lane at <= one wavefront
  // per SIMD up to 2^16, so they share the SIMDs' issue slots; before round 5 the stages waited
  // for it, ~1.2 ms of a 26 ms 2^16 transform).  A point outside the subgroup (the result is
  // read after the stages) discards the GLV result and reruns the integer stages from the input.
  uint32_t *hb = nullptr;
  unsigned cgrid = 0;
  // Every exit path -- a throw from the stages or the fallback in recoverable error mode included --
  // waits for the side stream's test and its copy into the pinned staging before this call returns,
  // so no late copy can land in the next call's staging or arena.
  struct AuxJoin {
    hipStream_t s = nullptr;
    ~AuxJoin() {
      if (s) (void)hipStreamSynchronize(s);
    }
  } aux_join;
  if (glv && C::NP64 == 6) {
    uint32_t *Acopy = dev.arena.take<uint32_t>(N * xw<F>());
    ZK_CHECK(hipMemcpyAsync(Acopy, A, N * xw<F>() * 4, hipMemcpyDeviceToDevice, st));
    hipEvent_t loaded = dev.split_event(0), checked = dev.split_event(1);
    ZK_CHECK(hipEventRecord(loaded, st));
    hipStream_t st2 = dev.aux_stream();
    ZK_CHECK(hipStreamWaitEvent(st2, loaded, 0));
    aux_join.s = st2;
    cgrid = (unsigned)(glanes / 256);
    hipLaunchKernelGGL(k_subgroup_check<C>, dim3(cgrid), dim3(256), 0, st2, (int)N, Acopy, beta, (int)glanes, bad);
    ZK_CHECK(hipGetLastError());
    hb = reinterpret_cast<uint32_t *>(dev.host_staging(cgrid * 4 + 64));
    ZK_CHECK(hipMemcpyAsync(hb, bad, cgrid * 4, hipMemcpyDeviceToHost, st2));
    ZK_CHECK(hipEventRecord(checked, st2));
  }
  // Stockham radix-2^b stages (natural order in and out)
  auto run_radix = [&] {
    zkh::Fe<HR> g, one, ninv;
    memcpy(g.v, gen, sizeof g.v);
    zkh::set_one(one);
    if (inverse) zkh::inv(g, g);
    W6 wb = {{0, 0, 0, 0, 0, 0}}, ws = {{0, 0, 0, 0, 0, 0}}, wn = {{0, 0, 0, 0, 0, 0}};
    for (int j = 0; j < 4; j++) { wb.w[j] = g.v[j]; ws.w[j] = one.v[j]; }
    hipLaunchKernelGGL(k_fft_tw_glv<Fr>, dim3(div_up(tw_cnt, 256)), dim3(256), 0, st, (int)tw_cnt, wb, ws, gp, twg);
    ZK_CHECK(hipGetLastError());
    uint64_t *twn = twg + tw_cnt * 8;
    if (inverse) {  // N^-1 folded into the first stage's scalars
      zkh::Fe<HR> nn = one;
      for (int k = 0; k < m; k++) zkh::add(nn, nn, nn);
      zkh::inv(ninv, nn);
      for (int j = 0; j < 4; j++) wn.w[j] = ninv.v[j];
      hipLaunchKernelGGL(k_fft_tw_glv<Fr>, dim3(div_up(tw_cnt, 256)), dim3(256), 0, st, (int)tw_cnt, wb, wn, gp, twn);
      ZK_CHECK(hipGetLastError());
    }
    uint32_t *in = A, *out = B;
    int done = 0;  // log2 L
    for (size_t i = 0; i < rbits.size(); i++) {
      const int b = rbits[i];
      const bool scaled = inverse && i == 0;
      const RadixPlan pl = make_radix_plan(b, scaled);
      const int lgG = m - done - b;
      const size_t np = (size_t)pl.D * (N >> b);
      size_t pl_lanes = std::min(2 * np, (size_t)1 << 17);
      pl_lanes = (pl_lanes + 255) & ~(size_t)255;
      hipLaunchKernelGGL(k_fft_radix_prod<C>, dim3((unsigned)(pl_lanes / 256)), dim3(256), 0, st, m, lgG, in, Pb,
                         scaled ? twn : twg, scaled ? 1 : 0, beta, scratch, (int)pl_lanes, pl);
      ZK_CHECK(hipGetLastError());
      const size_t slanes = N << (b < 2 ? b : 2);
      hipLaunchKernelGGL(k_fft_radix_sum<C>, dim3(div_up(slanes, 256)), dim3(256), 0, st, m, lgG, in, Pb, out, pl);
      ZK_CHECK(hipGetLastError());
      std::swap(in, out);
      done += b;
    }
    return in;
  };
  auto run_glv = [&] {
    // twiddles (decomposed): forward w^e; inverse (w^-1)^e with the 1/2 per level deferred to one
    // multiplication by N^-1 folded into the first stage (on the subgroup the m halvings = N^-1)
    zkh::Fe<HR> g, one, ninv;
    memcpy(g.v, gen, sizeof g.v);
    zkh::set_one(one);
    if (inverse) zkh::inv(g, g);
    W6 wb = {{0, 0, 0, 0, 0, 0}}, ws = {{0, 0, 0, 0, 0, 0}}, wn = {{0, 0, 0, 0, 0, 0}};
    for (int j = 0; j < 4; j++) { wb.w[j] = g.v[j]; ws.w[j] = one.v[j]; }
    hipLaunchKernelGGL(k_fft_tw_glv<Fr>, dim3(div_up(tw_cnt, 256)), dim3(256), 0, st, (int)tw_cnt, wb, ws, gp, twg);
    ZK_CHECK(hipGetLastError());
    const unsigned grid = (unsigned)(glanes / 256);
    uint32_t *in = A, *out = B;
    int k0 = 0;
    if (inverse) {  // first stage with N^-1 folded in: twn = (w^-1)^j N^-1, dkn = N^-1 (decomposed)
      zkh::Fe<HR> nn = one;
      for (int k = 0; k < m; k++) zkh::add(nn, nn, nn);
      zkh::inv(ninv, nn);
      for (int j = 0; j < 4; j++) wn.w[j] = ninv.v[j];
      uint64_t *twn = twg + tw_cnt * 8, *dkn = twg + 2 * tw_cnt * 8;
      hipLaunchKernelGGL(k_fft_tw_glv<Fr>, dim3(div_up(tw_cnt, 256)), dim3(256), 0, st, (int)tw_cnt, wb, wn, gp, twn);
      ZK_CHECK(hipGetLastError());
      hipLaunchKernelGGL(k_fft_tw_glv<Fr>, dim3(1), dim3(256), 0, st, 1, wb, wn, gp, dkn);
      ZK_CHECK(hipGetLastError());
      hipLaunchKernelGGL(k_fft_inv_first_glv<C>, dim3(grid), dim3(256), 0, st, m, in, out, twn, dkn, beta, scratch,
                         (int)glanes);
      ZK_CHECK(hipGetLastError());
      std::swap(in, out);
      k0 = 1;
    }
    for (int k = k0; k < m; k++) {
      const int s = inverse ? m - k : k + 1;
      if (inverse)
        hipLaunchKernelGGL(k_fft_inv_stage_glv<C>, dim3(grid), dim3(256), 0, st, m, s, in, out, twg, beta, scratch,
                           (int)glanes);
      else
        hipLaunchKernelGGL(k_fft_fwd_stage_glv<C>, dim3(grid), dim3(256), 0, st, m, s, in, out, twg, beta, scratch,
                           (int)glanes);
      ZK_CHECK(hipGetLastError());
      std::swap(in, out);
    }
    return in;
  };
  auto run_int = [&] {
    // twiddles: forward w^e; inverse (w^-1)^e / 2 -- the reference's gpow sequences
    // (G1_proj.c:705-711, 758-764), canonical Fr, standard form
    zkh::Fe<HR> g, scale;
    memcpy(g.v, gen, sizeof g.v);
    zkh::set_one(scale);
    if (inverse) {
      zkh::inv(g, g);
      zkh::Fe<HR> two;
      zkh::add(two, scale, scale);
      zkh::inv(scale, two);  // Montgomery(1/2) = the reference's oneHalf (G1_proj.c:727)
    }
    W6 wb = {{0, 0, 0, 0, 0, 0}}, ws = {{0, 0, 0, 0, 0, 0}};
    for (int j = 0; j < 4; j++) { wb.w[j] = g.v[j]; ws.w[j] = scale.v[j]; }
    hipLaunchKernelGGL(k_fft_tw<Fr>, dim3(div_up(tw_cnt, 256)), dim3(256), 0, st, (int)tw_cnt, wb, ws, tw);
    ZK_CHECK(hipGetLastError());
    const unsigned grid = (unsigned)(lanes / 256);
    uint32_t *in = A, *out = B;
    for (int k = 0; k < m; k++) {
      const int s = inverse ? m - k : k + 1;
      if (inverse)
        hipLaunchKernelGGL(k_fft_inv_stage<C>, dim3(grid), dim3(256), 0, st, m, s, in, out, tw, scratch, (int)lanes);
      else
        hipLaunchKernelGGL(k_fft_fwd_stage<C>, dim3(grid), dim3(256), 0, st, m, s, in, out, tw, scratch, (int)lanes);
      ZK_CHECK(hipGetLastError());
      std::swap(in, out);
    }
    return in;
  };
  bool out_natural = false;
  if (glv) {
    uint32_t *res = use_radix ? run_radix() : run_glv();
    if (hb) {  // the speculative membership test's verdict
      const hipEvent_t checked = dev.split_event(1);
      for (;;) {
        const hipError_t e = hipEventQuery(checked);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) ZK_CHECK(e);
        std::this_thread::yield();
      }
      for (unsigned i = 0; i < cgrid; i++) glv = glv && hb[i] == 0;
    }
    if (glv) {
      A = res;
      out_natural = use_radix;
    } else {  // some point lies outside the r-subgroup: the reference's exact integer schedule
      ZK_CHECK(hipStreamSynchronize(st));
      load_points(false);
      A = run_int();
    }
  } else if (m > 0) {
    A = run_int();
  }
  g1_fft_last_glv().store(glv ? 1 : 0);
  const int chk = norm_chk(N);
  launch_norm<C, MODE_XYZZ_TO_PROJ>(st, (int)N, chk, A, nscratch, dt, exp_p_minus_2<HF>(),
                                    (inverse && !out_natural) ? m : 0);
  ZK_CHECK(hipGetLastError());
  if (host_io) copy_to_host(dev, st, tgt, dt, N * 3 * NP * 8);  // fresh caller arrays: zk_runtime.hpp
  ZK_CHECK(hipStreamSynchronize(st));
}

// ---------------------------------------------------------------------------- public

void g1_batch_from_affine(int curve, int n, const uint64_t *src, uint64_t *tgt, bool host_io, bool jac) {
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  if (curve == 0) batch_from_affine_t<BN254>(dev, n, src, tgt, host_io, jac);
  else batch_from_affine_t<BLS381>(dev, n, src, tgt, host_io, jac);
}
void g1_batch_to_affine(int curve, int n, const uint64_t *src, uint64_t *tgt, bool host_io, bool jac) {
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  if (curve == 0) batch_to_affine_t<BN254>(dev, n, src, tgt, host_io, jac);
  else batch_to_affine_t<BLS381>(dev, n, src, tgt, host_io, jac);
}
int g1_fft_plan(int curve, int m, int *bits, int cap) {
  if (m <= 0) return 0;
  const std::vector<int> v = radix_plan(m, curve == 0 ? fft_waves<BN254>() : fft_waves<BLS381>());
  for (int i = 0; i < (int)v.size() && i < cap; i++) bits[i] = v[i];
  return (int)v.size();
}
int g1_fft_radix_products(int b) { return b >= 1 && b <= 4 ? radix_products(b) : 0; }
void g1_fft(int curve, int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt, bool host_io, bool inverse,
            bool jac) {
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  if (curve == 0) g1_fft_t<BN254>(dev, m, gen, src, tgt, host_io, inverse, jac);
  else g1_fft_t<BLS381>(dev, m, gen, src, tgt, host_io, inverse, jac);
}

}  // namespace zk
