// zk_host.hpp -- host-side (CPU) Montgomery arithmetic and G1 point ops.
//
// Product code, NOT the oracle: the library uses it for what is cheaper on one CPU
// core than on a GPU lane-chain -- the final Horner combine of per-window bucket
// sums (reference: the window loop, bls12_381_G1_proj.c:577-583), the affine /
// normalised outputs (bls12_381_G1_proj.c:79-98, 133-145), twiddle seeds and the
// deterministic synthetic-input generator.  Same Montgomery representation as the
// reference (64-bit limbs, R = 2^(64*n64)); canonical outputs throughout.
#pragma once
#include <stdint.h>
#include <string.h>
#include "zk_params.inc"
#include "zk_host_adx.inc"
#if defined(__x86_64__)
#include <cpuid.h>
#endif

namespace zkh {

typedef unsigned __int128 u128;

#define ZKH_DEFINE_FIELD(NAME, PFX)                                                   \
  struct NAME {                                                                       \
    static constexpr int N = PFX##_N64;                                               \
    static constexpr int BITS = PFX##_BITS;                                           \
    static constexpr uint64_t MINV = PFX##_MINV64;                                    \
    static constexpr uint64_t P[N] = PFX##_P64;                                       \
    static constexpr uint64_t ONE[N] = PFX##_R64;                                     \
    static constexpr uint64_t R2[N] = PFX##_R2_64;                                    \
  };

ZKH_DEFINE_FIELD(BN_Fp, ZK_BN128_FP)
ZKH_DEFINE_FIELD(BN_Fr, ZK_BN128_FR)
ZKH_DEFINE_FIELD(BLS_Fp, ZK_BLS12_381_FP)
ZKH_DEFINE_FIELD(BLS_Fr, ZK_BLS12_381_FR)

template <class F>
struct Fe {
  uint64_t v[F::N];
};

template <class F> inline void set_zero(Fe<F> &r) { memset(r.v, 0, sizeof r.v); }
template <class F> inline void set_one(Fe<F> &r) { memcpy(r.v, F::ONE, sizeof r.v); }
template <class F> inline bool is_zero(const Fe<F> &a) {
  uint64_t acc = 0;
  for (int i = 0; i < F::N; i++) acc |= a.v[i];
  return acc == 0;
}
template <class F> inline bool eq(const Fe<F> &a, const Fe<F> &b) {
  return memcmp(a.v, b.v, sizeof a.v) == 0;
}
template <class F> inline bool is_one(const Fe<F> &a) { return memcmp(a.v, F::ONE, sizeof a.v) == 0; }

// x >= p ?
template <class F> inline bool geq_p(const uint64_t *x) {
  for (int i = F::N - 1; i >= 0; i--) {
    if (x[i] != F::P[i]) return x[i] > F::P[i];
  }
  return true;
}
template <class F> inline void sub_p(uint64_t *x) {
  uint64_t br = 0;
  for (int i = 0; i < F::N; i++) {
    u128 d = (u128)x[i] - F::P[i] - br;
    x[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}
// Branch-free modular add / sub (the chain of doublings in finish_host is latency-bound; a
// data-dependent compare-and-subtract branch mispredicts on random values).  p has a spare top
// bit, so a + b < 2p never carries out.
template <class F> inline void add(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  constexpr int N = F::N;
  uint64_t s[N], d[N], c = 0, br = 0;
  for (int i = 0; i < N; i++) {
    const u128 x = (u128)a.v[i] + b.v[i] + c;
    s[i] = (uint64_t)x;
    c = (uint64_t)(x >> 64);
  }
  for (int i = 0; i < N; i++) {
    const u128 y = (u128)s[i] - F::P[i] - br;
    d[i] = (uint64_t)y;
    br = (uint64_t)(y >> 64) & 1;
  }
  const uint64_t keep = 0 - br;  // all ones: s < p, keep s
  for (int i = 0; i < N; i++) r.v[i] = (s[i] & keep) | (d[i] & ~keep);
}
template <class F> inline void sub(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  constexpr int N = F::N;
  uint64_t d[N], br = 0, c = 0;
  for (int i = 0; i < N; i++) {
    const u128 x = (u128)a.v[i] - b.v[i] - br;
    d[i] = (uint64_t)x;
    br = (uint64_t)(x >> 64) & 1;
  }
  const uint64_t mask = 0 - br;  // a < b: add p back
  for (int i = 0; i < N; i++) {
    const u128 y = (u128)d[i] + (F::P[i] & mask) + c;
    r.v[i] = (uint64_t)y;
    c = (uint64_t)(y >> 64);
  }
}
// t (N words, value < 2p, plus a carry word `hi` in {0, 1}) -> canonical, branch-free
template <class F> inline void reduce_once(uint64_t *r, const uint64_t *t, uint64_t hi) {
  constexpr int N = F::N;
  uint64_t d[N], br = 0;
  for (int i = 0; i < N; i++) {
    const u128 y = (u128)t[i] - F::P[i] - br;
    d[i] = (uint64_t)y;
    br = (uint64_t)(y >> 64) & 1;
  }
  const uint64_t keep = 0 - (br & (hi ^ 1));  // t < p and no carry word: keep t
  for (int i = 0; i < N; i++) r[i] = (t[i] & keep) | (d[i] & ~keep);
}
template <class F> inline void neg(Fe<F> &r, const Fe<F> &a) {
  Fe<F> z;
  set_zero(z);
  sub(r, z, a);
}
// ADX + BMI2 on this CPU (CPUID leaf 7: EBX bits 19 and 8), checked once
inline bool cpu_has_adx() {
#if defined(__x86_64__)
  static const bool v = [] {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
    return (b & (1u << 19)) != 0 && (b & (1u << 8)) != 0;
  }();
  return v;
#else
  return false;
#endif
}
// Montgomery product (CIOS, 64-bit limbs), fully unrolled so t stays in registers; p's top
// word leaves a spare bit, so t < 2p fits N + 1 words and the extra carry word is at most 1
template <class F> inline void mul_cios(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  constexpr int N = F::N;
  uint64_t t[N + 2] = {0};
#pragma clang loop unroll(full)
  for (int i = 0; i < N; i++) {
    uint64_t c = 0;
#pragma clang loop unroll(full)
    for (int j = 0; j < N; j++) {
      const u128 x = (u128)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    u128 s = (u128)t[N] + c;
    t[N] = (uint64_t)s;
    t[N + 1] = (uint64_t)(s >> 64);
    const uint64_t m = t[0] * F::MINV;
    u128 x = (u128)m * F::P[0] + t[0];
    c = (uint64_t)(x >> 64);
#pragma clang loop unroll(full)
    for (int j = 1; j < N; j++) {
      x = (u128)m * F::P[j] + t[j] + c;
      t[j - 1] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    s = (u128)t[N] + c;
    t[N - 1] = (uint64_t)s;
    t[N] = t[N + 1] + (uint64_t)(s >> 64);
  }
  reduce_once<F>(r.v, t, t[N]);
}
// Montgomery square (SOS): the 2N-word square with every cross product once, doubled,
// then N reduction rows -- N(N+1)/2 + N^2 word products instead of 2N^2
template <class F> inline void sqr_sos(Fe<F> &r, const Fe<F> &a) {
  constexpr int N = F::N;
  uint64_t t[2 * N + 1] = {0};
#pragma clang loop unroll(full)
  for (int i = 0; i < N; i++) {
    uint64_t c = 0;
#pragma clang loop unroll(full)
    for (int j = i + 1; j < N; j++) {
      const u128 x = (u128)a.v[i] * a.v[j] + t[i + j] + c;
      t[i + j] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    t[i + N] = c;
  }
  uint64_t top2 = 0;
#pragma clang loop unroll(full)
  for (int k = 0; k < 2 * N; k++) {  // double the cross products
    const uint64_t nt = t[k] >> 63;
    t[k] = (t[k] << 1) | top2;
    top2 = nt;
  }
  uint64_t c = 0;
#pragma clang loop unroll(full)
  for (int i = 0; i < N; i++) {  // diagonal
    const u128 x = (u128)a.v[i] * a.v[i] + t[2 * i] + c;
    t[2 * i] = (uint64_t)x;
    const u128 y = (u128)t[2 * i + 1] + (uint64_t)(x >> 64);
    t[2 * i + 1] = (uint64_t)y;
    c = (uint64_t)(y >> 64);
  }
  t[2 * N] = c;
  uint64_t top = 0;  // carry out of the previous row into t[i + N]
#pragma clang loop unroll(full)
  for (int i = 0; i < N; i++) {  // Montgomery reduction rows
    const uint64_t m = t[i] * F::MINV;
    uint64_t cc = 0;
#pragma clang loop unroll(full)
    for (int j = 0; j < N; j++) {
      const u128 x = (u128)m * F::P[j] + t[i + j] + cc;
      t[i + j] = (uint64_t)x;
      cc = (uint64_t)(x >> 64);
    }
    const u128 y = (u128)t[i + N] + cc + top;
    t[i + N] = (uint64_t)y;
    top = (uint64_t)(y >> 64);
  }
  t[2 * N] += top;
  reduce_once<F>(r.v, t + N, t[2 * N]);
}

// the MULX / ADCX / ADOX product (zk_host_adx.inc) when the CPU has it, else the portable CIOS
template <class F> inline void mul_adx(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  static_assert(F::N == 4 || F::N == 6, "ADX products are generated for 4 and 6 words");
  uint64_t t[F::N];
  if constexpr (F::N == 6) mont_mul_adx_6(t, a.v, b.v, F::P, F::MINV);
  else mont_mul_adx_4(t, a.v, b.v, F::P, F::MINV);
  reduce_once<F>(r.v, t, 0);  // < 2p -> canonical
}
template <class F> inline void mul(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  if constexpr (F::N == 4 || F::N == 6) {
    if (cpu_has_adx()) return mul_adx(r, a, b);
  }
  mul_cios(r, a, b);
}
template <class F> inline void sqr(Fe<F> &r, const Fe<F> &a) {
  if constexpr (F::N == 4 || F::N == 6) {
    if (cpu_has_adx()) return mul_adx(r, a, a);  // faster than the portable squaring
  }
  sqr_sos(r, a);
}

// standard <-> Montgomery
template <class F> inline void to_mont(Fe<F> &r, const Fe<F> &a) {
  Fe<F> r2;
  memcpy(r2.v, F::R2, sizeof r2.v);
  mul(r, a, r2);
}
template <class F> inline void from_mont(Fe<F> &r, const Fe<F> &a) {
  Fe<F> one;
  set_zero(one);
  one.v[0] = 1;
  mul(r, a, one);
}

// a^e for a little-endian exponent of `ne` words (Montgomery in, Montgomery out)
template <class F> inline void pow(Fe<F> &r, const Fe<F> &a, const uint64_t *e, int ne) {
  Fe<F> acc, base = a;
  set_one(acc);
  for (int i = 0; i < ne; i++) {
    uint64_t w = e[i];
    for (int b = 0; b < 64; b++) {
      if (w & 1) mul(acc, acc, base);
      sqr(base, base);
      w >>= 1;
    }
  }
  r = acc;
}
// inverse via Fermat (a^(p-2)); 0 -> 0 like the reference (Fr_std.c:298-301)
template <class F> inline void inv(Fe<F> &r, const Fe<F> &a) {
  if (is_zero(a)) { set_zero(r); return; }
  uint64_t e[F::N];
  memcpy(e, F::P, sizeof e);
  // p - 2 (p odd, p > 2: no borrow past limb 0 unless P[0] < 2)
  uint64_t br = 2;
  for (int i = 0; i < F::N && br; i++) {
    uint64_t o = e[i];
    e[i] = o - br;
    br = (o < br) ? 1 : 0;
  }
  pow(r, a, e, F::N);
}

// ---------------------------------------------------------------------------
// Fp2 = Fp[u]/(u^2 + 1) (both curves; <C>_Fp2_mont.c:183-215): an element is c0 || c1,
// N64 limbs each, exactly the reference layout.  Overloads below are picked over the
// generic templates by partial ordering, so Proj / Xyzz code instantiates on Fp2.
template <class B>
struct HF2 {
  using Base = B;
  static constexpr int N = 2 * B::N;
};
template <class B> inline void f2s(Fe<B> &c0, Fe<B> &c1, const Fe<HF2<B>> &a) {
  memcpy(c0.v, a.v, sizeof c0.v);
  memcpy(c1.v, a.v + B::N, sizeof c1.v);
}
template <class B> inline void f2j(Fe<HF2<B>> &r, const Fe<B> &c0, const Fe<B> &c1) {
  memcpy(r.v, c0.v, sizeof c0.v);
  memcpy(r.v + B::N, c1.v, sizeof c1.v);
}
template <class B> inline void set_one(Fe<HF2<B>> &r) {
  Fe<B> o, z;
  set_one(o);
  set_zero(z);
  f2j(r, o, z);
}
template <class B> inline bool is_one(const Fe<HF2<B>> &a) {
  Fe<B> a0, a1;
  f2s(a0, a1, a);
  return is_one(a0) && is_zero(a1);
}
template <class B> inline void add(Fe<HF2<B>> &r, const Fe<HF2<B>> &a, const Fe<HF2<B>> &b) {
  Fe<B> a0, a1, b0, b1;
  f2s(a0, a1, a);
  f2s(b0, b1, b);
  add(a0, a0, b0);
  add(a1, a1, b1);
  f2j(r, a0, a1);
}
template <class B> inline void sub(Fe<HF2<B>> &r, const Fe<HF2<B>> &a, const Fe<HF2<B>> &b) {
  Fe<B> a0, a1, b0, b1;
  f2s(a0, a1, a);
  f2s(b0, b1, b);
  sub(a0, a0, b0);
  sub(a1, a1, b1);
  f2j(r, a0, a1);
}
template <class B> inline void neg(Fe<HF2<B>> &r, const Fe<HF2<B>> &a) {
  Fe<HF2<B>> z;
  set_zero(z);
  sub(r, z, a);
}
template <class B> inline void mul(Fe<HF2<B>> &r, const Fe<HF2<B>> &a, const Fe<HF2<B>> &b) {
  Fe<B> a0, a1, b0, b1, t0, t1, s, u;
  f2s(a0, a1, a);
  f2s(b0, b1, b);
  mul(t0, a0, b0);
  mul(t1, a1, b1);
  add(s, a0, a1);
  add(u, b0, b1);
  mul(s, s, u);
  sub(s, s, t0);
  sub(s, s, t1);
  sub(t0, t0, t1);
  f2j(r, t0, s);
}
template <class B> inline void sqr(Fe<HF2<B>> &r, const Fe<HF2<B>> &a) { mul(r, a, a); }
// 1/(a0 + a1 u) = (a0 - a1 u) / (a0^2 + a1^2); 0 -> 0
template <class B> inline void inv(Fe<HF2<B>> &r, const Fe<HF2<B>> &a) {
  Fe<B> a0, a1, n, t;
  f2s(a0, a1, a);
  mul(n, a0, a0);
  mul(t, a1, a1);
  add(n, n, t);
  inv(n, n);
  mul(a0, a0, n);
  mul(a1, a1, n);
  neg(a1, a1);
  f2j(r, a0, a1);
}

// ---------------------------------------------------------------------------
// G1 in homogeneous projective coordinates (x = X/Z, y = Y/Z), a = 0.
// Infinity: Z == 0 (canonical form (0 : 1 : 0), reference set_infinity
// bls12_381_G1_proj.c:179-183).  Affine infinity: all-0xFF bytes (G1_affine.c:1-6).

template <class F>
struct Proj {
  Fe<F> X, Y, Z;
};
template <class F>
struct Aff {
  Fe<F> x, y;
};

template <class F> inline void proj_set_inf(Proj<F> &r) {
  set_zero(r.X);
  set_one(r.Y);
  set_zero(r.Z);
}
template <class F> inline bool proj_is_inf(const Proj<F> &a) { return is_zero(a.Z); }
template <class F> inline bool aff_is_inf(const Aff<F> &a) {
  for (int i = 0; i < F::N; i++)
    if (a.x.v[i] != ~0ull || a.y.v[i] != ~0ull) return false;
  return true;
}
template <class F> inline void aff_set_inf(Aff<F> &a) { memset(&a, 0xff, sizeof a); }

template <class F> inline void proj_from_aff(Proj<F> &r, const Aff<F> &a) {
  if (aff_is_inf(a)) { proj_set_inf(r); return; }
  r.X = a.x;
  r.Y = a.y;
  set_one(r.Z);
}

// complete addition for a = 0 (Renes-Costello-Batina 2015, alg. 7); b3 = 3*B (Montgomery)
template <class F> inline void proj_add(Proj<F> &r, const Proj<F> &P, const Proj<F> &Q, const Fe<F> &b3) {
  Fe<F> t0, t1, t2, t3, t4, X3, Y3, Z3;
  mul(t0, P.X, Q.X);
  mul(t1, P.Y, Q.Y);
  mul(t2, P.Z, Q.Z);
  add(t3, P.X, P.Y);
  add(t4, Q.X, Q.Y);
  mul(t3, t3, t4);
  add(t4, t0, t1);
  sub(t3, t3, t4);
  add(t4, P.Y, P.Z);
  add(X3, Q.Y, Q.Z);
  mul(t4, t4, X3);
  add(X3, t1, t2);
  sub(t4, t4, X3);
  add(X3, P.X, P.Z);
  add(Y3, Q.X, Q.Z);
  mul(X3, X3, Y3);
  add(Y3, t0, t2);
  sub(Y3, X3, Y3);
  add(X3, t0, t0);
  add(t0, X3, t0);
  mul(t2, b3, t2);
  add(Z3, t1, t2);
  sub(t1, t1, t2);
  mul(Y3, b3, Y3);
  mul(X3, t4, Y3);
  mul(t2, t3, t1);
  sub(X3, t2, X3);
  mul(Y3, Y3, t0);
  mul(t1, t1, Z3);
  add(Y3, t1, Y3);
  mul(t0, t0, t3);
  mul(Z3, Z3, t4);
  add(Z3, Z3, t0);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}
template <class F> inline void proj_dbl(Proj<F> &r, const Proj<F> &P, const Fe<F> &b3) {
  proj_add(r, P, P, b3);  // the complete formula doubles correctly
}

template <class F> inline void proj_to_aff(Aff<F> &r, const Proj<F> &P) {
  if (is_zero(P.Z)) { aff_set_inf(r); return; }
  Fe<F> zi;
  inv(zi, P.Z);
  mul(r.x, P.X, zi);
  mul(r.y, P.Y, zi);
}
// canonical projective form: Z = 1, or (0 : 1 : 0) for infinity (reference normalize,
// bls12_381_G1_proj.c:79-98)
template <class F> inline void proj_normalize(Proj<F> &r, const Proj<F> &P) {
  if (is_zero(P.Z)) { proj_set_inf(r); return; }
  if (is_one(P.Z)) { r = P; return; }
  Fe<F> zi;
  inv(zi, P.Z);
  mul(r.X, P.X, zi);
  mul(r.Y, P.Y, zi);
  set_one(r.Z);
}

// k * P for a little-endian multi-word integer k (double-and-add, MSB first)
template <class F> inline void proj_scale(Proj<F> &r, const Proj<F> &P, const uint64_t *k, int nk,
                                          const Fe<F> &b3) {
  Proj<F> acc;
  proj_set_inf(acc);
  for (int i = nk - 1; i >= 0; i--) {
    for (int b = 63; b >= 0; b--) {
      proj_dbl(acc, acc, b3);
      if ((k[i] >> b) & 1) proj_add(acc, acc, P, b3);
    }
  }
  r = acc;
}

// ---------------------------------------------------------------------------
// G1 in extended Jacobian "XYZZ" coordinates (x = X/ZZ, y = Y/ZZZ), a = 0 -- the
// form the device bucket sums arrive in; used for the host Horner combine.
// Infinity: ZZ == 0.  Curves here have no 2-torsion (odd group order), so Y != 0
// for every finite point.
template <class F>
struct Xyzz {
  Fe<F> X, Y, ZZ, ZZZ;
};
template <class F> inline void xyzz_set_inf(Xyzz<F> &r) {
  set_one(r.X);
  set_one(r.Y);
  set_zero(r.ZZ);
  set_zero(r.ZZZ);
}
template <class F> inline bool xyzz_is_inf(const Xyzz<F> &a) { return is_zero(a.ZZ); }
// r = 2p (dbl-2008-s-1): 6M + 3S
template <class F> inline void xyzz_dbl(Xyzz<F> &r, const Xyzz<F> &p) {
  if (xyzz_is_inf(p)) { r = p; return; }
  Fe<F> U, V, W, S, M, t, X3;
  add(U, p.Y, p.Y);
  sqr(V, U);
  mul(W, U, V);
  mul(S, p.X, V);
  sqr(t, p.X);
  add(M, t, t);
  add(M, M, t);
  sqr(t, M);
  sub(t, t, S);
  sub(X3, t, S);
  sub(t, S, X3);
  mul(t, M, t);
  mul(U, W, p.Y);
  sub(r.Y, t, U);
  r.X = X3;
  mul(r.ZZ, V, p.ZZ);
  mul(r.ZZZ, W, p.ZZZ);
}
// r = a + b (add-2008-s), all special cases
template <class F> inline void xyzz_add(Xyzz<F> &r, const Xyzz<F> &a, const Xyzz<F> &b) {
  if (xyzz_is_inf(b)) { r = a; return; }
  if (xyzz_is_inf(a)) { r = b; return; }
  Fe<F> U1, U2, S1, S2, P, R;
  mul(U1, a.X, b.ZZ);
  mul(U2, b.X, a.ZZ);
  mul(S1, a.Y, b.ZZZ);
  mul(S2, b.Y, a.ZZZ);
  sub(P, U2, U1);
  sub(R, S2, S1);
  if (is_zero(P)) {
    if (is_zero(R)) xyzz_dbl(r, a);
    else xyzz_set_inf(r);
    return;
  }
  Fe<F> PP, PPP, Q, t, X3;
  sqr(PP, P);
  mul(PPP, P, PP);
  mul(Q, U1, PP);
  sqr(t, R);
  sub(t, t, PPP);
  sub(t, t, Q);
  sub(X3, t, Q);
  sub(t, Q, X3);
  mul(t, R, t);
  mul(S1, S1, PPP);
  sub(r.Y, t, S1);
  r.X = X3;
  mul(t, a.ZZ, b.ZZ);
  mul(r.ZZ, t, PP);
  mul(t, a.ZZZ, b.ZZZ);
  mul(r.ZZZ, t, PPP);
}
// Jacobian (x = X/Z^2, y = Y/Z^3; infinity Z == 0), a = 0: the host Horner chain's
// doublings cost 2M + 5S here against 6M + 3S in XYZZ
template <class F>
struct Jac {
  Fe<F> X, Y, Z;
};
template <class F> inline bool jac_is_inf(const Jac<F> &a) { return is_zero(a.Z); }
template <class F> inline void jac_set_inf(Jac<F> &r) {
  set_one(r.X);
  set_one(r.Y);
  set_zero(r.Z);
}
// dbl-2009-l
template <class F> inline void jac_dbl(Jac<F> &r, const Jac<F> &p) {
  if (jac_is_inf(p)) { r = p; return; }
  Fe<F> A, B, C, D, E, Fv, t;
  sqr(A, p.X);
  sqr(B, p.Y);
  sqr(C, B);
  add(t, p.X, B);
  sqr(t, t);
  sub(t, t, A);
  sub(t, t, C);
  add(D, t, t);
  add(E, A, A);
  add(E, E, A);
  sqr(Fv, E);
  Fe<F> X3, Z3;
  sub(X3, Fv, D);
  sub(X3, X3, D);
  mul(Z3, p.Y, p.Z);
  add(r.Z, Z3, Z3);
  sub(t, D, X3);
  mul(t, E, t);
  add(C, C, C);
  add(C, C, C);
  add(C, C, C);
  sub(r.Y, t, C);
  r.X = X3;
}
// add-2007-bl, all special cases
template <class F> inline void jac_add(Jac<F> &r, const Jac<F> &a, const Jac<F> &b) {
  if (jac_is_inf(b)) { r = a; return; }
  if (jac_is_inf(a)) { r = b; return; }
  Fe<F> Z1Z1, Z2Z2, U1, U2, S1, S2, t;
  sqr(Z1Z1, a.Z);
  sqr(Z2Z2, b.Z);
  mul(U1, a.X, Z2Z2);
  mul(U2, b.X, Z1Z1);
  mul(t, b.Z, Z2Z2);
  mul(S1, a.Y, t);
  mul(t, a.Z, Z1Z1);
  mul(S2, b.Y, t);
  Fe<F> H, R;
  sub(H, U2, U1);
  sub(R, S2, S1);
  if (is_zero(H)) {
    if (is_zero(R)) jac_dbl(r, a);
    else jac_set_inf(r);
    return;
  }
  add(R, R, R);
  Fe<F> I, J, V, X3;
  add(I, H, H);
  sqr(I, I);
  mul(J, H, I);
  mul(V, U1, I);
  sqr(X3, R);
  sub(X3, X3, J);
  sub(X3, X3, V);
  sub(X3, X3, V);
  sub(t, V, X3);
  mul(t, R, t);
  mul(S1, S1, J);
  add(S1, S1, S1);
  Fe<F> Z3;
  add(Z3, a.Z, b.Z);
  sqr(Z3, Z3);
  sub(Z3, Z3, Z1Z1);
  sub(Z3, Z3, Z2Z2);
  mul(r.Z, Z3, H);
  sub(r.Y, t, S1);
  r.X = X3;
}
// XYZZ -> Jacobian with Z = ZZ ZZZ: X ZZ ZZZ^2, Y ZZ^3 ZZZ^2
template <class F> inline void xyzz_to_jac(Jac<F> &r, const Xyzz<F> &a) {
  if (xyzz_is_inf(a)) { jac_set_inf(r); return; }
  Fe<F> z3s, t, u;
  sqr(z3s, a.ZZZ);
  mul(t, a.ZZ, z3s);   // ZZ ZZZ^2
  mul(r.X, a.X, t);
  sqr(u, a.ZZ);
  mul(u, u, t);        // ZZ^3 ZZZ^2
  mul(r.Y, a.Y, u);
  mul(r.Z, a.ZZ, a.ZZZ);
}
template <class F> inline void jac_to_xyzz(Xyzz<F> &r, const Jac<F> &a) {
  if (jac_is_inf(a)) { xyzz_set_inf(r); return; }
  r.X = a.X;
  r.Y = a.Y;
  sqr(r.ZZ, a.Z);
  mul(r.ZZZ, r.ZZ, a.Z);
}

// -> homogeneous projective (X ZZZ : Y ZZ : ZZ ZZZ)
template <class F> inline void xyzz_to_proj(Proj<F> &r, const Xyzz<F> &a) {
  if (xyzz_is_inf(a)) { proj_set_inf(r); return; }
  mul(r.X, a.X, a.ZZZ);
  mul(r.Y, a.Y, a.ZZ);
  mul(r.Z, a.ZZ, a.ZZZ);
}

}  // namespace zkh
