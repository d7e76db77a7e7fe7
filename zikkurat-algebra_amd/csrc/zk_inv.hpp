// zk_inv.hpp -- modular inversion by Bernstein-Yang divsteps ("safegcd"), constant iteration count,
// host and device (the same code is checked on the CPU by tests/native/test_safegcd.cpp).
//
// Replaces the Fermat inversions (x^(p-2): 489 dependent 381-bit products, 323 for the scalar field)
// in the batch conversions, the group FFT's normalisation and the Fr batch inversion -- the role of
// the reference's binary extended Euclid `*_std_inv` (bls12_381_Fr_std.c:251-315, called by its
// Montgomery `inv`) -- with ~2d divsteps on 64-bit words in batches of 62 and one 2x2-matrix
// update of the full-size values per batch: d = 381 bits -> 18 batches, 254/255 -> 12
// (ceil((49 d + 57) / 17) divsteps, the Bernstein-Yang bound for d >= 46; ZK_<F>_S62_BATCHES).
//
// Numbers: L signed 62-bit limbs (value = sum l_i 2^(62 i)), l_0 .. l_(L-2) in [0, 2^62), the top
// limb signed.  The invariants f = d x, g = e x (mod p) hold throughout; at the end g = 0 and
// f = +-1, so x^-1 = +-d.  |d|, |e| grow by at most p per batch (|d'| <= max(|d|, |e|) + p), so
// they stay below (NB + 1) p < 32 p and one normalisation at the end brings d into [0, p).
// Branch-free: every lane runs the same instruction stream (no divergence inside a wavefront).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define ZK_HD __host__ __device__ __forceinline__
#else
#define ZK_HD inline
#endif

namespace zk {

constexpr int64_t S62_MASK = (int64_t)((1ull << 62) - 1);
template <int B>
constexpr int64_t sg_mask() { return (int64_t)((1ull << B) - 1); }

// 62 divsteps on the low 64 bits of f (odd) and g; t = (u, v, q, r) with 2^62 (f', g') = (u f + v g,
// q f + r g).  delta starts at 1.
ZK_HD int64_t sg_divsteps62(int64_t delta, uint64_t f, uint64_t g, int64_t t[4]) {
  int64_t u = 1, v = 0, q = 0, r = 1;
  for (int i = 0; i < 62; i++) {
    // swap when delta > 0 and g odd: (f, g) <- (g, -f), (u, v) <- (q, r), (q, r) <- (-u, -v), delta <- -delta
    const int64_t sw = -(int64_t)((delta > 0) & (int64_t)(g & 1));
    const uint64_t usw = (uint64_t)sw;
    const uint64_t nf = (f & ~usw) | (g & usw);
    const uint64_t ng = (g & ~usw) | ((0 - f) & usw);
    const int64_t nu = (u & ~sw) | (q & sw), nv = (v & ~sw) | (r & sw);
    const int64_t nq = (q & ~sw) | ((0 - u) & sw), nr = (r & ~sw) | ((0 - v) & sw);
    delta = (delta ^ sw) - sw;
    // g odd: g += f, (q, r) += (u, v); then g /= 2, (u, v) *= 2, delta += 1
    const int64_t od = -(int64_t)(ng & 1);
    g = (uint64_t)((int64_t)(ng + (nf & (uint64_t)od)) >> 1);
    q = nq + (nu & od);
    r = nr + (nv & od);
    f = nf;
    u = nu * 2;
    v = nv * 2;
    delta += 1;
  }
  t[0] = u;
  t[1] = v;
  t[2] = q;
  t[3] = r;
  return delta;
}

// 30 divsteps on the low 32 bits of f (odd) and g, in 32-bit arithmetic (|u|, |v|, |q|, |r| <= 2^30
// after 30 steps): the same step as sg_divsteps62, each on one register instead of a pair
ZK_HD int32_t sg_divsteps30(int32_t delta, uint32_t f, uint32_t g, int32_t t[4]) {
  int32_t u = 1, v = 0, q = 0, r = 1;
  for (int i = 0; i < 30; i++) {
    const int32_t sw = -(int32_t)((delta > 0) & (int32_t)(g & 1));
    const uint32_t usw = (uint32_t)sw;
    const uint32_t nf = (f & ~usw) | (g & usw);
    const uint32_t ng = (g & ~usw) | ((0u - f) & usw);
    const int32_t nu = (u & ~sw) | (q & sw), nv = (v & ~sw) | (r & sw);
    const int32_t nq = (q & ~sw) | ((0 - u) & sw), nr = (r & ~sw) | ((0 - v) & sw);
    delta = (delta ^ sw) - sw;
    const int32_t od = -(int32_t)(ng & 1);
    g = (uint32_t)((int32_t)(ng + (nf & (uint32_t)od)) >> 1);
    q = nq + (nu & od);
    r = nr + (nv & od);
    f = nf;
    u = nu * 2;
    v = nv * 2;
    delta += 1;
  }
  t[0] = u;
  t[1] = v;
  t[2] = q;
  t[3] = r;
  return delta;
}
// 60 divsteps as two 30-step rounds: the first round's matrix applied to the low 64 bits of (f, g)
// gives the low 34 bits of (f, g) / 2^30 for the second; t = M2 M1 (entries <= 2^60)
ZK_HD int64_t sg_divsteps60(int64_t delta, uint64_t f, uint64_t g, int64_t t[4]) {
  int32_t a[4], b[4];
  int32_t d = sg_divsteps30((int32_t)delta, (uint32_t)f, (uint32_t)g, a);
  const uint64_t f1 = (uint64_t)((int64_t)((uint64_t)(int64_t)a[0] * f + (uint64_t)(int64_t)a[1] * g) >> 30);
  const uint64_t g1 = (uint64_t)((int64_t)((uint64_t)(int64_t)a[2] * f + (uint64_t)(int64_t)a[3] * g) >> 30);
  d = sg_divsteps30(d, (uint32_t)f1, (uint32_t)g1, b);
  t[0] = (int64_t)b[0] * a[0] + (int64_t)b[1] * a[2];
  t[1] = (int64_t)b[0] * a[1] + (int64_t)b[1] * a[3];
  t[2] = (int64_t)b[2] * a[0] + (int64_t)b[3] * a[2];
  t[3] = (int64_t)b[2] * a[1] + (int64_t)b[3] * a[3];
  return d;
}

// (f, g) <- (u f + v g, q f + r g) / 2^B (exact), B-bit limbs
template <int L, int B = 62>
ZK_HD void sg_update_fg(int64_t *f, int64_t *g, const int64_t t[4]) {
  __int128 cf = (__int128)t[0] * f[0] + (__int128)t[1] * g[0];
  __int128 cg = (__int128)t[2] * f[0] + (__int128)t[3] * g[0];
  cf >>= B;
  cg >>= B;
#pragma unroll
  for (int i = 1; i < L; i++) {
    cf += (__int128)t[0] * f[i] + (__int128)t[1] * g[i];
    cg += (__int128)t[2] * f[i] + (__int128)t[3] * g[i];
    f[i - 1] = (int64_t)cf & sg_mask<B>();
    g[i - 1] = (int64_t)cg & sg_mask<B>();
    cf >>= B;
    cg >>= B;
  }
  f[L - 1] = (int64_t)cf;
  g[L - 1] = (int64_t)cg;
}

// (d, e) <- (u d + v e + md p, q d + r e + me p) / 2^B, md / me chosen so the low B bits vanish
// (pinv = p^-1 mod 2^62, which is p^-1 mod 2^B as well)
template <int L, int B = 62>
ZK_HD void sg_update_de(int64_t *d, int64_t *e, const int64_t t[4], const int64_t *P, uint64_t pinv) {
  const uint64_t d0 = (uint64_t)d[0], e0 = (uint64_t)e[0];
  const uint64_t td = (uint64_t)t[0] * d0 + (uint64_t)t[1] * e0;  // mod 2^64
  const uint64_t te = (uint64_t)t[2] * d0 + (uint64_t)t[3] * e0;
  const int64_t md = (int64_t)((0 - td * pinv) & (uint64_t)sg_mask<B>());
  const int64_t me = (int64_t)((0 - te * pinv) & (uint64_t)sg_mask<B>());
  __int128 cd = (__int128)t[0] * d[0] + (__int128)t[1] * e[0] + (__int128)md * P[0];
  __int128 ce = (__int128)t[2] * d[0] + (__int128)t[3] * e[0] + (__int128)me * P[0];
  cd >>= B;
  ce >>= B;
#pragma unroll
  for (int i = 1; i < L; i++) {
    cd += (__int128)t[0] * d[i] + (__int128)t[1] * e[i] + (__int128)md * P[i];
    ce += (__int128)t[2] * d[i] + (__int128)t[3] * e[i] + (__int128)me * P[i];
    d[i - 1] = (int64_t)cd & sg_mask<B>();
    e[i - 1] = (int64_t)ce & sg_mask<B>();
    cd >>= B;
    ce >>= B;
  }
  d[L - 1] = (int64_t)cd;
  e[L - 1] = (int64_t)ce;
}

// d <- d + k P (k small, signed), limbs renormalised
template <int L, int B = 62>
ZK_HD void sg_add_mul(int64_t *d, const int64_t *P, int64_t k) {
  __int128 c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    c += (__int128)d[i] + (__int128)k * P[i];
    d[i] = (i < L - 1) ? ((int64_t)c & sg_mask<B>()) : (int64_t)c;
    c >>= B;
  }
}

// x^-1 mod p for 0 < x < p given as n64 little-endian u64 words; result as n64 words in [0, p).
// x = 0 gives 0.
// B = 62: batches of 62 divsteps in 64-bit arithmetic; B = 60 (round 6): batches of 2 x 30 divsteps
// in 32-bit arithmetic (sg_divsteps60, about half the instructions per divstep), 60-bit limbs
template <int L, int NB, int B = 62>
ZK_HD void sg_inverse_words(uint64_t *out, const uint64_t *in, int n64, const int64_t *P, uint64_t pinv) {
  static_assert(B == 62 || B == 60, "62-bit or 60-bit limbs");
  int64_t f[L], g[L], d[L], e[L];
#pragma unroll
  for (int i = 0; i < L; i++) {  // B-bit slices of the input
    const int bit = B * i, w = bit >> 6, o = bit & 63;
    uint64_t x = w < n64 ? in[w] >> o : 0;
    if (o > 64 - B && w + 1 < n64) x |= in[w + 1] << (64 - o);
    g[i] = (int64_t)(x & (uint64_t)sg_mask<B>());
    f[i] = P[i];
    d[i] = 0;
    e[i] = 0;
  }
  e[0] = 1;
  int64_t delta = 1;
#pragma unroll 1
  for (int b = 0; b < NB; b++) {
    int64_t t[4];
    const uint64_t f64 = (uint64_t)f[0] | ((uint64_t)f[1] << B), g64 = (uint64_t)g[0] | ((uint64_t)g[1] << B);
    if constexpr (B == 62) delta = sg_divsteps62(delta, f64, g64, t);
    else delta = sg_divsteps60(delta, f64, g64, t);
    sg_update_fg<L, B>(f, g, t);
    sg_update_de<L, B>(d, e, t, P, pinv);
  }
  // f = +-1 (0 when x = 0, then d = 0): x^-1 = sign(f) d; bring d from (-32p, 32p) into [0, p)
  const int64_t neg = f[L - 1] >> 63;  // -1 when f = -1
  {
    int64_t nd[L];
    __int128 c = 0;
#pragma unroll
    for (int i = 0; i < L; i++) {  // nd = -d, limbs renormalised
      c -= (__int128)d[i];
      nd[i] = (i < L - 1) ? ((int64_t)c & sg_mask<B>()) : (int64_t)c;
      c >>= B;
    }
#pragma unroll
    for (int i = 0; i < L; i++) d[i] = (nd[i] & neg) | (d[i] & ~neg);
  }
  sg_add_mul<L, B>(d, P, 32);  // now in [0, 64p)
#pragma unroll
  for (int s = 5; s >= 0; s--) {  // conditional subtraction ladder 32p, 16p, ..., p
    int64_t t[L];
#pragma unroll
    for (int i = 0; i < L; i++) t[i] = d[i];
    sg_add_mul<L, B>(t, P, -(int64_t)(1 << s));
    const int64_t keep = t[L - 1] >> 63;  // -1: t < 0, keep d
#pragma unroll
    for (int i = 0; i < L; i++) d[i] = (d[i] & keep) | (t[i] & ~keep);
  }
#pragma unroll
  for (int w = 0; w < n64; w++) out[w] = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {  // repack B-bit limbs into 64-bit words
    const uint64_t x = (uint64_t)d[i];
    const int bit = B * i, w = bit >> 6, o = bit & 63;
    if (w < n64) out[w] |= x << o;
    if (o > 64 - B && w + 1 < n64) out[w + 1] |= x >> (64 - o);
  }
}

}  // namespace zk
