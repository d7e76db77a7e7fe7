/*
 * zk_oracle.c -- CPU restatement (plain C) of the reference's MSM and NTT hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see zk_oracle.h).  Written from the reference's algorithm,
 * not copied: one generic field engine parameterised by a descriptor instead of the
 * reference's per-field generated files, constants derived at start-up from the primes.
 *
 *   field ops      bls12_381_Fr_mont.c:84-116 (add/sub), :140-199 (product + REDC),
 *                  :201-204 + bls12_381_Fr_std.c:251-315 (inverse: binary ext. Euclid, x R^3),
 *                  :330-335 (to_std)
 *   G1 projective  bls12_381_G1_proj.c:173-183 (infinity), :121-145 (affine conv.),
 *                  :231-264 (dbl-2007-bl), :273-314 (add-2015-rcb), :334-374 (madd-1998-cmo)
 *   MSM            bls12_381_G1_proj.c:507-587 (bucket method), :597-605 (window rule),
 *                  :611-620 (naive reference), :630-670 (mont / affine wrappers)
 *   NTT            bls12_381_poly_mont.c:418-452 (forward DIT), :472-511 (inverse DIF, 1/2 per level)
 * (bn128_* files: same line numbers.)
 */
#include "zk_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

#define MAXL 6

typedef struct {
  int n;               /* 64-bit limbs */
  int bits;
  uint64_t p[MAXL];
  uint64_t minv;       /* -p^-1 mod 2^64 */
  uint64_t one[MAXL];  /* R mod p */
  uint64_t r2[MAXL];
  uint64_t r3[MAXL];
} fld_t;

static fld_t FLD[4];

static const char *PRIME_HEX[4] = {
    "30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47", /* bn Fp */
    "30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001", /* bn Fr */
    "1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB", /* bls Fp */
    "73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001", /* bls Fr */
};

/* curve data: base field id, scalar field id, B, generator (standard form hex), fft gen (decimal) */
typedef struct {
  int fp, fr;
  int B;
  const char *gx, *gy;
  const char *fftgen_hex;
  int fftlog;
  uint64_t b3[MAXL];   /* 3B in Montgomery form */
  uint64_t gxm[MAXL], gym[MAXL];
  uint64_t fftgen[4];  /* Montgomery */
} curve_t;

static curve_t CRV[2] = {
    {0, 1, 3, "1", "2",
     /* 19103219067921713944291392827692070036145651957329286315305642004821462161904 */
     "2A3C09F0A58A7E8500E0A7EB8EF62ABC402D111E41112ED49BD61B6E725B19F0", 28, {0}, {0}, {0}, {0}},
    {2, 3, 4,
     "17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB",
     "08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1",
     /* 10238227357739495823651030575849232062558860180284477541189508159991286009131 */
     "16A2A19EDFE81F20D09B681922C813B4B63683508C2280B93829971F439F0D2B", 32, {0}, {0}, {0}, {0}},
};

/* ---------------------------------------------------------------- limb helpers */

static void hex_to_limbs(const char *h, uint64_t *w, int n) {
  memset(w, 0, 8 * (size_t)n);
  int len = (int)strlen(h);
  for (int i = 0; i < len; i++) {
    char ch = h[len - 1 - i];
    int v = (ch >= '0' && ch <= '9') ? ch - '0' : ((ch | 32) - 'a' + 10);
    w[i / 16] |= (uint64_t)v << (4 * (i % 16));
  }
}

static int big_cmp(const uint64_t *a, const uint64_t *b, int n) {
  for (int i = n - 1; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i] ? 1 : -1;
  }
  return 0;
}
static uint64_t big_add(uint64_t *r, const uint64_t *a, const uint64_t *b, int n) {
  u128 c = 0;
  for (int i = 0; i < n; i++) {
    c += (u128)a[i] + b[i];
    r[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}
static uint64_t big_sub(uint64_t *r, const uint64_t *a, const uint64_t *b, int n) {
  uint64_t br = 0;
  for (int i = 0; i < n; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}
static int big_is_zero(const uint64_t *a, int n) {
  for (int i = 0; i < n; i++)
    if (a[i]) return 0;
  return 1;
}
static int big_is_one(const uint64_t *a, int n) {
  if (a[0] != 1) return 0;
  for (int i = 1; i < n; i++)
    if (a[i]) return 0;
  return 1;
}
static void big_shr1(uint64_t *a, int n) {
  for (int i = 0; i < n; i++) a[i] = (a[i] >> 1) | (i + 1 < n ? a[i + 1] << 63 : 0);
}

/* ---------------------------------------------------------------- field engine */

static void f_add(const fld_t *F, const uint64_t *a, const uint64_t *b, uint64_t *r) {
  uint64_t t[MAXL];
  uint64_t c = big_add(t, a, b, F->n);
  if (c || big_cmp(t, F->p, F->n) >= 0) big_sub(t, t, F->p, F->n);
  memcpy(r, t, 8 * (size_t)F->n);
}
static void f_sub(const fld_t *F, const uint64_t *a, const uint64_t *b, uint64_t *r) {
  uint64_t t[MAXL];
  if (big_sub(t, a, b, F->n)) big_add(t, t, F->p, F->n);
  memcpy(r, t, 8 * (size_t)F->n);
}
static __attribute__((unused)) void f_neg(const fld_t *F, const uint64_t *a, uint64_t *r) {
  uint64_t z[MAXL] = {0};
  f_sub(F, z, a, r);
}
/* full product followed by a separate REDC (the reference's structure, Fr_mont.c:140-199) */
static void f_redc(const fld_t *F, uint64_t *T /* 2n+1 limbs, T[2n] scratch */, uint64_t *r) {
  const int n = F->n;
  T[2 * n] = 0;
  for (int i = 0; i < n; i++) {
    uint64_t m = T[i] * F->minv;
    u128 acc = 0;
    for (int j = 0; j < n; j++) {
      acc += (u128)m * F->p[j] + T[i + j];
      T[i + j] = (uint64_t)acc;
      acc >>= 64;
    }
    for (int k = i + n; k <= 2 * n && acc; k++) {
      acc += T[k];
      T[k] = (uint64_t)acc;
      acc >>= 64;
    }
  }
  uint64_t t[MAXL];
  memcpy(t, T + n, 8 * (size_t)n);
  if (T[2 * n] || big_cmp(t, F->p, n) >= 0) big_sub(t, t, F->p, n);
  memcpy(r, t, 8 * (size_t)n);
}
static void f_mul(const fld_t *F, const uint64_t *a, const uint64_t *b, uint64_t *r) {
  const int n = F->n;
  uint64_t T[2 * MAXL + 1];
  memset(T, 0, sizeof T);
  for (int i = 0; i < n; i++) {
    u128 acc = 0;
    for (int j = 0; j < n; j++) {
      acc += (u128)a[i] * b[j] + T[i + j];
      T[i + j] = (uint64_t)acc;
      acc >>= 64;
    }
    T[i + n] = (uint64_t)acc;
  }
  f_redc(F, T, r);
}
static void f_to_std(const fld_t *F, const uint64_t *a, uint64_t *r) {
  uint64_t T[2 * MAXL + 1];
  memset(T, 0, sizeof T);
  memcpy(T, a, 8 * (size_t)F->n);
  f_redc(F, T, r);
}
/* half of x mod p for x < p */
static void f_half_std(const fld_t *F, uint64_t *x) {
  if (x[0] & 1) {
    uint64_t c = big_add(x, x, F->p, F->n);
    big_shr1(x, F->n);
    x[F->n - 1] |= c << 63;
  } else {
    big_shr1(x, F->n);
  }
}
/* inverse of a Montgomery element: binary extended Euclid on the raw integer, then x R^3
   (Fr_std.c:251-315, Fr_mont.c:201-204).  0 -> 0. */
static void f_inv(const fld_t *F, const uint64_t *a, uint64_t *r) {
  const int n = F->n;
  if (big_is_zero(a, n)) { memset(r, 0, 8 * (size_t)n); return; }
  uint64_t u[MAXL], v[MAXL], x1[MAXL] = {0}, x2[MAXL] = {0};
  memcpy(u, a, 8 * (size_t)n);
  memcpy(v, F->p, 8 * (size_t)n);
  x1[0] = 1;
  while (!big_is_one(u, n) && !big_is_one(v, n)) {
    while (!(u[0] & 1)) { big_shr1(u, n); f_half_std(F, x1); }
    while (!(v[0] & 1)) { big_shr1(v, n); f_half_std(F, x2); }
    if (big_cmp(u, v, n) >= 0) { big_sub(u, u, v, n); f_sub(F, x1, x2, x1); }
    else { big_sub(v, v, u, n); f_sub(F, x2, x1, x2); }
  }
  uint64_t t[MAXL];
  memcpy(t, big_is_one(u, n) ? x1 : x2, 8 * (size_t)n);
  f_mul(F, t, F->r3, r);
}

static void derive_field(fld_t *F, const char *hex) {
  memset(F, 0, sizeof *F);
  int nib = (int)strlen(hex);
  F->n = (nib * 4 + 63) / 64;
  hex_to_limbs(hex, F->p, F->n);
  int top = F->n - 1;
  F->bits = 64 * top + (64 - __builtin_clzll(F->p[top]));
  uint64_t inv = 1;  /* Newton iteration for p^-1 mod 2^64 */
  for (int i = 0; i < 7; i++) inv *= 2 - F->p[0] * inv;
  F->minv = (uint64_t)0 - inv;
  /* R mod p, R^2, R^3 by modular doubling of 1 */
  uint64_t x[MAXL] = {0};
  x[0] = 1;
  for (int k = 1; k <= 3 * 64 * F->n; k++) {
    f_add(F, x, x, x);
    if (k == 64 * F->n) memcpy(F->one, x, sizeof x);
    if (k == 2 * 64 * F->n) memcpy(F->r2, x, sizeof x);
    if (k == 3 * 64 * F->n) memcpy(F->r3, x, sizeof x);
  }
}
static void f_from_std(const fld_t *F, const uint64_t *a, uint64_t *r) { f_mul(F, a, F->r2, r); }

int zko_init(void) {
  static int done = 0;
  if (done) return 0;
  for (int i = 0; i < 4; i++) derive_field(&FLD[i], PRIME_HEX[i]);
  for (int c = 0; c < 2; c++) {
    curve_t *C = &CRV[c];
    const fld_t *Fp = &FLD[C->fp], *Fr = &FLD[C->fr];
    uint64_t t[MAXL] = {0};
    t[0] = (uint64_t)(3 * C->B);
    f_from_std(Fp, t, C->b3);
    hex_to_limbs(C->gx, t, Fp->n);
    f_from_std(Fp, t, C->gxm);
    hex_to_limbs(C->gy, t, Fp->n);
    f_from_std(Fp, t, C->gym);
    hex_to_limbs(C->fftgen_hex, t, Fr->n);
    f_from_std(Fr, t, C->fftgen);
  }
  done = 1;
  return 0;
}

void zko_fadd(int f, const uint64_t *a, const uint64_t *b, uint64_t *r) { zko_init(); f_add(&FLD[f], a, b, r); }
void zko_fsub(int f, const uint64_t *a, const uint64_t *b, uint64_t *r) { zko_init(); f_sub(&FLD[f], a, b, r); }
void zko_fmul(int f, const uint64_t *a, const uint64_t *b, uint64_t *r) { zko_init(); f_mul(&FLD[f], a, b, r); }
void zko_finv(int f, const uint64_t *a, uint64_t *r) { zko_init(); f_inv(&FLD[f], a, r); }
void zko_to_std(int f, const uint64_t *a, uint64_t *r) { zko_init(); f_to_std(&FLD[f], a, r); }

/* ---------------------------------------------------------------- G1 projective */

typedef struct { uint64_t X[MAXL], Y[MAXL], Z[MAXL]; } pt_t;

static void pt_set_inf(const fld_t *F, pt_t *r) {
  memset(r, 0, sizeof *r);
  memcpy(r->Y, F->one, 8 * (size_t)F->n);
}
/* G1_proj.c:173-177 */
static int pt_is_inf(const fld_t *F, const pt_t *a) {
  return big_is_zero(a->Z, F->n) && !big_is_zero(a->Y, F->n) && big_is_zero(a->X, F->n);
}
static int aff_is_inf(const fld_t *F, const uint64_t *a) {
  for (int i = 0; i < 2 * F->n; i++)
    if (a[i] != ~(uint64_t)0) return 0;
  return 1;
}
static void pt_from_aff(const fld_t *F, const uint64_t *a, pt_t *r) {
  if (aff_is_inf(F, a)) { pt_set_inf(F, r); return; }
  memcpy(r->X, a, 8 * (size_t)F->n);
  memcpy(r->Y, a + F->n, 8 * (size_t)F->n);
  memcpy(r->Z, F->one, 8 * (size_t)F->n);
}

/* dbl-2007-bl, a = 0 (G1_proj.c:231-264) */
static void pt_dbl(const fld_t *F, const pt_t *P, pt_t *out) {
  uint64_t XX[MAXL], w[MAXL], s[MAXL], ss[MAXL], R[MAXL], RR[MAXL], B[MAXL], h[MAXL];
  pt_t r;
  f_mul(F, P->X, P->X, XX);
  f_add(F, XX, XX, w);
  f_add(F, w, XX, w);          /* w = 3 XX */
  f_mul(F, P->Y, P->Z, s);
  f_add(F, s, s, s);           /* s = 2 Y Z */
  f_mul(F, s, s, ss);
  f_mul(F, P->Y, s, R);
  f_mul(F, R, R, RR);
  f_add(F, P->X, R, B);
  f_mul(F, B, B, B);
  f_sub(F, B, XX, B);
  f_sub(F, B, RR, B);          /* B = (X+R)^2 - XX - RR */
  f_mul(F, w, w, h);
  f_sub(F, h, B, h);
  f_sub(F, h, B, h);           /* h = w^2 - 2B */
  f_mul(F, s, ss, r.Z);
  f_mul(F, h, s, r.X);
  f_sub(F, B, h, r.Y);
  f_mul(F, r.Y, w, r.Y);
  f_sub(F, r.Y, RR, r.Y);
  f_sub(F, r.Y, RR, r.Y);
  *out = r;
}

/* add-2015-rcb, a = 0 (G1_proj.c:273-314); b3 = 3B */
static void pt_add(const fld_t *F, const uint64_t *b3, const pt_t *P, const pt_t *Q, pt_t *out) {
  uint64_t t0[MAXL], t1[MAXL], t2[MAXL], t3[MAXL], t4[MAXL], t5[MAXL];
  pt_t r;
  f_mul(F, P->X, Q->X, t0);
  f_mul(F, P->Y, Q->Y, t1);
  f_mul(F, P->Z, Q->Z, t2);
  f_add(F, P->X, P->Y, t3);
  f_add(F, Q->X, Q->Y, t4);
  f_mul(F, t3, t4, t3);
  f_add(F, t0, t1, t4);
  f_sub(F, t3, t4, t3);
  f_add(F, P->X, P->Z, t4);
  f_add(F, Q->X, Q->Z, t5);
  f_mul(F, t4, t5, t4);
  f_add(F, t0, t2, t5);
  f_sub(F, t4, t5, t4);
  f_add(F, P->Y, P->Z, t5);
  f_add(F, Q->Y, Q->Z, r.X);
  f_mul(F, t5, r.X, t5);
  f_add(F, t1, t2, r.X);
  f_sub(F, t5, r.X, t5);
  f_mul(F, b3, t2, r.X);
  memcpy(r.Z, r.X, sizeof r.Z);
  f_sub(F, t1, r.Z, r.X);
  f_add(F, r.Z, t1, r.Z);
  f_mul(F, r.X, r.Z, r.Y);
  f_add(F, t0, t0, t1);
  f_add(F, t1, t0, t1);
  f_mul(F, b3, t4, t4);
  f_mul(F, t1, t4, t0);
  f_add(F, r.Y, t0, r.Y);
  f_mul(F, t4, t5, t0);
  f_mul(F, r.X, t3, r.X);
  f_sub(F, r.X, t0, r.X);
  f_mul(F, t1, t3, t0);
  f_mul(F, r.Z, t5, r.Z);
  f_add(F, r.Z, t0, r.Z);
  *out = r;
}

/* madd-1998-cmo with the reference's special cases (G1_proj.c:334-374) */
static void pt_madd(const fld_t *F, const uint64_t *b3, const pt_t *P, const uint64_t *A, pt_t *out) {
  (void)b3;
  if (pt_is_inf(F, P)) { pt_from_aff(F, A, out); return; }
  if (aff_is_inf(F, A)) { *out = *P; return; }
  const int n = F->n;
  uint64_t u[MAXL], uu[MAXL], v[MAXL], vv[MAXL], vvv[MAXL], R[MAXL], Aa[MAXL];
  f_mul(F, A + n, P->Z, u);
  f_sub(F, u, P->Y, u);
  f_mul(F, A, P->Z, v);
  f_sub(F, v, P->X, v);
  if (big_is_zero(u, n) && big_is_zero(v, n)) { pt_dbl(F, P, out); return; }
  pt_t r;
  f_mul(F, u, u, uu);
  f_mul(F, v, v, vv);
  f_mul(F, v, vv, vvv);
  f_mul(F, vv, P->X, R);
  f_mul(F, uu, P->Z, Aa);
  f_sub(F, Aa, vvv, Aa);
  f_sub(F, Aa, R, Aa);
  f_sub(F, Aa, R, Aa);
  f_mul(F, v, Aa, r.X);
  f_mul(F, P->Z, vvv, r.Z);
  f_sub(F, R, Aa, R);
  f_mul(F, vvv, P->Y, vvv);
  f_mul(F, u, R, r.Y);
  f_sub(F, r.Y, vvv, r.Y);
  *out = r;
}

static void pt_load(const fld_t *F, const uint64_t *p, pt_t *r) {
  memcpy(r->X, p, 8 * (size_t)F->n);
  memcpy(r->Y, p + F->n, 8 * (size_t)F->n);
  memcpy(r->Z, p + 2 * F->n, 8 * (size_t)F->n);
}
static void pt_store(const fld_t *F, const pt_t *r, uint64_t *p) {
  memcpy(p, r->X, 8 * (size_t)F->n);
  memcpy(p + F->n, r->Y, 8 * (size_t)F->n);
  memcpy(p + 2 * F->n, r->Z, 8 * (size_t)F->n);
}

/* G1_proj.c:133-145 */
void zko_proj_to_affine(int curve, const uint64_t *p, uint64_t *a) {
  zko_init();
  const fld_t *F = &FLD[CRV[curve].fp];
  pt_t P;
  pt_load(F, p, &P);
  if (big_is_zero(P.Z, F->n)) { memset(a, 0xff, 16 * (size_t)F->n); return; }
  uint64_t zi[MAXL];
  f_inv(F, P.Z, zi);
  f_mul(F, P.X, zi, a);
  f_mul(F, P.Y, zi, a + F->n);
}
/* G1_proj.c:79-98 */
void zko_proj_normalize(int curve, const uint64_t *p, uint64_t *q) {
  zko_init();
  const fld_t *F = &FLD[CRV[curve].fp];
  pt_t P, Q;
  pt_load(F, p, &P);
  if (big_is_zero(P.Z, F->n)) {
    pt_set_inf(F, &Q);
  } else if (big_cmp(P.Z, F->one, F->n) == 0) {
    Q = P;
  } else {
    uint64_t zi[MAXL];
    f_inv(F, P.Z, zi);
    f_mul(F, P.X, zi, Q.X);
    f_mul(F, P.Y, zi, Q.Y);
    memcpy(Q.Z, F->one, sizeof Q.Z);
  }
  pt_store(F, &Q, q);
}
void zko_proj_add(int curve, const uint64_t *p, const uint64_t *q, uint64_t *r) {
  zko_init();
  const fld_t *F = &FLD[CRV[curve].fp];
  pt_t P, Q, R;
  pt_load(F, p, &P);
  pt_load(F, q, &Q);
  pt_add(F, CRV[curve].b3, &P, &Q, &R);
  pt_store(F, &R, r);
}

/* ---------------------------------------------------------------- MSM */

/* bits [A, B) of a little-endian multi-limb integer, B - A <= 64 */
static uint64_t bit_window(const uint64_t *e, int A, int B) {
  int w = B - A;
  uint64_t lo = e[A >> 6] >> (A & 63);
  if ((A & 63) && ((B - 1) >> 6) != (A >> 6)) lo |= e[(A >> 6) + 1] << (64 - (A & 63));
  return w >= 64 ? lo : (lo & (((uint64_t)1 << w) - 1));
}

/* G1_proj.c:507-587 */
void zko_msm_std_proj_variable(int curve, int n, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt,
                               int nl, int window) {
  zko_init();
  const curve_t *C = &CRV[curve];
  const fld_t *F = &FLD[C->fp];
  if (window < 1) window = 1;
  if (window > 30) window = 30;  /* the reference's int mask is UB beyond this */
  const int bits = 64 * nl;
  const int nwin = (bits + window - 1) / window;
  const int nbkt = 1 << window;
  pt_t *S = (pt_t *)malloc(sizeof(pt_t) * (size_t)(nbkt - 1));
  pt_t acc;
  pt_set_inf(F, &acc);
  for (int K = nwin - 1; K >= 0; K--) {
    const int A = K * window;
    int Bb = A + window;
    if (Bb > bits) Bb = bits;
    for (int b = 0; b < nbkt - 1; b++) pt_set_inf(F, &S[b]);
    for (int j = 0; j < n; j++) {
      uint64_t e = bit_window(expos + (size_t)nl * j, A, Bb);
      if (e) pt_madd(F, C->b3, &S[e - 1], grps + (size_t)2 * F->n * j, &S[e - 1]);
    }
    pt_t T, R;
    pt_set_inf(F, &T);
    pt_set_inf(F, &R);
    for (int b = nbkt - 2; b >= 0; b--) {
      pt_add(F, C->b3, &T, &S[b], &T);
      pt_add(F, C->b3, &R, &T, &R);
    }
    if (!pt_is_inf(F, &acc))
      for (int i = 0; i < window; i++) pt_dbl(F, &acc, &acc);
    pt_add(F, C->b3, &acc, &R, &acc);
  }
  free(S);
  pt_store(F, &acc, tgt);
}

/* window rule round(log2 n - 3.5), clamped (G1_proj.c:600-602) */
static int ref_window(int n) {
  int c = (int)round(log2((double)n) - 3.5);
  if (n <= 0) c = 1;
  if (c < 1) c = 1;
  if (c > 64) c = 64;
  return c;
}
void zko_msm_std_proj(int curve, int n, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int nl) {
  if (n <= 0) {
    zko_init();
    pt_t z;
    pt_set_inf(&FLD[CRV[curve].fp], &z);
    pt_store(&FLD[CRV[curve].fp], &z, tgt);
    return;
  }
  zko_msm_std_proj_variable(curve, n, expos, grps, tgt, nl, ref_window(n));
}
void zko_msm_mont_proj(int curve, int n, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int nl) {
  zko_init();
  const fld_t *Fr = &FLD[CRV[curve].fr];
  uint64_t *std = (uint64_t *)malloc(8 * (size_t)nl * (size_t)(n > 0 ? n : 1));
  for (int i = 0; i < n; i++) f_to_std(Fr, expos + (size_t)nl * i, std + (size_t)nl * i);
  zko_msm_std_proj(curve, n, std, grps, tgt, nl);
  free(std);
}
void zko_msm_std_affine(int curve, int n, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int nl) {
  uint64_t p[3 * MAXL];
  zko_msm_std_proj(curve, n, expos, grps, p, nl);
  zko_proj_to_affine(curve, p, tgt);
}
void zko_msm_mont_affine(int curve, int n, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int nl) {
  uint64_t p[3 * MAXL];
  zko_msm_mont_proj(curve, n, expos, grps, p, nl);
  zko_proj_to_affine(curve, p, tgt);
}
/* naive: sum of double-and-add multiples (G1_proj.c:390-409, 611-620) */
void zko_msm_naive_affine(int curve, int n, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int nl) {
  zko_init();
  const curve_t *C = &CRV[curve];
  const fld_t *F = &FLD[C->fp];
  pt_t acc;
  pt_set_inf(F, &acc);
  for (int i = 0; i < n; i++) {
    pt_t base, sum;
    pt_from_aff(F, grps + (size_t)2 * F->n * i, &base);
    pt_set_inf(F, &sum);
    for (int b = 0; b < 64 * nl; b++) {
      if ((expos[(size_t)nl * i + (b >> 6)] >> (b & 63)) & 1) pt_add(F, C->b3, &sum, &base, &sum);
      pt_add(F, C->b3, &base, &base, &base);
    }
    pt_add(F, C->b3, &acc, &sum, &acc);
  }
  uint64_t p[3 * MAXL];
  pt_store(F, &acc, p);
  zko_proj_to_affine(curve, p, tgt);
}

/* ---------------------------------------------------------------- NTT */

/* forward DIT, poly_mont.c:418-452 */
static void ntt_fwd_rec(const fld_t *F, int m, int stride, const uint64_t *gen, const uint64_t *src, uint64_t *buf,
                        uint64_t *tgt) {
  const int L = F->n;
  if (m == 0) { memcpy(tgt, src, 8 * (size_t)L); return; }
  if (m == 1) {
    f_add(F, src, src + (size_t)stride * L, tgt);
    f_sub(F, src, src + (size_t)stride * L, tgt + L);
    return;
  }
  const size_t N = (size_t)1 << m, half = N >> 1;
  uint64_t g2[MAXL], gp[MAXL];
  f_mul(F, gen, gen, g2);
  ntt_fwd_rec(F, m - 1, stride * 2, g2, src, buf + N * L, buf);
  ntt_fwd_rec(F, m - 1, stride * 2, g2, src + (size_t)stride * L, buf + N * L, buf + half * L);
  memcpy(gp, F->one, sizeof gp);
  for (size_t j = 0; j < half; j++) {
    uint64_t t[MAXL];
    f_mul(F, buf + (j + half) * L, gp, t);
    f_add(F, buf + j * L, t, tgt + j * L);
    f_sub(F, buf + j * L, t, tgt + (j + half) * L);
    f_mul(F, gp, gen, gp);
  }
}

/* inverse DIF with a factor 1/2 per level, poly_mont.c:472-511 */
static void ntt_inv_rec(const fld_t *F, const uint64_t *half_m, int m, int tstride, const uint64_t *gen,
                        const uint64_t *src, uint64_t *buf, uint64_t *tgt) {
  const int L = F->n;
  if (m == 0) { memcpy(tgt, src, 8 * (size_t)L); return; }
  if (m == 1) {
    uint64_t a[MAXL], b[MAXL];
    f_add(F, src, src + L, a);
    f_sub(F, src, src + L, b);
    f_mul(F, a, half_m, tgt);
    f_mul(F, b, half_m, tgt + (size_t)tstride * L);
    return;
  }
  const size_t N = (size_t)1 << m, half = N >> 1;
  uint64_t ginv[MAXL], gp[MAXL], g2[MAXL];
  f_inv(F, gen, ginv);
  memcpy(gp, half_m, sizeof gp);
  for (size_t j = 0; j < half; j++) {
    uint64_t a[MAXL], b[MAXL];
    f_add(F, src + j * L, src + (j + half) * L, a);
    f_sub(F, src + j * L, src + (j + half) * L, b);
    f_mul(F, a, half_m, buf + j * L);
    f_mul(F, b, gp, buf + (j + half) * L);
    f_mul(F, gp, ginv, gp);
  }
  f_mul(F, gen, gen, g2);
  ntt_inv_rec(F, half_m, m - 1, tstride * 2, g2, buf, buf + N * L, tgt);
  ntt_inv_rec(F, half_m, m - 1, tstride * 2, g2, buf + half * L, buf + N * L, tgt + (size_t)tstride * L);
}

void zko_ntt_forward(int curve, int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {
  zko_init();
  const fld_t *F = &FLD[CRV[curve].fr];
  size_t N = (size_t)1 << m;
  uint64_t *buf = (uint64_t *)malloc(8 * (size_t)F->n * 2 * N);
  ntt_fwd_rec(F, m, 1, gen, src, buf, tgt);
  free(buf);
}
void zko_ntt_inverse(int curve, int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {
  zko_init();
  const fld_t *F = &FLD[CRV[curve].fr];
  uint64_t two[MAXL] = {0}, half_m[MAXL];
  two[0] = 2;
  f_from_std(F, two, two);
  f_inv(F, two, half_m);
  size_t N = (size_t)1 << m;
  uint64_t *buf = (uint64_t *)malloc(8 * (size_t)F->n * 2 * N);
  ntt_inv_rec(F, half_m, m, 1, gen, src, buf, tgt);
  free(buf);
}

/* ---------------------------------------------------------------- synthetic inputs */

static uint64_t sm64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void draw_below(const fld_t *F, uint64_t state, uint64_t *w) {
  int topbits = F->bits - 64 * (F->n - 1);
  uint64_t mask = topbits >= 64 ? ~(uint64_t)0 : (((uint64_t)1 << topbits) - 1);
  do {
    for (int i = 0; i < F->n; i++) w[i] = sm64(&state);
    w[F->n - 1] &= mask;
  } while (big_cmp(w, F->p, F->n) >= 0);
}
static uint64_t stream0(uint64_t seed, uint64_t i) { return seed ^ (0xD1B54A32D192ED03ull * (i + 1)); }

void zko_gen_fr(int curve, uint64_t seed, int64_t start, int64_t count, uint64_t *out) {
  zko_init();
  const fld_t *Fr = &FLD[CRV[curve].fr];
  for (int64_t k = 0; k < count; k++) draw_below(Fr, stream0(seed, (uint64_t)(start + k)), out + (size_t)k * Fr->n);
}

/* P_i = (a + i b) G, computed here by plain double-and-add of the integer a + i*b mod r */
void zko_gen_g1_points(int curve, uint64_t seed, int64_t start, int64_t count, uint64_t *out) {
  zko_init();
  const curve_t *C = &CRV[curve];
  const fld_t *Fp = &FLD[C->fp], *Fr = &FLD[C->fr];
  uint64_t a[MAXL] = {0}, b[MAXL] = {0};
  draw_below(Fr, stream0(seed ^ 0xA0761D6478BD642Full, 0), a);
  draw_below(Fr, stream0(seed ^ 0xE7037ED1A0B428DBull, 0), b);
  /* scalar arithmetic mod r in standard form via Montgomery round trips */
  uint64_t am[MAXL], bm[MAXL];
  f_from_std(Fr, a, am);
  f_from_std(Fr, b, bm);
  uint64_t G[2 * MAXL];
  memcpy(G, C->gxm, 8 * (size_t)Fp->n);
  memcpy(G + Fp->n, C->gym, 8 * (size_t)Fp->n);
  for (int64_t k = 0; k < count; k++) {
    uint64_t im[MAXL] = {0}, s[MAXL], sm[MAXL];
    im[0] = (uint64_t)(start + k);
    f_from_std(Fr, im, im);
    f_mul(Fr, im, bm, sm);
    f_add(Fr, sm, am, sm);
    f_to_std(Fr, sm, s);          /* k-th scalar a + i*b mod r */
    uint64_t pr[3 * MAXL];
    zko_msm_naive_affine(curve, 1, s, G, out + (size_t)k * 2 * Fp->n, Fr->n);
    (void)pr;
  }
}

void zko_fft_generator(int curve, int m, uint64_t *out) {
  zko_init();
  const curve_t *C = &CRV[curve];
  const fld_t *Fr = &FLD[C->fr];
  uint64_t g[MAXL];
  memcpy(g, C->fftgen, sizeof g);
  for (int i = m; i < C->fftlog; i++) f_mul(Fr, g, g, g);
  memcpy(out, g, 8 * (size_t)Fr->n);
}

/* ==========================================================================
 * Fr vector operations (lib/cbits/curves/array/mont/bls12_381_arr_mont.c) and
 * division by a vanishing polynomial (lib/cbits/curves/poly/mont/bls12_381_poly_mont.c).
 * Op codes = zikkurat-algebra_amd/csrc/zk_arr.hpp ArrOp. */
#define FR_OF(c) (&FLD[CRV[c].fr])
#define EL(p, i) ((p) + 4 * (size_t)(i))

/* Fr_mont_batch_inv (bls12_381_Fr_mont.c:258-285): prefix products, one inversion,
   backward sweep -- a zero anywhere makes every output zero */
static void batch_inv(const fld_t *F, int n, const uint64_t *src, uint64_t *tgt) {
  if (n <= 0) return;
  uint64_t *prods = malloc(32 * (size_t)n), *recips = malloc(32 * (size_t)n);
  memcpy(EL(prods, 0), EL(src, 0), 32);
  for (int i = 1; i < n; i++) f_mul(F, EL(prods, i - 1), EL(src, i), EL(prods, i));
  f_inv(F, EL(prods, n - 1), EL(recips, n - 1));
  for (int i = n - 2; i >= 0; i--) f_mul(F, EL(recips, i + 1), EL(src, i + 1), EL(recips, i));
  uint64_t first[4];
  memcpy(first, EL(recips, 0), 32);
  for (int i = n - 1; i >= 1; i--) f_mul(F, EL(recips, i), EL(prods, i - 1), EL(tgt, i));
  memcpy(EL(tgt, 0), first, 32);
  free(prods);
  free(recips);
}

void zko_arr_op(int curve, int op, int n, const uint64_t *a, const uint64_t *b, const uint64_t *c,
                const uint64_t *kA, const uint64_t *kB, uint64_t *tgt) {
  zko_init();
  const fld_t *F = FR_OF(curve);
  if (op == 15 || op == 16) { /* inv / div (arr_mont.c: inv, div) */
    if (n <= 0) return;
    uint64_t *tmp = malloc(32 * (size_t)n);
    batch_inv(F, n, op == 15 ? a : b, tmp);
    for (int i = 0; i < n; i++) {
      if (op == 15) memcpy(EL(tgt, i), EL(tmp, i), 32);
      else f_mul(F, EL(a, i), EL(tmp, i), EL(tgt, i));
    }
    free(tmp);
    return;
  }
  for (int i = 0; i < n; i++) {
    uint64_t t[4], u[4];
    switch (op) {
      case 0: f_neg(F, EL(a, i), t); break;
      case 1: f_add(F, EL(a, i), EL(b, i), t); break;
      case 2: f_sub(F, EL(a, i), EL(b, i), t); break;
      case 3: f_sub(F, EL(b, i), EL(a, i), t); break;                 /* sub_inplace_reverse */
      case 4: f_mul(F, EL(a, i), EL(a, i), t); break;
      case 5: f_mul(F, EL(a, i), EL(b, i), t); break;
      case 6: f_mul(F, EL(a, i), EL(b, i), u); f_add(F, u, EL(c, i), t); break;  /* mul_add */
      case 7: f_mul(F, EL(a, i), EL(b, i), u); f_sub(F, u, EL(c, i), t); break;  /* mul_sub */
      case 8: f_mul(F, kA, EL(a, i), t); break;                        /* scale */
      case 9: f_mul(F, kA, EL(a, i), u); f_add(F, u, EL(b, i), t); break;        /* Ax_plus_y */
      case 10: {                                                       /* Ax_plus_By */
        uint64_t v[4];
        f_mul(F, kA, EL(a, i), u);
        f_mul(F, kB, EL(b, i), v);
        f_add(F, u, v, t);
        break;
      }
      case 11: f_from_std(F, EL(a, i), t); break;
      case 12: f_to_std(F, EL(a, i), t); break;
      case 13: memcpy(t, EL(a, i), 32); break;
      default: memcpy(t, kA, 32); break;                               /* set_const */
    }
    memcpy(EL(tgt, i), t, 32);
  }
}

void zko_arr_dot(int curve, int n, const uint64_t *a, const uint64_t *b, uint64_t *tgt) {
  zko_init();
  const fld_t *F = FR_OF(curve);
  uint64_t acc[4] = {0}, t[4];
  for (int i = 0; i < n; i++) {
    f_mul(F, EL(a, i), EL(b, i), t);
    f_add(F, acc, t, acc);
  }
  memcpy(tgt, acc, 32);
}

void zko_arr_powers(int curve, int n, const uint64_t *kA, const uint64_t *kB, uint64_t *tgt) {
  zko_init();
  const fld_t *F = FR_OF(curve);
  if (n <= 0) return;
  memcpy(EL(tgt, 0), kA, 32);
  for (int i = 1; i < n; i++) f_mul(F, EL(tgt, i - 1), kB, EL(tgt, i));
}

/* poly_mont_div_by_vanishing (bls12_381_poly_mont.c:317-397): quotient / remainder of
   p(x) by x^n - eta; returns 1 if the remainder is zero (quot_by_vanishing, :402-413) */
int zko_div_by_vanishing(int curve, int n1, const uint64_t *src, int n, const uint64_t *eta, int nquot,
                         uint64_t *quot, int nrem, uint64_t *rem) {
  zko_init();
  const fld_t *F = FR_OF(curve);
  int deg = -1;
  for (int i = n1 - 1; i >= 0; i--)
    if (!big_is_zero(EL(src, i), 4)) { deg = i; break; }
  memset(quot, 0, 32 * (size_t)(nquot > 0 ? nquot : 0));
  if (rem) memset(rem, 0, 32 * (size_t)(nrem > 0 ? nrem : 0));
  uint64_t *r = rem;
  uint64_t *tmp = NULL;
  if (!r) { tmp = calloc((size_t)n, 32); r = tmp; }
  if (deg < n) {
    if (deg >= 0) memcpy(r, src, 32 * (size_t)(deg + 1));
  } else {
    for (int j = deg - n; j >= 0; j--) {
      if (j + n <= deg - n) {
        uint64_t t[4];
        f_mul(F, EL(quot, j + n), eta, t);
        f_add(F, EL(src, j + n), t, EL(quot, j));
      } else {
        memcpy(EL(quot, j), EL(src, j + n), 32);
      }
    }
    for (int j = 0; j < n; j++) {
      if (j <= deg - n) {
        uint64_t t[4];
        f_mul(F, EL(quot, j), eta, t);
        f_add(F, EL(src, j), t, EL(r, j));
      } else {
        memcpy(EL(r, j), EL(src, j), 32);
      }
    }
  }
  int ok = 1;
  for (int j = 0; j < n; j++)
    if (!big_is_zero(EL(r, j), 4)) { ok = 0; break; }
  free(tmp);
  return ok;
}
