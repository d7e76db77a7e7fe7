// zk_msm.hip -- Pippenger bucket MSM for G1 (BN128 and BLS12-381) on gfx950.
//
// Replaces <C>_G1_proj_MSM_std_coeff_proj_out_variable (bls12_381_G1_proj.c:507-587)
// and its callers (:597-670).  Same mathematical result (sum_i k_i * P_i with the
// 256-bit scalars used verbatim -- no reduction mod r, no GLV, so the result is
// identical for points outside the order-r subgroup too), computed with
// a GPU-shaped schedule:
//
//   1. k_digits     scalar (Montgomery -> standard by REDC, Fr_mont.c:330-335) ->
//                   signed c-bit digits for all W windows + per-bucket histogram
//   2. scan         exclusive scan of the W*B bucket counts (hipCUB)
//   3. k_scatter    counting-sort scatter: (point index | sign) into bucket order
//   4. k_accum      balanced bucket accumulation: every thread adds exactly CH
//                   consecutive sorted entries (mixed XYZZ += affine adds), flushing
//                   complete buckets directly and boundary runs to head/tail slots
//   5. k_fixup      stitches buckets that straddle chunks
//   6. k_seg        per (window, segment of L buckets): T = sum B_m, R = sum (m-lo+1) B_m
//   7. k_bitsum     sum_m m B_m = sum_s R_s + L * sum_k 2^k U_k, U_k = sum_{s: bit k} T_s:
//                   every term is a plain point sum -> wide, shallow reductions
//   8. k_sumseg     further plain-sum levels until one point per (window, job)
//   9. host         Horner over the power-of-two exponents, normalise / to_affine
//
// Every phase is wide (>= ~1e5 threads at 2^20) except the last tiny levels: a lone
// wavefront's serial chain of 381-bit point adds is slow on CDNA4, so the
// deep-but-narrow tail runs on one host core (step 9).
#include <hipcub/hipcub.hpp>
#include "zk_curve.hpp"
#include "zk_host.hpp"
#include "zk_runtime.hpp"
#include "zk_msm.hpp"

namespace zk {

// ---------------------------------------------------------------------------
// XYZZ storage: 4 consecutive field elements, F::N u32 words each.
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

// 0. affine points: reference form -> internal form (once per call)
template <class C>
__global__ void __launch_bounds__(256) k_points_int(const uint64_t *__restrict__ pts, int n,
                                                    uint32_t *__restrict__ out) {
  using F = typename C::Fp;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  aff_ref_to_int<F>(out + (size_t)i * aff_words<F>(), pts + (size_t)i * 2 * F::N64);
}

// ---------------------------------------------------------------------------
// 1. digits + histogram
template <class C>
__global__ void __launch_bounds__(256) k_digits(const uint64_t *__restrict__ scalars, int n, int nl, int mont,
                                                int c, int W, uint32_t *__restrict__ digits,
                                                uint32_t *__restrict__ counts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  using Fr = typename C::Fr;
  uint32_t k[9];
  {
#pragma unroll
    for (int j = 0; j < 4; j++) {  // std scalars of 1..3 limbs: zero-extended
      const uint64_t w = (j < nl) ? scalars[(size_t)i * nl + j] : 0;
      k[2 * j] = (uint32_t)w;
      k[2 * j + 1] = (uint32_t)(w >> 32);
    }
    k[8] = 0;
    if (mont) {  // Montgomery -> standard (REDC), Fr_mont.c:330-335
      Fe<Fr> s, t;
      fe_unpack(s, k);
      fe_ref_to_std(t, s);
      fe_pack(k, t);
    }
  }
  const uint32_t B = 1u << (c - 1);
  const uint32_t full = 1u << c;
  const uint32_t mask = full - 1;
  uint32_t carry = 0;
  for (int w = 0; w < W; w++) {
    uint32_t raw = (k[0] & mask) + carry;
    // shift the 256-bit scalar right by c (c < 32)
#pragma unroll
    for (int j = 0; j < 8; j++) k[j] = __builtin_amdgcn_alignbit(k[j + 1], k[j], c);
    uint32_t code = 0;
    if (raw > B) {
      code = (full - raw) | 0x80000000u;  // negative digit raw - 2^c  (0 if raw == 2^c)
      carry = 1;
      if (raw == full) code = 0;
    } else {
      code = raw;
      carry = 0;
    }
    digits[(size_t)w * n + i] = code;
    if (code) atomicAdd(&counts[(size_t)w * B + (code & 0x7fffffffu) - 1], 1u);
  }
}

// 3. counting-sort scatter
__global__ void __launch_bounds__(256) k_scatter(const uint32_t *__restrict__ digits, int n, int c, int W,
                                                 uint32_t *__restrict__ cursor, uint32_t *__restrict__ list) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t B = 1u << (c - 1);
  for (int w = 0; w < W; w++) {
    uint32_t code = digits[(size_t)w * n + i];
    if (code) {
      uint32_t b = (uint32_t)w * B + (code & 0x7fffffffu) - 1;
      uint32_t pos = atomicAdd(&cursor[b], 1u);
      list[pos] = (uint32_t)i | (code & 0x80000000u);
    }
  }
}

// first bucket index b with offsets[b+1] > e  (offsets has nb+1 entries)
__device__ __forceinline__ uint32_t bucket_of(const uint32_t *__restrict__ offsets, uint32_t nb, uint32_t e) {
  uint32_t lo = 0, hi = nb;  // answer in [lo, hi)
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= e) lo = mid; else hi = mid;
  }
  return lo;
}

template <class F>
__device__ __forceinline__ void load_signed_point(Aff<F> &a, bool &inf, const uint32_t *__restrict__ points,
                                                  uint32_t code) {
  const uint32_t idx = code & 0x7fffffffu;
  inf = !aff_load(a, points + (size_t)idx * aff_words<F>());
  if (!inf && (code & 0x80000000u)) {
    Fe<F> ny;
    fe_neg(ny, a.y);
    a.y = ny;
  }
}

// 4. balanced accumulation: thread t owns sorted entries [t*CH, min((t+1)*CH, total))
template <class C>
__global__ void __launch_bounds__(256) k_accum(const uint32_t *__restrict__ points,
                                               const uint32_t *__restrict__ list,
                                               const uint32_t *__restrict__ offsets, uint32_t nb,
                                               uint32_t total, int CH, uint32_t *__restrict__ buckets,
                                               uint32_t *__restrict__ heads, uint32_t *__restrict__ tails) {
  using F = typename C::Fp;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t cs = t * (uint32_t)CH;
  if (cs >= total) return;
  const uint32_t ce = min(total, cs + (uint32_t)CH);
  uint32_t b = bucket_of(offsets, nb, cs);
  uint32_t bend = offsets[b + 1];
  bool first_run = true;
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  for (uint32_t e = cs; e < ce; e++) {
    if (e >= bend) {
      // flush the run of bucket b
      if (first_run) xyzz_store(heads + (size_t)t * xyzz_words<F>(), acc);
      else xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);  // complete inside the chunk
      first_run = false;
      xyzz_set_inf(acc);
      do { b++; bend = offsets[b + 1]; } while (bend <= e);
    }
    Aff<F> P;
    bool inf;
    load_signed_point(P, inf, points, list[e]);
    if (!inf) xyzz_add_aff(acc, P);
  }
  // last run
  if (first_run) xyzz_store(heads + (size_t)t * xyzz_words<F>(), acc);
  else if (bend > ce) xyzz_store(tails + (size_t)t * xyzz_words<F>(), acc);
  else xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);
}

// 5. stitch buckets that straddle chunks; write infinity into empty buckets
template <class C>
__global__ void __launch_bounds__(256) k_fixup(const uint32_t *__restrict__ offsets, uint32_t nb, int CH,
                                               uint32_t *__restrict__ buckets,
                                               const uint32_t *__restrict__ heads,
                                               const uint32_t *__restrict__ tails) {
  using F = typename C::Fp;
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint32_t ob = offsets[b], oe = offsets[b + 1];
  Xyzz<F> acc;
  if (ob == oe) {
    xyzz_set_inf(acc);
    xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);
    return;
  }
  const uint32_t t0 = ob / (uint32_t)CH, t1 = (oe - 1) / (uint32_t)CH;
  if (ob == t0 * (uint32_t)CH) {
    xyzz_load(acc, heads + (size_t)t0 * xyzz_words<F>());
  } else {
    if (t1 == t0) return;  // complete inside chunk t0, already written
    xyzz_load(acc, tails + (size_t)t0 * xyzz_words<F>());
  }
  for (uint32_t t = t0 + 1; t <= t1; t++) {
    Xyzz<F> h;
    xyzz_load(h, heads + (size_t)t * xyzz_words<F>());
    xyzz_add(acc, h);
  }
  xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);
}

// 6. per (window, segment): T = sum B_m, R = sum (m - lo + 1) B_m over L buckets
template <class C>
__global__ void __launch_bounds__(256) k_seg(const uint32_t *__restrict__ buckets, int W, int B, int L,
                                             uint32_t *__restrict__ Tout, uint32_t *__restrict__ Rout) {
  using F = typename C::Fp;
  const int S = B / L;
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= W * S) return;
  const int w = g / S, s = g % S;
  Xyzz<F> T, R;
  xyzz_set_inf(T);
  xyzz_set_inf(R);
  for (int m = L - 1; m >= 0; m--) {
    Xyzz<F> bm;
    xyzz_load(bm, buckets + ((size_t)w * B + (size_t)s * L + m) * xyzz_words<F>());
    xyzz_add(T, bm);
    xyzz_add(R, T);
  }
  xyzz_store(Tout + (size_t)g * xyzz_words<F>(), T);
  xyzz_store(Rout + (size_t)g * xyzz_words<F>(), R);
}

// 7. job j < logS: partial sums of T_s over s with bit j set; job logS: partial sums of R_s.
//    thread per (window, job, chunk)
template <class C>
__global__ void __launch_bounds__(256) k_bitsum(const uint32_t *__restrict__ T, const uint32_t *__restrict__ R,
                                                int W, int S, int logS, int CH2, int nchunk,
                                                uint32_t *__restrict__ out) {
  using F = typename C::Fp;
  const int J = logS + 1;
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= W * J * nchunk) return;
  const int ch = g % nchunk;
  const int j = (g / nchunk) % J;
  const int w = g / (nchunk * J);
  const int n = (j < logS) ? (S >> 1) : S;
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  const int e0 = ch * CH2, e1 = min(n, e0 + CH2);
  for (int e = e0; e < e1; e++) {
    Xyzz<F> p;
    if (j < logS) {
      const int lowmask = (1 << j) - 1;
      const int s = ((e & ~lowmask) << 1) | (1 << j) | (e & lowmask);
      xyzz_load(p, T + ((size_t)w * S + s) * xyzz_words<F>());
    } else {
      xyzz_load(p, R + ((size_t)w * S + e) * xyzz_words<F>());
    }
    xyzz_add(acc, p);
  }
  xyzz_store(out + (size_t)g * xyzz_words<F>(), acc);
}

// 8. plain segmented sum: in[grp][n] -> out[grp][ceil(n/G)]
template <class C>
__global__ void __launch_bounds__(256) k_sumseg(const uint32_t *__restrict__ in, int ngrp, int n, int G,
                                                uint32_t *__restrict__ out) {
  using F = typename C::Fp;
  const int nout = (n + G - 1) / G;
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngrp * nout) return;
  const int grp = g / nout, o = g % nout;
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  const int e1 = min(n, (o + 1) * G);
  for (int e = o * G; e < e1; e++) {
    Xyzz<F> p;
    xyzz_load(p, in + ((size_t)grp * n + e) * xyzz_words<F>());
    xyzz_add(acc, p);
  }
  xyzz_store(out + (size_t)g * xyzz_words<F>(), acc);
}

// export: XYZZ (device form) -> canonical reference-form coordinates, 4 x NP64 u64
template <class C>
__global__ void k_export(const uint32_t *__restrict__ in, int n, uint64_t *__restrict__ out) {
  using F = typename C::Fp;
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  Xyzz<F> p;
  xyzz_load(p, in + (size_t)g * xyzz_words<F>());
  uint64_t *o = out + (size_t)g * 4 * F::N64;
  Fe<F> t;
  fe_to_ref(t, p.X);
  fe_store_ref(o + 0 * F::N64, t);
  fe_to_ref(t, p.Y);
  fe_store_ref(o + 1 * F::N64, t);
  fe_to_ref(t, p.ZZ);
  fe_store_ref(o + 2 * F::N64, t);
  fe_to_ref(t, p.ZZZ);
  fe_store_ref(o + 3 * F::N64, t);
}

// ---------------------------------------------------------------------------
// host orchestration

struct MsmShape {
  int n, c, W, B, L, S, logS, J, CH, CH2, nchunk;
};

static int ilog2(unsigned x) { int r = 0; while ((1u << (r + 1)) <= x) r++; return r; }

int msm_default_window(int n) {
  // GPU window: more buckets are cheap on a wide device, fewer windows save
  // accumulation work.  (The reference uses round(log2 n - 3.5), G1_proj.c:600; the
  // result does not depend on the choice.)
  if (n <= 1) return 4;
  int lg = ilog2((unsigned)n);
  int c = lg - 4;
  if (c < 4) c = 4;
  if (c > 20) c = 20;
  return c;
}

static MsmShape make_shape(int n, int c, int nl) {
  MsmShape s;
  s.n = n;
  s.c = c;
  s.W = (64 * nl) / c + 1;  // signed digits: one extra window absorbs the final carry
  s.B = 1 << (c - 1);
  s.L = s.B >= 8 ? 4 : (s.B >= 2 ? s.B / 2 : 1);
  s.S = s.B / s.L;
  s.logS = ilog2((unsigned)s.S);
  s.J = s.logS + 1;
  s.CH = 32;
  s.CH2 = 16;
  s.nchunk = (s.S + s.CH2 - 1) / s.CH2;
  return s;
}

template <class C>
static size_t workspace_bytes(const MsmShape &s) {
  using F = typename C::Fp;
  const size_t xw = xyzz_words<F>() * 4;  // bytes per XYZZ
  const size_t nb = (size_t)s.W * s.B;
  const size_t maxent = (size_t)s.W * s.n;
  const size_t nchunks = (maxent + s.CH - 1) / s.CH + 1;
  size_t cub = 0;
  ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)(nb + 1)));
  size_t bytes = 0;
  auto add = [&](size_t b) { bytes += (b + 255) & ~size_t(255); };
  add((size_t)s.n * 4 * 8);          // staged scalars (<= 4 limbs)
  add((size_t)s.n * 2 * C::NP64 * 8);  // staged points
  add((size_t)s.n * aff_words<F>() * 4);  // internal-form points
  add(maxent * 4);                   // digits
  add((nb + 1) * 4);                 // counts
  add((nb + 1) * 4);                 // offsets
  add((nb + 1) * 4);                 // cursor
  add(maxent * 4);                   // list
  add(nchunks * xw * 2);             // heads + tails
  add(nb * xw);                      // buckets
  add((size_t)s.W * s.S * xw * 2);   // T, R
  add((size_t)s.W * s.J * s.nchunk * xw * 2);  // bitsum + sumseg ping-pong
  add((size_t)s.W * s.J * 4 * C::NP64 * 8);    // export
  add(cub);
  return bytes + (1 << 20);
}

template <class C>
static void finish_host(const MsmShape &s, const uint64_t *exported, zkh::Proj<typename HostOf<C>::Fp> &out);

// Run the device pipeline. scalars/points are DEVICE pointers (or host pointers when
// host_inputs, in which case they are staged).  Result: projective point in
// reference Montgomery form (not normalised), written to `out`.
template <class C>
static void msm_run(Device &dev, int n, const uint64_t *scalars, int nl, const uint64_t *points, bool host_inputs,
                    bool mont, int window, zkh::Proj<typename HostOf<C>::Fp> &out) {
  using HF = typename HostOf<C>::Fp;
  using F = typename C::Fp;
  if (n <= 0) {
    zkh::proj_set_inf<HF>(out);
    return;
  }
  const int c = (window >= 4 && window <= 24) ? window : msm_default_window(n);
  ZK_REQUIRE(nl >= 1 && nl <= 4, "msm: expo_nlimbs must be in 1..4 (scalars up to 256 bits)");
  ZK_REQUIRE(!mont || nl == 4, "msm: Montgomery coefficients must have expo_nlimbs == 4");
  MsmShape s = make_shape(n, c, nl);
  const size_t nb = (size_t)s.W * s.B;
  const size_t xw = xyzz_words<F>();
  hipStream_t st = dev.stream;

  dev.arena.reserve(workspace_bytes<C>(s));
  dev.arena.reset();
  const uint64_t *d_sc = scalars, *d_pt = points;
  if (host_inputs) {
    uint64_t *a = dev.arena.take<uint64_t>((size_t)n * nl);
    uint64_t *b = dev.arena.take<uint64_t>((size_t)n * 2 * C::NP64);
    ZK_CHECK(hipMemcpyAsync(a, scalars, (size_t)n * nl * 8, hipMemcpyHostToDevice, st));
    ZK_CHECK(hipMemcpyAsync(b, points, (size_t)n * 2 * C::NP64 * 8, hipMemcpyHostToDevice, st));
    d_sc = a;
    d_pt = b;
  }
  uint32_t *pts_int = dev.arena.take<uint32_t>((size_t)n * aff_words<F>());
  uint32_t *digits = dev.arena.take<uint32_t>((size_t)s.W * n);
  uint32_t *counts = dev.arena.take<uint32_t>(nb + 1);
  uint32_t *offsets = dev.arena.take<uint32_t>(nb + 1);
  uint32_t *cursor = dev.arena.take<uint32_t>(nb + 1);
  uint32_t *list = dev.arena.take<uint32_t>((size_t)s.W * n);
  const size_t maxent = (size_t)s.W * n;
  const size_t nchunks = (maxent + s.CH - 1) / s.CH + 1;
  uint32_t *heads = dev.arena.take<uint32_t>(nchunks * xw);
  uint32_t *tails = dev.arena.take<uint32_t>(nchunks * xw);
  uint32_t *buckets = dev.arena.take<uint32_t>(nb * xw);
  uint32_t *T = dev.arena.take<uint32_t>((size_t)s.W * s.S * xw);
  uint32_t *R = dev.arena.take<uint32_t>((size_t)s.W * s.S * xw);
  uint32_t *P0 = dev.arena.take<uint32_t>((size_t)s.W * s.J * s.nchunk * xw);
  uint32_t *P1 = dev.arena.take<uint32_t>((size_t)s.W * s.J * s.nchunk * xw);
  uint64_t *exp = dev.arena.take<uint64_t>((size_t)s.W * s.J * 4 * C::NP64);
  size_t cub = 0;
  ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub, counts, offsets, (int)(nb + 1), st));
  void *cubtmp = dev.arena.take<char>(cub);

  ZK_CHECK(hipMemsetAsync(counts, 0, (nb + 1) * 4, st));
  hipLaunchKernelGGL(k_points_int<C>, dim3(div_up(n, 256)), dim3(256), 0, st, d_pt, n, pts_int);
  ZK_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_digits<C>, dim3(div_up(n, 256)), dim3(256), 0, st, d_sc, n, nl, mont ? 1 : 0, c, s.W,
                     digits, counts);
  ZK_CHECK(hipGetLastError());
  ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(cubtmp, cub, counts, offsets, (int)(nb + 1), st));
  ZK_CHECK(hipMemcpyAsync(cursor, offsets, (nb + 1) * 4, hipMemcpyDeviceToDevice, st));
  hipLaunchKernelGGL(k_scatter, dim3(div_up(n, 256)), dim3(256), 0, st, digits, n, c, s.W, cursor, list);
  ZK_CHECK(hipGetLastError());
  uint32_t total = 0;
  ZK_CHECK(hipMemcpyAsync(&total, offsets + nb, 4, hipMemcpyDeviceToHost, st));
  ZK_CHECK(hipStreamSynchronize(st));

  KernelTimer &kt = dominant_timer();
  if (total > 0) {
    const uint32_t nthreads = (total + s.CH - 1) / s.CH;
    if (kt.enabled) ZK_CHECK(hipEventRecord(kt.ev0, st));
    hipLaunchKernelGGL(k_accum<C>, dim3(div_up(nthreads, 256)), dim3(256), 0, st, pts_int, list, offsets,
                       (uint32_t)nb, total, s.CH, buckets, heads, tails);
    ZK_CHECK(hipGetLastError());
    if (kt.enabled) ZK_CHECK(hipEventRecord(kt.ev1, st));
  }
  hipLaunchKernelGGL(k_fixup<C>, dim3(div_up(nb, 256)), dim3(256), 0, st, offsets, (uint32_t)nb, s.CH, buckets,
                     heads, tails);
  ZK_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_seg<C>, dim3(div_up((size_t)s.W * s.S, 256)), dim3(256), 0, st, buckets, s.W, s.B, s.L,
                     T, R);
  ZK_CHECK(hipGetLastError());
  const int ngrp = s.W * s.J;
  hipLaunchKernelGGL(k_bitsum<C>, dim3(div_up((size_t)ngrp * s.nchunk, 256)), dim3(256), 0, st, T, R, s.W, s.S,
                     s.logS, s.CH2, s.nchunk, P0);
  ZK_CHECK(hipGetLastError());
  int cur = s.nchunk;
  uint32_t *src = P0, *dst = P1;
  while (cur > 1) {
    const int G = 4;  // narrow levels: depth G each; G=4 minimises total serial depth
    const int nout = (cur + G - 1) / G;
    hipLaunchKernelGGL(k_sumseg<C>, dim3(div_up((size_t)ngrp * nout, 256)), dim3(256), 0, st, src, ngrp, cur, G,
                       dst);
    ZK_CHECK(hipGetLastError());
    cur = nout;
    uint32_t *tmp = src; src = dst; dst = tmp;
  }
  hipLaunchKernelGGL(k_export<C>, dim3(div_up(ngrp, 64)), dim3(64), 0, st, src, ngrp, exp);
  ZK_CHECK(hipGetLastError());
  const size_t expbytes = (size_t)ngrp * 4 * C::NP64 * 8;
  uint64_t *h = reinterpret_cast<uint64_t *>(dev.host_staging(expbytes));
  ZK_CHECK(hipMemcpyAsync(h, exp, expbytes, hipMemcpyDeviceToHost, st));
  ZK_CHECK(hipStreamSynchronize(st));
  if (kt.enabled && total > 0) {
    float ms = 0;
    ZK_CHECK(hipEventElapsedTime(&ms, kt.ev0, kt.ev1));
    kt.total_ms += ms;
    kt.launches++;
  }
  finish_host<C>(s, h, out);
}

// host: combine the per-(window, job) sums:
//   V_w = sum_s R_s + L * sum_k 2^k U_k ;  result = sum_w 2^(c w) V_w
// Every term is 2^e * Z with e = c*w (R job) or c*w + log2(L) + k (U_k job); those
// exponents never collide across windows, so one Horner pass over e does it all.
template <class C>
static void finish_host(const MsmShape &s, const uint64_t *exported, zkh::Proj<typename HostOf<C>::Fp> &out) {
  using HF = typename HostOf<C>::Fp;
  const int NP = C::NP64;
  zkh::Fe<HF> b3;
  HostOf<C>::b3(b3);
  const int logL = ilog2((unsigned)s.L);
  const int emax = s.c * (s.W - 1) + logL + s.logS + 1;
  std::vector<zkh::Proj<HF>> Z(emax + 1);
  for (auto &z : Z) zkh::proj_set_inf(z);
  for (int w = 0; w < s.W; w++) {
    for (int j = 0; j < s.J; j++) {
      const uint64_t *q = exported + ((size_t)w * s.J + j) * 4 * NP;
      zkh::Fe<HF> X, Y, ZZ, ZZZ;
      memcpy(X.v, q + 0 * NP, NP * 8);
      memcpy(Y.v, q + 1 * NP, NP * 8);
      memcpy(ZZ.v, q + 2 * NP, NP * 8);
      memcpy(ZZZ.v, q + 3 * NP, NP * 8);
      if (zkh::is_zero(ZZ)) continue;
      zkh::Proj<HF> p;  // (X*ZZZ : Y*ZZ : ZZ*ZZZ)
      zkh::mul(p.X, X, ZZZ);
      zkh::mul(p.Y, Y, ZZ);
      zkh::mul(p.Z, ZZ, ZZZ);
      const int e = (j < s.logS) ? s.c * w + logL + j : s.c * w;
      zkh::proj_add(Z[e], Z[e], p, b3);
    }
  }
  zkh::Proj<HF> acc;
  zkh::proj_set_inf(acc);
  for (int e = emax; e >= 0; e--) {
    if (!zkh::proj_is_inf(acc)) zkh::proj_dbl(acc, acc, b3);
    if (!zkh::proj_is_inf(Z[e])) zkh::proj_add(acc, acc, Z[e], b3);
  }
  out = acc;
}

// ---------------------------------------------------------------------------
// public (C++) entry points used by the C ABI layer

template <class C>
void msm_g1(int n, const uint64_t *scalars, int nl, const uint64_t *points, bool host_inputs, bool mont,
            int window, uint64_t *out_proj) {
  using HF = typename HostOf<C>::Fp;
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  zkh::Proj<HF> r;
  msm_run<C>(dev, n, scalars, nl, points, host_inputs, mont, window, r);
  memcpy(out_proj + 0 * C::NP64, r.X.v, C::NP64 * 8);
  memcpy(out_proj + 1 * C::NP64, r.Y.v, C::NP64 * 8);
  memcpy(out_proj + 2 * C::NP64, r.Z.v, C::NP64 * 8);
}

template void msm_g1<BN254>(int, const uint64_t *, int, const uint64_t *, bool, bool, int, uint64_t *);
template void msm_g1<BLS381>(int, const uint64_t *, int, const uint64_t *, bool, bool, int, uint64_t *);

}  // namespace zk
