// zk_msm.hip -- Pippenger bucket MSM for G1 (BN128 and BLS12-381) on gfx950.
//
// Replaces <C>_G1_proj_MSM_std_coeff_proj_out_variable (bls12_381_G1_proj.c:507-587)
// and its callers (:597-670).  Same mathematical result (sum_i k_i * P_i with the
// 256-bit scalars used verbatim -- no reduction mod r, no GLV, so the result is
// identical for points outside the order-r subgroup too), computed with
// a GPU-shaped schedule:
//
//   0. k_points_int affine points -> internal radix (one product per coordinate)
//   1. k_digits     scalar (Montgomery -> standard by REDC, Fr_mont.c:330-335) ->
//                   signed c-bit digits for all W windows -> (bucket key, index|sign)
//   2. sort         LSD radix sort of the W*n pairs by bucket key (hipCUB onesweep)
//   3. k_offsets    bucket start offsets from the sorted keys
//   4. k_accum      balanced bucket accumulation: every thread adds exactly CH
//                   consecutive sorted entries (mixed XYZZ += affine adds), flushing
//                   complete runs to their bucket and boundary runs as partial items
//   5. k_stitch     partial items are compacted and summed per bucket with the same
//                   balanced scheme, level after level (log_{SCH/2} levels): no serial
//                   loop anywhere, so skewed scalars (all equal, carry windows) stay fast
//   6. k_seg        per (window, segment of L buckets): T = sum B_m, R = sum (m-lo+1) B_m
//   7. k_jobsum     sum_m m B_m = sum_s R_s + L * sum_k 2^k U_k, U_k = sum_{s: bit k} T_s:
//                   every term is a plain point sum; one workgroup per (window, job)
//                   with an LDS tree
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
// 1. digits -> (key, value) pairs for the bucket sort.
//    key = w * B + (|digit| - 1), or nb (sentinel, sorts last) for a zero digit
//    value = point index | sign << 31
template <class C>
__global__ void __launch_bounds__(256) k_digits(const uint64_t *__restrict__ scalars, int n, int nl, int mont,
                                                int c, int W, uint32_t *__restrict__ keys,
                                                uint32_t *__restrict__ vals) {
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
  const uint32_t nb = (uint32_t)W * B;
  uint32_t carry = 0;
  for (int w = 0; w < W; w++) {
    uint32_t raw = (k[0] & mask) + carry;
    // shift the 256-bit scalar right by c (c < 32)
#pragma unroll
    for (int j = 0; j < 8; j++) k[j] = __builtin_amdgcn_alignbit(k[j + 1], k[j], c);
    uint32_t mag, sign;
    if (raw > B) {  // negative digit raw - 2^c (zero when raw == 2^c)
      mag = full - raw;
      sign = 0x80000000u;
      carry = 1;
    } else {
      mag = raw;
      sign = 0;
      carry = 0;
    }
    keys[(size_t)w * n + i] = mag ? (uint32_t)w * B + mag - 1 : nb;
    vals[(size_t)w * n + i] = (uint32_t)i | sign;
  }
}

// 3. bucket offsets from the sorted keys: offsets[b] = first position with key >= b,
//    one binary search per bucket (no serial loops, whatever the key distribution)
__global__ void __launch_bounds__(256) k_offsets(const uint32_t *__restrict__ skeys, uint32_t M, uint32_t nb,
                                                 uint32_t *__restrict__ offsets) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nb) return;
  uint32_t lo = 0, hi = M;  // first index in [lo, hi] with key >= b
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (skeys[mid] < b) lo = mid + 1; else hi = mid;
  }
  offsets[b] = lo;
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

// 4. level-0 balanced accumulation: thread t owns sorted entries [t*CH, min((t+1)*CH, total)).
//    Runs of one bucket that lie entirely inside the chunk are written straight to
//    buckets[b]; a run that crosses the chunk boundary (the chunk's first and/or last run)
//    becomes a "partial item" (key b, XYZZ sum) in slot 2t / 2t+1 of the item arrays.
//    Item slots that stay empty carry key = nb (dropped by the compaction).
template <class C>
__global__ void __launch_bounds__(256) k_accum(const uint32_t *__restrict__ points,
                                               const uint32_t *__restrict__ list,
                                               const uint32_t *__restrict__ offsets, uint32_t nb,
                                               int CH, uint32_t *__restrict__ buckets,
                                               uint32_t *__restrict__ ikeys, uint32_t *__restrict__ ivals,
                                               uint32_t nslots) {
  using F = typename C::Fp;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * t >= nslots) return;
  const uint32_t total = offsets[nb];
  const uint32_t cs = t * (uint32_t)CH;
  uint32_t k0 = nb, k1 = nb;  // item keys of slots 2t, 2t+1
  if (cs < total) {
    const uint32_t ce = min(total, cs + (uint32_t)CH);
    uint32_t b = bucket_of(offsets, nb, cs);
    uint32_t bbeg = offsets[b], bend = offsets[b + 1];
    bool first_run = true;
    Xyzz<F> acc;
    xyzz_set_inf(acc);
    for (uint32_t e = cs; e < ce; e++) {
      if (e >= bend) {  // run of bucket b ends inside the chunk
        if (first_run && bbeg < cs) {
          xyzz_store(ivals + (size_t)(2 * t) * xyzz_words<F>(), acc);
          k0 = b;
        } else {
          xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);
        }
        first_run = false;
        xyzz_set_inf(acc);
        do { b++; bbeg = offsets[b]; bend = offsets[b + 1]; } while (bend <= e);
      }
      Aff<F> P;
      bool inf;
      load_signed_point(P, inf, points, list[e]);
      if (!inf) xyzz_add_aff(acc, P);
    }
    // last run: partial if it started before the chunk or continues after it
    if (bbeg < cs || bend > ce) {
      const uint32_t slot = first_run ? 2 * t : 2 * t + 1;
      xyzz_store(ivals + (size_t)slot * xyzz_words<F>(), acc);
      if (first_run) k0 = b; else k1 = b;
    } else {
      xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);
    }
  }
  ikeys[2 * t] = k0;
  ikeys[2 * t + 1] = k1;
}

// 5a. compaction of the partial items (keys < nb), order preserving: scatter by a
//     prefix sum of the valid flags (scan done by hipCUB on `flags`)
__global__ void __launch_bounds__(256) k_item_flags(const uint32_t *__restrict__ ikeys, const uint32_t *__restrict__ count,
                                                    uint32_t nslots_max, uint32_t nb, uint32_t *__restrict__ flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots_max) return;
  const uint32_t n = count ? *count : nslots_max;
  flags[i] = (i < n && ikeys[i] < nb) ? 1u : 0u;
}
template <class C>
__global__ void __launch_bounds__(256) k_item_compact(const uint32_t *__restrict__ ikeys, const uint32_t *__restrict__ ivals,
                                                      const uint32_t *__restrict__ flags, const uint32_t *__restrict__ pos,
                                                      uint32_t nslots_max, uint32_t *__restrict__ okeys,
                                                      uint32_t *__restrict__ ovals, uint32_t *__restrict__ ocount) {
  using F = typename C::Fp;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots_max) return;
  if (i == nslots_max - 1) *ocount = pos[i] + flags[i];
  if (!flags[i]) return;
  const uint32_t o = pos[i];
  okeys[o] = ikeys[i];
  const uint4 *s = reinterpret_cast<const uint4 *>(ivals + (size_t)i * xyzz_words<F>());
  uint4 *d = reinterpret_cast<uint4 *>(ovals + (size_t)o * xyzz_words<F>());
#pragma unroll
  for (int q = 0; q < xyzz_words<F>() / 4; q++) d[q] = s[q];
}

// 5b. stitch level: the compacted items (sorted by key) are summed per key with the
//     same balanced-chunk scheme; complete runs go to buckets[b], runs crossing a chunk
//     boundary become the next level's items.  Levels repeat until one chunk remains.
template <class C>
__global__ void __launch_bounds__(256) k_stitch(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                const uint32_t *__restrict__ count, uint32_t nb, int CH,
                                                uint32_t *__restrict__ buckets, uint32_t *__restrict__ okeys,
                                                uint32_t *__restrict__ ovals, uint32_t nslots) {
  using F = typename C::Fp;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * t >= nslots) return;
  const uint32_t M = *count;
  const uint32_t cs = t * (uint32_t)CH;
  uint32_t k0 = nb, k1 = nb;
  if (cs < M) {
    const uint32_t ce = min(M, cs + (uint32_t)CH);
    uint32_t b = keys[cs];
    const bool cont_in = cs > 0 && keys[cs - 1] == b;
    bool first_run = true;
    Xyzz<F> acc;
    xyzz_set_inf(acc);
    for (uint32_t e = cs; e < ce; e++) {
      const uint32_t k = keys[e];
      if (k != b) {
        if (first_run && cont_in) {
          xyzz_store(ovals + (size_t)(2 * t) * xyzz_words<F>(), acc);
          k0 = b;
        } else {
          xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);
        }
        first_run = false;
        xyzz_set_inf(acc);
        b = k;
      }
      Xyzz<F> v;
      xyzz_load(v, vals + (size_t)e * xyzz_words<F>());
      xyzz_add(acc, v);
    }
    const bool cont_out = ce < M && keys[ce] == b;
    if ((first_run && cont_in) || cont_out) {
      const uint32_t slot = first_run ? 2 * t : 2 * t + 1;
      xyzz_store(ovals + (size_t)slot * xyzz_words<F>(), acc);
      if (first_run) k0 = b; else k1 = b;
    } else {
      xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);
    }
  }
  okeys[2 * t] = k0;
  okeys[2 * t + 1] = k1;
}

// 6. per (window, segment): T = sum B_m, R = sum (m - lo + 1) B_m over L buckets
template <class C>
__global__ void __launch_bounds__(256) k_seg(const uint32_t *__restrict__ buckets,
                                             const uint32_t *__restrict__ offsets, int W, int B, int L,
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
    const size_t b = (size_t)w * B + (size_t)s * L + m;
    if (offsets[b + 1] > offsets[b]) {  // empty buckets hold garbage (never written)
      Xyzz<F> bm;
      xyzz_load(bm, buckets + b * xyzz_words<F>());
      xyzz_add(T, bm);
    }
    xyzz_add(R, T);
  }
  xyzz_store(Tout + (size_t)g * xyzz_words<F>(), T);
  xyzz_store(Rout + (size_t)g * xyzz_words<F>(), R);
}

// 7. one workgroup per (window, job): job j < logS sums U_j = sum_{s: bit j of s} T_s,
//    job logS sums R_s.  Each thread first adds a strided share of the job's items, then
//    the workgroup folds the partials with an LDS tree: serial depth ~ items/JT + log2(JT)
//    point adds (the narrow tail of the reduction is latency bound on CDNA4).
constexpr int JT = 256;
template <class C>
__global__ void __launch_bounds__(JT) k_jobsum(const uint32_t *__restrict__ T, const uint32_t *__restrict__ R,
                                              int S, int logS, uint32_t *__restrict__ out) {
  using F = typename C::Fp;
  extern __shared__ uint32_t lds[];
  const int J = logS + 1;
  const int w = blockIdx.x / J, j = blockIdx.x % J;
  const int n = (j < logS) ? (S >> 1) : S;
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  for (int e = threadIdx.x; e < n; e += JT) {
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
  int active = min(JT, n);
  for (int stride = JT / 2; stride >= 1; stride >>= 1) {
    if (stride >= active) continue;  // uniform across the block
    if (threadIdx.x >= stride && threadIdx.x < 2 * stride && threadIdx.x < active)
      xyzz_store(lds + (size_t)(threadIdx.x - stride) * xyzz_words<F>(), acc);
    __syncthreads();
    if (threadIdx.x < stride && threadIdx.x + stride < active) {
      Xyzz<F> p;
      xyzz_load(p, lds + (size_t)threadIdx.x * xyzz_words<F>());
      xyzz_add(acc, p);
    }
    __syncthreads();
    active = stride;
  }
  if (threadIdx.x == 0) xyzz_store(out + (size_t)blockIdx.x * xyzz_words<F>(), acc);
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

static int key_bits(size_t nb) {  // keys are in [0, nb]
  int b = 1;
  while (((size_t)1 << b) <= nb) b++;
  return b;
}

struct MsmShape {
  int n, c, W, B, L, S, logS, J, CH, CH2, nchunk, SCH;
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
  s.CH = 64;   // entries per thread in the level-0 accumulation
  s.SCH = 8;   // items per thread in the stitch levels (mostly pairs: keep it wide)
  s.CH2 = 16;
  s.nchunk = (s.S + s.CH2 - 1) / s.CH2;
  return s;
}

static size_t stitch_slots0(const MsmShape &s) { return 2 * (((size_t)s.W * s.n + s.CH - 1) / s.CH); }
static size_t stitch_slots1(const MsmShape &s) { return 2 * ((stitch_slots0(s) + s.SCH - 1) / s.SCH) + 2; }

template <class C>
static size_t workspace_bytes(const MsmShape &s) {
  using F = typename C::Fp;
  const size_t xw = xyzz_words<F>() * 4;  // bytes per XYZZ
  const size_t nb = (size_t)s.W * s.B;
  const size_t maxent = (size_t)s.W * s.n;
  const size_t ns0 = stitch_slots0(s), ns1 = stitch_slots1(s);
  size_t cub = 0, cub2 = 0;
  ZK_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, cub, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                              (uint32_t *)nullptr, (uint32_t *)nullptr, (int)maxent, 0,
                                              key_bits(nb)));
  ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub2, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)ns0));
  size_t bytes = 0;
  auto add = [&](size_t b) { bytes += (b + 255) & ~size_t(255); };
  add((size_t)s.n * 4 * 8);               // staged scalars (<= 4 limbs)
  add((size_t)s.n * 2 * C::NP64 * 8);     // staged points
  add((size_t)s.n * aff_words<F>() * 4);  // internal-form points
  add(maxent * 4 * 4);                    // keys, vals, sorted keys, sorted vals
  add((nb + 1) * 4);                      // offsets
  add(ns0 * (xw + 4) * 2 + ns0 * 8 + 64); // level-0 items, compacted items, flags, pos, count
  add(ns1 * (xw + 4) * 2);                // stitch ping-pong
  add(nb * xw);                           // buckets
  add((size_t)s.W * s.S * xw * 2);        // T, R
  add((size_t)s.W * s.J * xw);               // per-(window, job) sums
  add((size_t)s.W * s.J * 4 * C::NP64 * 8);    // export
  add(cub > cub2 ? cub : cub2);
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
  const size_t maxent = (size_t)s.W * n;
  uint32_t *keys = dev.arena.take<uint32_t>(maxent);
  uint32_t *vals = dev.arena.take<uint32_t>(maxent);
  uint32_t *skeys = dev.arena.take<uint32_t>(maxent);
  uint32_t *list = dev.arena.take<uint32_t>(maxent);  // sorted values
  uint32_t *offsets = dev.arena.take<uint32_t>(nb + 1);
  const size_t ns0 = stitch_slots0(s), ns1 = stitch_slots1(s);
  uint32_t *ikeys0 = dev.arena.take<uint32_t>(ns0);
  uint32_t *ivals0 = dev.arena.take<uint32_t>(ns0 * xw);
  uint32_t *ckeys = dev.arena.take<uint32_t>(ns0);
  uint32_t *cvals = dev.arena.take<uint32_t>(ns0 * xw);
  uint32_t *flags = dev.arena.take<uint32_t>(ns0);
  uint32_t *pos = dev.arena.take<uint32_t>(ns0);
  uint32_t *ccount = dev.arena.take<uint32_t>(16);
  uint32_t *okA = dev.arena.take<uint32_t>(ns1);
  uint32_t *ovA = dev.arena.take<uint32_t>(ns1 * xw);
  uint32_t *okB = dev.arena.take<uint32_t>(ns1);
  uint32_t *ovB = dev.arena.take<uint32_t>(ns1 * xw);
  uint32_t *buckets = dev.arena.take<uint32_t>(nb * xw);
  uint32_t *T = dev.arena.take<uint32_t>((size_t)s.W * s.S * xw);
  uint32_t *R = dev.arena.take<uint32_t>((size_t)s.W * s.S * xw);
  uint32_t *P0 = dev.arena.take<uint32_t>((size_t)s.W * s.J * xw);
  uint64_t *exp = dev.arena.take<uint64_t>((size_t)s.W * s.J * 4 * C::NP64);
  size_t cub = 0, cub2 = 0;
  const int kbits = key_bits(nb);
  ZK_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, cub, keys, skeys, vals, list, (int)maxent, 0, kbits, st));
  ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub2, flags, pos, (int)ns0, st));
  if (cub2 > cub) cub = cub2;
  void *cubtmp = dev.arena.take<char>(cub);

  hipLaunchKernelGGL(k_points_int<C>, dim3(div_up(n, 256)), dim3(256), 0, st, d_pt, n, pts_int);
  ZK_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_digits<C>, dim3(div_up(n, 256)), dim3(256), 0, st, d_sc, n, nl, mont ? 1 : 0, c, s.W,
                     keys, vals);
  ZK_CHECK(hipGetLastError());
  ZK_CHECK(hipcub::DeviceRadixSort::SortPairs(cubtmp, cub, keys, skeys, vals, list, (int)maxent, 0, kbits, st));
  hipLaunchKernelGGL(k_offsets, dim3(div_up(nb + 1, 256)), dim3(256), 0, st, skeys, (uint32_t)maxent,
                     (uint32_t)nb, offsets);
  ZK_CHECK(hipGetLastError());

  KernelTimer &kt = dominant_timer();
  {
    if (kt.enabled) ZK_CHECK(hipEventRecord(kt.ev0, st));
    // upper bound on the chunk count; threads past offsets[nb] only clear their item slots
    hipLaunchKernelGGL(k_accum<C>, dim3(div_up(ns0 / 2, 256)), dim3(256), 0, st, pts_int, list, offsets,
                       (uint32_t)nb, s.CH, buckets, ikeys0, ivals0, (uint32_t)ns0);
    ZK_CHECK(hipGetLastError());
    if (kt.enabled) ZK_CHECK(hipEventRecord(kt.ev1, st));
  }
  // stitch levels: compact the partial items, sum them per bucket, repeat
  {
    const uint32_t *inK = ikeys0, *inV = ivals0;
    const uint32_t *inCount = nullptr;  // level 0: every slot is examined
    size_t slots = ns0;
    uint32_t *outK = okA, *outV = ovA, *altK = okB, *altV = ovB;
    for (;;) {
      hipLaunchKernelGGL(k_item_flags, dim3(div_up(slots, 256)), dim3(256), 0, st, inK, inCount, (uint32_t)slots,
                         (uint32_t)nb, flags);
      ZK_CHECK(hipGetLastError());
      size_t cb = cub;
      ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(cubtmp, cb, flags, pos, (int)slots, st));
      hipLaunchKernelGGL(k_item_compact<C>, dim3(div_up(slots, 256)), dim3(256), 0, st, inK, inV, flags, pos,
                         (uint32_t)slots, ckeys, cvals, ccount);
      ZK_CHECK(hipGetLastError());
      const bool final_level = slots <= (size_t)s.SCH;  // all items fit one chunk: everything completes
      const size_t nout = final_level ? 2 : 2 * ((slots + s.SCH - 1) / s.SCH);
      hipLaunchKernelGGL(k_stitch<C>, dim3(div_up(nout / 2, 256)), dim3(256), 0, st, ckeys, cvals, ccount,
                         (uint32_t)nb, s.SCH, buckets, outK, outV, (uint32_t)nout);
      ZK_CHECK(hipGetLastError());
      if (final_level) break;
      // most levels past the first are empty for well-spread scalars: check and stop
      uint32_t *hc = reinterpret_cast<uint32_t *>(dev.host_staging(4));
      ZK_CHECK(hipMemcpyAsync(hc, ccount, 4, hipMemcpyDeviceToHost, st));
      ZK_CHECK(hipStreamSynchronize(st));
      if (*hc <= (uint32_t)s.SCH) break;  // this level's stitch had one chunk: all complete
      inK = outK; inV = outV; inCount = nullptr; slots = nout;
      uint32_t *tk = outK, *tv = outV;
      outK = altK; outV = altV; altK = tk; altV = tv;
    }
  }
  hipLaunchKernelGGL(k_seg<C>, dim3(div_up((size_t)s.W * s.S, 256)), dim3(256), 0, st, buckets, offsets, s.W, s.B,
                     s.L, T, R);
  ZK_CHECK(hipGetLastError());
  const int ngrp = s.W * s.J;
  {
    const size_t lds = (size_t)(JT / 2) * xyzz_words<F>() * 4;
    ZK_CHECK(hipFuncSetAttribute((const void *)k_jobsum<C>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_jobsum<C>, dim3(ngrp), dim3(JT), lds, st, T, R, s.S, s.logS, P0);
    ZK_CHECK(hipGetLastError());
  }
  uint32_t *src = P0;
  hipLaunchKernelGGL(k_export<C>, dim3(div_up(ngrp, 64)), dim3(64), 0, st, src, ngrp, exp);
  ZK_CHECK(hipGetLastError());
  const size_t expbytes = (size_t)ngrp * 4 * C::NP64 * 8;
  uint64_t *h = reinterpret_cast<uint64_t *>(dev.host_staging(expbytes));
  ZK_CHECK(hipMemcpyAsync(h, exp, expbytes, hipMemcpyDeviceToHost, st));
  ZK_CHECK(hipStreamSynchronize(st));
  if (kt.enabled) {
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
