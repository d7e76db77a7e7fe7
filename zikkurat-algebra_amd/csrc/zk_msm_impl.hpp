#pragma once
// zk_msm_impl.hpp -- (template bodies; instantiated in zk_msm.hip / zk_msm_g2.hip) Pippenger bucket MSM for G1 (BN128 and BLS12-381) on gfx950.
//
// Replaces <C>_G1_proj_MSM_std_coeff_proj_out_variable (bls12_381_G1_proj.c:507-587)
// and its callers (:597-670).  Same mathematical result (sum_i k_i * P_i with the
// 256-bit scalars used verbatim -- no reduction mod r, no GLV, so the result is
// identical for points outside the order-r subgroup too), computed with
// a GPU-shaped schedule:
//
//   0. k_points_int   affine points -> internal radix (one product per coordinate)
//   1. k_digits       scalar (Montgomery -> standard by REDC, Fr_mont.c:330-335) ->
//                     signed c-bit digits of every window
//      k_coarse/k_fine  bucket sort of the (window, point) entries: two-level LDS counting
//                     sort (coarse bins, then the fine buckets of each bin) -> bucket
//                     offsets + bucket-ordered list of point index | sign;
//                     bucket rank = window * B + |digit| - 1
//   2. k_accum        balanced bucket accumulation: every thread adds exactly CH
//                     consecutive list entries (mixed XYZZ += affine adds), flushing
//                     complete runs to their bucket and boundary runs as partial items
//   3. k_stitch_blk   partial items are compacted and summed per bucket by block-level
//      k_stitch_raw   segmented scans (level 0: device-wide compaction + k_stitch_blk; the
//                     few-slot levels after it: one k_stitch_raw each, block-local packing and
//                     a segmented tree), level after level: no serial loop anywhere, so
//                     skewed scalars (all equal, carry windows) stay fast
//   4. k_ysum(2)      digit split of the bucket weights into plain sums Y0, Y1
//   5. k_jobsum_blk   the weighted Y sums by bit jobs (a block of quad-cooperative additions per job)
//   6. host           Horner over the power-of-two exponents and the windows
// Windows are processed in groups when W n exceeds one pass's sort capacity.
//
// Every phase is wide (>= ~1e5 threads at 2^20) except the last tiny levels: a lone
// wavefront's serial chain of 381-bit point adds is slow on CDNA4, so the
// deep-but-narrow tail runs on the host (step 6).
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>
#include "zk_curve.hpp"
#include "zk_quad.hpp"
#include "zk_host.hpp"
#include "zk_runtime.hpp"
#include "zk_msm.hpp"
#include "zk_ntt.hpp"

namespace zk {

// 0. affine points: reference form -> internal form (once per call).  The block's 256 points
// are one contiguous span on both sides (96 / 64 B in, 128 / 96 B out): they are staged through
// LDS so that every HBM access is a 16-B-per-lane run over consecutive lanes (a thread reading
// or writing its own point alone touches 64 separate rows per wavefront instruction).
// BLS12-381 2^20: 0.070-0.078 -> 0.061-0.067 ms (profiles/r03aa_points_coarse_ab.txt).
template <class C>
__global__ void __launch_bounds__(256) k_points_int(const uint64_t *__restrict__ pts, int n,
                                                    uint32_t *__restrict__ out) {
  using F = typename C::Fp;
  constexpr int IN4 = 2 * F::N64 * 8 / 16;  // 16-B chunks per input point (6 / 4)
  constexpr int OUT4 = aff_words<F>() / 4;  // 16-B chunks per output point (8 / 6)
  constexpr int ST4 = IN4 > OUT4 ? IN4 : OUT4;
  __shared__ uint4 stage[256 * ST4];
  const int t = threadIdx.x;
  const int p0 = blockIdx.x * 256;
  const int np = min(256, n - p0);
  const uint4 *src = reinterpret_cast<const uint4 *>(pts + (size_t)p0 * 2 * F::N64);
  for (int j = t; j < np * IN4; j += 256) stage[j] = src[j];
  __syncthreads();
  uint32_t res[aff_words<F>()];
  if (t < np) {
    uint64_t in[2 * F::N64];
    const uint64_t *me = reinterpret_cast<const uint64_t *>(&stage[t * IN4]);
#pragma unroll
    for (int j = 0; j < 2 * F::N64; j++) in[j] = me[j];
    aff_ref_to_int<F>(res, in);
  }
  __syncthreads();
  if (t < np) {
    uint4 *me = &stage[t * OUT4];
#pragma unroll
    for (int j = 0; j < OUT4; j++) me[j] = make_uint4(res[4 * j], res[4 * j + 1], res[4 * j + 2], res[4 * j + 3]);
  }
  __syncthreads();
  uint4 *dst = reinterpret_cast<uint4 *>(out + (size_t)p0 * aff_words<F>());
  for (int j = t; j < np * OUT4; j += 256) dst[j] = stage[j];
}

// ---------------------------------------------------------------------------
// 1. Signed c-bit digits of one scalar, window by window.
//    Scalar i is the integer in limbs [loff, loff + nread) of its `stride`-limb row (nread
//    <= 4; longer std scalars are split into 256-bit slices by msm_g1), converted from
//    Montgomery form first when `mont` (REDC, Fr_mont.c:330-335).  A digit is raw - 2^c
//    (negative) when raw = bits + carry > 2^(c-1), so |digit| <= 2^(c-1) = B.
template <class C>
struct DigitStream {
  uint32_t k[9];
  uint32_t carry;
  __device__ __forceinline__ void load(const uint64_t *__restrict__ scalars, int i, int stride, int loff, int nread,
                                       int mont) {
    using Fr = typename C::Fr;
#pragma unroll
    for (int j = 0; j < 4; j++) {  // fewer than 4 limbs: zero-extended
      const uint64_t w = (j < nread) ? scalars[(size_t)i * stride + loff + j] : 0;
      k[2 * j] = (uint32_t)w;
      k[2 * j + 1] = (uint32_t)(w >> 32);
    }
    k[8] = 0;
    if (mont) {
      Fe<Fr> s, t;
      fe_unpack(s, k);
      fe_ref_to_std(t, s);
      fe_pack(k, t);
    }
    carry = 0;
  }
  // next window's |digit| (0 .. B) and sign (0x80000000 for negative)
  __device__ __forceinline__ uint32_t next(int c, uint32_t &sign) {
    const uint32_t full = 1u << c, B = full >> 1;
    const uint32_t raw = (k[0] & (full - 1)) + carry;
#pragma unroll
    for (int j = 0; j < 8; j++) k[j] = __builtin_amdgcn_alignbit(k[j + 1], k[j], c);  // >>= c (c < 32)
    if (raw > B) {  // negative digit raw - 2^c (zero when raw == 2^c)
      sign = 0x80000000u;
      carry = 1;
      return full - raw;
    }
    sign = 0;
    carry = 0;
    return raw;
  }
};

// 2. Bucket sort of the (window, point) entries.  Buckets are ranked window-major:
//    rank = (w - wbase) * B + |digit| - 1 over the windows [wbase, wbase + Wg) of this
//    pipeline pass (B = 2^(c-1) buckets per window); zero digits belong to no bucket.  The
//    result is the bucket offsets (nb + 1 entries, offsets[nb] = total) and the
//    bucket-ordered list of point index | sign << 31 (n < 2^31 by the C ABI's int).
//
//    Two-level counting sort, every write coalesced: k_digits writes one u32 per entry
//    (|digit| | sign, window-major).  Level 1 sorts by COARSE bin = (|digit| - 1) >> s
//    (MSM_COARSE_BINS bins per window): k_coarse<false> counts each workgroup's entries per
//    coarse bin in LDS into a (window, bin, workgroup) matrix, an exclusive scan of that
//    matrix is every workgroup's slot range in every bin, k_coarse<true> scatters
//    (value, fine index) in runs of ~M / 256 entries per bin.  Level 2 (k_fine): one
//    workgroup per coarse bin counts its 2^s fine buckets in LDS, writes their offsets and
//    places its entries inside the bin's own small output range (lines merge in L2).
//    A single-level scatter of 4-B entries to random buckets measured 600 MB of HBM
//    writes for 67 MB of entries at BLS12-381 2^20 (profiles/r02j_pmc.json).  The order
//    inside a bucket depends on atomic timing; bucket sums are group sums, so the
//    canonical result does not.
template <class C>
__global__ void __launch_bounds__(256) k_digits(const uint64_t *__restrict__ scalars, int n, int plo, int phi,
                                                int stride, int loff, int nread, int mont, int c, int wbase, int Wg,
                                                uint32_t *__restrict__ out) {
  const int i = plo + blockIdx.x * blockDim.x + threadIdx.x;  // points [plo, phi) of n
  if (i >= phi) return;
  DigitStream<C> ds;
  ds.load(scalars, i, stride, loff, nread, mont);
  for (int w = 0; w < wbase + Wg; w++) {
    uint32_t sign;
    const uint32_t mag = ds.next(c, sign);
    if (w < wbase) continue;
    out[(size_t)(w - wbase) * n + i] = mag | sign;
  }
}

constexpr int MSM_COARSE_BINS = 256;  // coarse bins per window (fewer when B is smaller)
#ifndef ZK_SORT_CHUNK
#define ZK_SORT_CHUNK 4096
#endif
constexpr int SORT_CHUNK = ZK_SORT_CHUNK;  // level-1 entries staged in LDS at a time (16 per thread)
constexpr int COUNT_ILP = 8;          // loads in flight per thread in the level-1 / 1.5 counting passes
constexpr int FINE_LDS_MAX = 8192;    // level-2 bins up to this size are placed in LDS
constexpr int FINE_LDS_BYTES = 150 * 1024;  // dynamic LDS of k_fine: 2^s counters + staging
static int fine_stage_cap(int s) {
  const int cap = (FINE_LDS_BYTES - (4 << s)) / 4;
  return cap < FINE_LDS_MAX ? cap : FINE_LDS_MAX;
}

// block-wide exclusive scan of one value per thread (256 threads); returns the thread's
// exclusive prefix, *total the sum
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t *tmp, uint32_t *total) {
  const int t = threadIdx.x;
  tmp[t] = v;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {
    const uint32_t o = t >= d ? tmp[t - d] : 0;
    __syncthreads();
    tmp[t] += o;
    __syncthreads();
  }
  const uint32_t incl = tmp[t];
  *total = tmp[255];
  __syncthreads();
  return incl - v;
}

// Level 1.  Workgroup (window w = blockIdx.y, entries [blockIdx.x * M, +M)).  Counting
// pass: per-bin counts into cnt[(w * nbins + bin) * nwg + wg].  Scatter pass: the scanned
// matrix gives this workgroup's first slot in every bin; entries go through LDS in chunks,
// sorted by bin there, so every bin's run leaves as consecutive lanes' stores.
template <bool SCATTER>
__global__ void __launch_bounds__(256) k_coarse(const uint32_t *__restrict__ dig, int n, int plo, int phi, int M,
                                                int s, int nbins, uint32_t *__restrict__ cnt,
                                                uint32_t *__restrict__ tmpv, uint16_t *__restrict__ tmpf) {
  __shared__ uint32_t hist[MSM_COARSE_BINS], lofs[MSM_COARSE_BINS], gcur[MSM_COARSE_BINS], scan_tmp[256];
  __shared__ uint32_t sv[SORT_CHUNK], sk[SORT_CHUNK];
  // window w = blockIdx.y over the points [plo, phi) of one split (tmpv / tmpf: that split's region)
  const uint32_t w = blockIdx.y, g = blockIdx.x, nwg = gridDim.x;
  const int t = threadIdx.x;
  const int e0 = plo + (int)g * M, e1 = min(phi, e0 + M);
  const uint32_t *d = dig + (size_t)w * n;
  uint32_t *cw = cnt + (size_t)w * nbins * nwg + g;
  if (!SCATTER) {
    if (w == 0 && g == 0 && t == 0) cnt[(size_t)gridDim.y * nbins * nwg] = 0;  // the scan's total slot
    for (int b = t; b < nbins; b += 256) hist[b] = 0;
    __syncthreads();
    for (int b0 = e0; b0 < e1; b0 += 256 * COUNT_ILP) {  // COUNT_ILP digits in flight per thread
      uint32_t mag[COUNT_ILP];
#pragma unroll
      for (int j = 0; j < COUNT_ILP; j++) {
        const int e = b0 + j * 256 + t;
        mag[j] = e < e1 ? d[e] & 0x7fffffffu : 0u;
      }
#pragma unroll
      for (int j = 0; j < COUNT_ILP; j++)
        if (mag[j]) atomicAdd(&hist[(mag[j] - 1) >> s], 1u);
    }
    __syncthreads();
    for (int b = t; b < nbins; b += 256) cw[(size_t)b * nwg] = hist[b];
    return;
  }
  for (int b = t; b < nbins; b += 256) gcur[b] = cw[(size_t)b * nwg];
  const uint32_t fmask = (1u << s) - 1;
  constexpr int PER = SORT_CHUNK / 256;
  for (int c0 = e0; c0 < e1; c0 += SORT_CHUNK) {
    for (int b = t; b < nbins; b += 256) hist[b] = 0;
    __syncthreads();
    uint32_t val[PER], key[PER], rank[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int e = c0 + k * 256 + t;
      const uint32_t v = e < e1 ? d[e] : 0u;
      const uint32_t mag = v & 0x7fffffffu;
      key[k] = 0xffffffffu;
      if (mag) {
        const uint32_t b = (mag - 1) >> s;
        key[k] = (b << 16) | ((mag - 1) & fmask);
        val[k] = (uint32_t)e | (v & 0x80000000u);
        rank[k] = atomicAdd(&hist[b], 1u);
      }
    }
    __syncthreads();
    uint32_t tot;
    const uint32_t h = t < nbins ? hist[t] : 0u;
    const uint32_t ex = block_excl_scan256(h, scan_tmp, &tot);
    if (t < nbins) lofs[t] = ex;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (key[k] != 0xffffffffu) {
        const uint32_t p = lofs[key[k] >> 16] + rank[k];
        sv[p] = val[k];
        sk[p] = key[k];
      }
    }
    __syncthreads();
    for (uint32_t i = t; i < tot; i += 256) {
      const uint32_t k = sk[i], b = k >> 16;
      const uint32_t slot = gcur[b] + (i - lofs[b]);
      tmpv[slot] = sv[i];
      tmpf[slot] = (uint16_t)(k & 0xffffu);
    }
    __syncthreads();
    if (t < nbins) gcur[t] += h;
  }
}

// Level 1.5 (large inputs, whose coarse bins outgrow level 2's LDS staging: BLS12-381 2^26 at
// c = 20 has bins of ~2^18 entries against 8192, and scattering them straight to 2048 fine
// buckets cost 24 ms of a 165 ms MSM, profiles/r04v_*): every coarse bin q is split by the top
// bits of its fine index into nsub sub-bins with the level-1 machinery -- workgroup g of the bin
// takes its share of the bin's range, per-workgroup LDS histograms go to a (bin, sub-bin,
// workgroup) matrix, an exclusive scan of it gives every run's slot, the scatter goes through LDS
// in chunks and leaves in runs.  Level 2 then sorts sub-bins of ~cap / 2 entries in LDS.  Sub-bin
// q' = q nsub + sub owns fine buckets [sub F', (sub + 1) F') of bin q (F' = F / nsub), so level 2's
// offsets[q' F' + f'] are exactly offsets[q F + f]: the layout downstream is unchanged.
template <bool SCATTER>
__global__ void __launch_bounds__(256) k_split(const uint32_t *__restrict__ coff, int nwg, int s2sh, int nsub,
                                               uint32_t *__restrict__ mat, const uint32_t *__restrict__ tmpv,
                                               const uint16_t *__restrict__ tmpf, uint32_t *__restrict__ outv,
                                               uint16_t *__restrict__ outf) {
  __shared__ uint32_t hist[256], lofs[256], gcur[256], scan_tmp[256];
  __shared__ uint32_t sv[SORT_CHUNK], sk[SORT_CHUNK];
  const uint32_t q = blockIdx.y, g = blockIdx.x, nwg2 = gridDim.x;
  const int t = threadIdx.x;
  const uint32_t start = coff[(size_t)q * nwg], end = coff[(size_t)(q + 1) * nwg];
  const uint32_t len = end - start, per = (len + nwg2 - 1) / nwg2;
  const uint32_t e0 = start + min(len, g * per), e1 = start + min(len, (g + 1) * per);
  // mat: the (bin, sub-bin, workgroup) counts (count pass) or their exclusive scan (scatter pass);
  // the bin's range always comes from the level-1 scan coff
  uint32_t *cw = mat + (size_t)q * nsub * nwg2 + g;
  const uint32_t lmask = (1u << s2sh) - 1;
  if (!SCATTER) {
    if (q == 0 && g == 0 && t == 0) mat[(size_t)gridDim.y * nsub * nwg2] = 0;  // the scan's total slot
    for (int b = t; b < nsub; b += 256) hist[b] = 0;
    __syncthreads();
    // COUNT_ILP keys in flight per thread before their LDS increments: with one load per
    // iteration the pass was latency-bound (2 B per lane: 0.58 ms at BLS12-381 2^23, ~0.4 TB/s)
    for (uint32_t b0 = e0; b0 < e1; b0 += 256 * COUNT_ILP) {
      uint32_t k[COUNT_ILP];
#pragma unroll
      for (int j = 0; j < COUNT_ILP; j++) {
        const uint32_t e = b0 + j * 256 + t;
        k[j] = e < e1 ? (uint32_t)tmpf[e] : 0xffffffffu;
      }
#pragma unroll
      for (int j = 0; j < COUNT_ILP; j++)
        if (k[j] != 0xffffffffu) atomicAdd(&hist[k[j] >> s2sh], 1u);
    }
    __syncthreads();
    for (int b = t; b < nsub; b += 256) cw[(size_t)b * nwg2] = hist[b];
    return;
  }
  for (int b = t; b < nsub; b += 256) gcur[b] = cw[(size_t)b * nwg2];
  constexpr int PER = SORT_CHUNK / 256;
  for (uint32_t c0 = e0; c0 < e1; c0 += SORT_CHUNK) {
    for (int b = t; b < nsub; b += 256) hist[b] = 0;
    __syncthreads();
    uint32_t val[PER], key[PER], rank[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t e = c0 + k * 256 + t;
      key[k] = 0xffffffffu;
      if (e < e1) {
        key[k] = tmpf[e];
        val[k] = tmpv[e];
      }
    }
#pragma unroll
    for (int k = 0; k < PER; k++)
      if (key[k] != 0xffffffffu) rank[k] = atomicAdd(&hist[key[k] >> s2sh], 1u);
    __syncthreads();
    uint32_t tot;
    const uint32_t h = t < nsub ? hist[t] : 0u;
    const uint32_t ex = block_excl_scan256(h, scan_tmp, &tot);
    if (t < nsub) lofs[t] = ex;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (key[k] != 0xffffffffu) {
        const uint32_t p = lofs[key[k] >> s2sh] + rank[k];
        sv[p] = val[k];
        sk[p] = key[k];
      }
    }
    __syncthreads();
    for (uint32_t i = t; i < tot; i += 256) {
      const uint32_t k = sk[i], b = k >> s2sh;
      const uint32_t slot = gcur[b] + (i - lofs[b]);
      outv[slot] = sv[i];
      outf[slot] = (uint16_t)(k & lmask);
    }
    __syncthreads();
    if (t < nsub) gcur[t] += h;
  }
}

// LDS counter increments with wavefront aggregation: lanes that hit the same counter are served
// by ONE atomic (leader = the lowest such lane) for up to 4 keys with >= 4 lanes each; the rest
// use plain per-lane atomics.  A bin whose entries share a few fine buckets -- binary 0/1 scalar
// vectors (one bucket per window), or the carry-only top window of c = 15 / 17 / 18 -- otherwise
// serialises 64 same-address LDS atomics per wavefront instruction.  Uniform inputs cost one
// ballot round (the first key has 1-2 lanes).  lds_count_agg: counting only (no return value).
template <bool RET>
__device__ __forceinline__ uint32_t lds_inc_agg(uint32_t *ctr, uint32_t key, bool active) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1;
  uint32_t r = 0;
  bool todo = active;
  for (int it = 0; it < 4; it++) {
    const uint64_t m = __ballot(todo);
    if (m == 0) break;
    const int leader = __ffsll((unsigned long long)m) - 1;
    const uint32_t lk = (uint32_t)__builtin_amdgcn_readlane((int)key, leader);  // leader is wavefront-uniform
    const bool mine = todo && key == lk;
    const uint64_t same = __ballot(mine);
    const int cnt = __popcll(same);
    if (cnt < 4) break;
    if (RET) {
      uint32_t base = 0;
      if ((int)lane == leader) base = atomicAdd(&ctr[lk], (uint32_t)cnt);
      base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
      if (mine) r = base + (uint32_t)__popcll(same & below);
    } else if ((int)lane == leader) {
      atomicAdd(&ctr[lk], (uint32_t)cnt);
    }
    if (mine) todo = false;
  }
  if (todo) {
    if (RET) r = atomicAdd(&ctr[key], 1u);
    else atomicAdd(&ctr[key], 1u);
  }
  return r;
}

// block-wide exclusive scan of one value per thread (BS threads, BS / 64 wavefronts): wavefront
// scans by DPP-free shuffles, then the wavefront totals
template <int BS>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *wtot, uint32_t *total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)x, d, 64);
    if (lane >= d) x += o;
  }
  if (lane == 63) wtot[w] = x;
  __syncthreads();
  uint32_t off = 0, all = 0;
#pragma unroll
  for (int k = 0; k < BS / 64; k++) {
    off += k < w ? wtot[k] : 0u;
    all += wtot[k];
  }
  *total = all;
  __syncthreads();
  return off + x - v;
}

// Level 2.  Workgroup (BS threads) = coarse bin q = w * nbins + b, entries [coff[q * nwg], next
// bin's start) of the level-1 order; 2^s fine buckets (dynamic LDS: 4 B counters, then the
// staging area).  A bin of at most `cap` entries is placed in LDS and leaves as one contiguous
// run; a larger one (skewed scalars) is scattered directly.  Every thread keeps FINE_ILP loads in
// flight and the counter updates are wavefront-aggregated (lds_inc_agg): a skewed bin is walked
// by ONE workgroup, which was latency-bound at 256 threads and one load each: with 1024 threads
// from 2^20 points per window (bins of >= 4096 entries), binary 0/1 scalars at BLS12-381 2^20 sort
// in 0.54 vs 1.16 ms, c = 17 at 2^22 in 3.1 vs 7.3 ms, c = 16 at 2^22 in 0.97 vs 1.23 ms.  Below
// that the round-2 shape (256 threads, one load each, plain atomics): the wide block lost 50-60 us
// at 2^16 and the aggregation / 4-deep loads at 256 threads ~0.1 ms at 2^18
// (profiles/r03s_fine_sort_ab.txt, profiles/r03t_fine_sort_ab.txt).
template <int FINE_BS, int FINE_ILP, bool AGG>
static __global__ void __launch_bounds__(FINE_BS) k_fine(const uint32_t *__restrict__ coff, int nwg, uint32_t nq,
                                                         int s, int cap, const uint32_t *__restrict__ tmpv,
                                                         const uint16_t *__restrict__ tmpf,
                                                         uint32_t *__restrict__ list, uint32_t *__restrict__ offsets,
                                                         uint32_t base) {
  // tmpv / tmpf / list point at this split's region, which starts at list position `base`:
  // the offsets written are absolute list positions
  extern __shared__ uint32_t fh[];
  __shared__ uint32_t wtot[FINE_BS / 64];
  const int F = 1 << s, t = threadIdx.x;
  uint32_t *sv = fh + F;
  const uint32_t q = blockIdx.x;
  const uint32_t start = coff[(size_t)q * nwg];
  const uint32_t end = coff[(size_t)(q + 1) * nwg];  // the matrix carries one extra entry: the total
  const bool staged = end - start <= (uint32_t)cap;
  constexpr uint32_t STEP = FINE_BS * FINE_ILP;
  for (int f = t; f < F; f += FINE_BS) fh[f] = 0;
  __syncthreads();
  for (uint32_t e0 = start; e0 < end; e0 += STEP) {  // block-uniform trip count (wavefront ballots inside)
    uint32_t k[FINE_ILP];
#pragma unroll
    for (int j = 0; j < FINE_ILP; j++) {
      const uint32_t e = e0 + j * FINE_BS + t;
      k[j] = e < end ? tmpf[e] : 0u;
    }
#pragma unroll
    for (int j = 0; j < FINE_ILP; j++) {
      const bool act = e0 + j * FINE_BS + t < end;
      if (AGG) lds_inc_agg<false>(fh, k[j], act);
      else if (act) atomicAdd(&fh[k[j]], 1u);
    }
  }
  __syncthreads();
  // exclusive scan of the F counters: thread t owns the contiguous span [t * per, +per)
  const int per = (F + FINE_BS - 1) / FINE_BS;
  uint32_t sum = 0;
  for (int j = 0; j < per; j++) {
    const int f = t * per + j;
    if (f < F) sum += fh[f];
  }
  uint32_t tot;
  uint32_t run = block_excl_scan<FINE_BS>(sum, wtot, &tot);
  for (int j = 0; j < per; j++) {
    const int f = t * per + j;
    if (f < F) {
      const uint32_t h = fh[f];
      fh[f] = staged ? run : start + run;
      offsets[(size_t)q * F + f] = base + start + run;
      run += h;
    }
  }
  if (q == nq - 1 && t == 0) offsets[(size_t)nq * F] = base + end;
  __syncthreads();
  for (uint32_t e0 = start; e0 < end; e0 += STEP) {
    uint32_t k[FINE_ILP], v[FINE_ILP];
#pragma unroll
    for (int j = 0; j < FINE_ILP; j++) {
      const uint32_t e = e0 + j * FINE_BS + t;
      k[j] = e < end ? tmpf[e] : 0u;
      v[j] = e < end ? tmpv[e] : 0u;
    }
#pragma unroll
    for (int j = 0; j < FINE_ILP; j++) {
      const bool act = e0 + j * FINE_BS + t < end;
      const uint32_t slot = AGG ? lds_inc_agg<true>(fh, k[j], act) : (act ? atomicAdd(&fh[k[j]], 1u) : 0u);
      if (act) {
        if (staged) sv[slot] = v[j];
        else list[slot] = v[j];
      }
    }
  }
  if (staged) {
    __syncthreads();
    for (uint32_t i = t; i < end - start; i += FINE_BS) list[start + i] = sv[i];
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

// 4. level-0 balanced accumulation: thread t owns list entries [t*CH, min((t+1)*CH, total)).
//    Runs of one bucket that lie entirely inside the chunk are written straight to
//    buckets[b]; a run that crosses the chunk boundary (the chunk's first and/or last run)
//    becomes a "partial item" (key b, XYZZ sum) in slot 2t / 2t+1 of the item arrays.
//    Item slots that stay empty carry key = nb (dropped by the compaction).
//
//    The next entry's point is gathered straight into LDS by global_load_lds (16 B per lane
//    per instruction, lane-linear image [chunk][lane][16 B] per wave) while the current
//    mixed add runs, so the prefetch costs no VGPRs (the 254-bit madd fits 3 waves per SIMD;
//    the 381-bit one stays at 2: forced to 3 it spills ~56 VGPRs inside the loop, measured
//    3.12 vs 2.56 ms at 2^20).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

#ifndef ZK_ACCUM_WAVES14
#define ZK_ACCUM_WAVES14 2  // the 381-bit madd (A/B hook: 3 spilled ~56 VGPRs in round 2)
#endif
#ifndef ZK_ACCUM_WAVES20
#define ZK_ACCUM_WAVES20 2  // BN254 G2: F2<BN_Fp>, 2 x 9 limbs (N = 18, i.e. 14 < N < 28); the macro keeps its old name
#endif
template <class F>
struct AccumOcc {  // minimum waves per SIMD k_accum is compiled for
  // 254-bit lazy madd: 3 waves (153 VGPRs); at 4 it spills 30 VGPRs inside the loop (1.49 vs
  // 1.44 ms at BN128 2^20, profiles/r02at_bn128_lazy_madd.txt)
  static constexpr int waves = F::N >= 28 ? 1 : (F::N > 14 ? ZK_ACCUM_WAVES20 : (F::N == 14 ? ZK_ACCUM_WAVES14 : 3));
};

template <class C>
__global__ void __launch_bounds__(256, AccumOcc<typename C::Fp>::waves)
    k_accum(const uint32_t *__restrict__ points, const uint32_t *__restrict__ list,
            const uint32_t *__restrict__ offsets, uint32_t nb, int CH, uint32_t W, uint32_t B,
            uint32_t *__restrict__ buckets, uint32_t *__restrict__ ikeys, uint32_t *__restrict__ ivals,
            uint32_t nslots, const uint8_t *__restrict__ filled) {
  using F = typename C::Fp;
  constexpr int AW = aff_words<F>();  // u32 per internal-form point (multiple of 8)
  constexpr int NCH = AW / 4;         // 16-B chunks per point
  __shared__ uint4 stage[4][NCH][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  // this launch's list range [offsets[0], offsets[nb]) (one split of a split pipeline)
  const uint32_t total = offsets[nb];
  const uint32_t cs = offsets[0] + t * (uint32_t)CH;
  const bool active = 2 * t < nslots && cs < total;
  uint32_t k0 = nb, k1 = nb;  // item keys of slots 2t, 2t+1
  uint32_t tail_b = nb, tail_slot = 0;  // the chunk's right-partial last run (began in the chunk), in acc
  bool head_end = false;                // slot 2t holds a head run that ends inside the chunk
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  // gathers the point of list entry `c` (index | sign) into this lane's LDS image
  auto prefetch = [&](uint32_t c) {
    const uint32_t *src = points + (size_t)(c & 0x7fffffffu) * AW;
#pragma unroll
    for (int j = 0; j < NCH; j++)
      __builtin_amdgcn_global_load_lds((glb_void_t *)(src + 4 * j), (lds_void_t *)&stage[wave][j][0], 16, 0, 0);
  };
  auto read_point = [&](Aff<F> &P) {
    uint32_t w[AW];
#pragma unroll
    for (int j = 0; j < NCH; j++) {
      const uint4 v = stage[wave][j][lane];
      w[4 * j] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < F::N; i++) {
      P.x.v[i] = w[i];
      P.y.v[i] = w[F::SN + i];
    }
  };
  // a run that starts in this chunk begins from the bucket's sum over the earlier splits
  // (filled), else from infinity; a run continuing from an earlier chunk starts empty (its
  // owner carries the earlier value)
  auto start_run = [&](uint32_t b) {
    if (filled && filled[b]) xyzz_load(acc, buckets + (size_t)b * xyzz_words<F>());
    else xyzz_set_inf(acc);
  };
  if (active) {
    const uint32_t ce = min(total, cs + (uint32_t)CH);
    uint32_t b = bucket_of(offsets, nb, cs);
    uint32_t bbeg = offsets[b], bend = offsets[b + 1];
    if (bbeg >= cs) start_run(b);
    uint32_t bnext = offsets[min(b + 2, nb)];  // end of the next bucket, loaded ahead
    bool first_run = true;
    // Flushes store the accumulator LAZILY (X < 14p for the 381-bit madd): every
    // consumer (xyzz_add / xyzz_dbl / the job sums' export) takes X and Y only into products, which
    // accept those values.  A settle here would cost two products per flush, paid by the
    // whole wavefront whenever any lane flushes (runs average 32 entries at 2^20).
    // Pipeline: the point of entry e+1 lands in LDS and the list index of entry e+2 in a
    // register while the madd of entry e runs (clamped to the chunk's last entry, so every
    // load is in bounds); infinity test and negation happen at use.
    const uint32_t last = ce - 1;
    uint32_t c0 = list[cs], c1 = list[min(cs + 1, last)];
    prefetch(c0);
    for (uint32_t e = cs; e < ce; e++) {
      Aff<F> P;
      read_point(P);  // waits for the gather of entry e
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS image read out before it is refilled
      prefetch(c1);
      const uint32_t c2 = list[min(e + 2, last)];
      if (e >= bend) {  // run of bucket b ends inside the chunk
        if (first_run && bbeg < cs) {
          xyzz_store(ivals + (size_t)(2 * t) * xyzz_words<F>(), acc);
          k0 = b;
        } else {
          xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);
        }
        first_run = false;
        do {  // next non-empty bucket; the next boundary is already in a register
          b++;
          bbeg = bend;
          bend = bnext;
          bnext = offsets[min(b + 2, nb)];
        } while (bend <= e);
        start_run(b);
      }
      if (P.x.v[0] != 0xffffffffu) {  // affine infinity is skipped
        if (c0 & 0x80000000u) {
          Fe<F> ny;
          fe_neg(ny, P.y);
          P.y = ny;
        }
        xyzz_acc_aff(acc, P);
      }
      c0 = c1;
      c1 = c2;
    }
    // last run: partial if it started before the chunk or continues after it
    const bool lpart = bbeg < cs, rpart = bend > ce;
    if (rpart && !(first_run && lpart)) {  // began in this chunk, continues: kept for the merge below
      tail_b = b;
      tail_slot = first_run ? 2 * t : 2 * t + 1;
    } else if (lpart || rpart) {  // through the whole chunk, or a head that ends exactly at ce
      xyzz_store(ivals + (size_t)(2 * t) * xyzz_words<F>(), acc);
      k0 = b;
    } else {
      xyzz_store(buckets + (size_t)b * xyzz_words<F>(), acc);
    }
    head_end = k0 != nb && !(first_run && rpart);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last gather and the head flush have landed
  }
  // the head flushes (plain stores of the other lanes of this wavefront) are published before
  // the merge below reads them: release here, acquire before the reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  // Merge across the chunk boundary inside the wavefront: lane t's right-partial last run
  // and lane t+1's head run (flushed to slot 2t+2 during its loop) are the same bucket's run
  // exactly when the run crosses that boundary and ends in chunk t+1 -- one add completes
  // the bucket here instead of two items in the stitch (a run through whole chunks, and the
  // lane-63 boundary, stay items).  The head is read back at L2 (the other lane's store is
  // not in this CU's L1).
  const uint32_t nhead = (uint32_t)__shfl_down((int)(head_end ? k0 : nb), 1, 64);
  const bool merge = tail_b != nb && lane < 63 && nhead == tail_b;
  if (__any(merge)) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (merge) {
      const uint32_t *src = ivals + (size_t)(2 * t + 2) * xyzz_words<F>();
      uint32_t wds[xyzz_words<F>()];
#pragma unroll
      for (int i = 0; i < xyzz_words<F>(); i++) wds[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      Xyzz<F> o;
      xyzz_load(o, wds);
      xyzz_add(acc, o);
    }
  }
  if (tail_b != nb) {
    if (merge) {
      xyzz_store(buckets + (size_t)tail_b * xyzz_words<F>(), acc);
    } else {
      xyzz_store(ivals + (size_t)tail_slot * xyzz_words<F>(), acc);
      if (tail_slot == 2 * t) k0 = tail_b; else k1 = tail_b;
    }
  }
  if (__shfl_up((int)merge, 1, 64) && lane > 0) k0 = nb;  // this lane's head went into the lane before
  if (2 * t < nslots) {
    ikeys[2 * t] = k0;
    ikeys[2 * t + 1] = k1;
  }
}

// split pipelines: filled[b] = bucket b holds a sum (some split so far had entries for it)
static __global__ void __launch_bounds__(256) k_fill_mark(const uint32_t *__restrict__ off, uint32_t nb, int first,
                                                          uint8_t *__restrict__ filled) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint8_t f = off[b + 1] > off[b] ? 1 : 0;
  filled[b] = first ? f : (uint8_t)(filled[b] | f);
}

// 5a. compaction of the partial items (keys < nb), order preserving: scatter by a
//     prefix sum of the valid flags (scan done by hipCUB on `flags`)
static __global__ void __launch_bounds__(256) k_item_flags(const uint32_t *__restrict__ ikeys, const uint32_t *__restrict__ count,
                                                    uint32_t nslots_max, uint32_t nb, uint32_t *__restrict__ flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots_max) return;
  const uint32_t n = count ? *count : nslots_max;
  flags[i] = (i < n && ikeys[i] < nb) ? 1u : 0u;
}
// 5c. block stitch level: BS consecutive compacted items (sorted by key; payload e at
//     vals[idx[e]]) per workgroup, one per lane, summed per key by a segmented
//     Hillis-Steele scan through LDS (step d: lane t adds lane t-d when both hold the same
//     key); steps stop as soon as no lane of the block needs one, so short runs (the
//     common tail-of-one-chunk + head-of-the-next pairs) cost one step and a run of any
//     length shrinks BS-fold per level.  The last lane of each segment owns its sum: a
//     whole run goes to its bucket, a run cut by the block edge becomes an item of the
//     next level in slot 2 blk (the block's first segment, when its run started earlier
//     -- or when it is also the last one) or 2 blk + 1 (the last segment, when its run
//     continues), the same layout as k_stitch with SCH = BS.
#ifndef ZK_STITCH_RAW
// Stitch levels after the first: 1 = one k_stitch_raw launch per level (block-local packing,
// segmented tree reduction); 0 = device-wide compaction + k_stitch_blk as on level 0.  Level 0
// keeps the compaction either way: there most slots are empty, and k_stitch_raw over all of them
// (2048 blocks of 64 KB LDS at BLS12-381 2^20) measured 0.155 vs 0.067 ms for the whole stitch
// (profiles/r03h_stitch_raw_ab.txt)
#define ZK_STITCH_RAW 1
#endif
template <class C, int BS>
__global__ void __launch_bounds__(BS) k_stitch_blk(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ idx,
                                                   const uint32_t *__restrict__ vals,
                                                   const uint32_t *__restrict__ count, uint32_t nb, uint32_t W,
                                                   uint32_t B, uint32_t *__restrict__ buckets,
                                                   uint32_t *__restrict__ okeys, uint32_t *__restrict__ ovals,
                                                   uint32_t nout) {
  using F = typename C::Fp;
  constexpr int XW = xyzz_words<F>();
  __shared__ uint4 stitch_lds4[BS * XW / 4];  // [BS][XW] partial sums (64 KB + skey: > 64 KB LDS, gfx950)
  uint32_t *lv = reinterpret_cast<uint32_t *>(stitch_lds4);
  __shared__ uint32_t skey[BS];
  const uint32_t M = *count;
  const uint32_t t = threadIdx.x, blk = blockIdx.x;
  const uint32_t base = blk * BS;
  if (base >= M) {  // no items: clear this block's output slots
    if (t < 2 && 2 * blk + t < nout) okeys[2 * blk + t] = nb;
    return;
  }
  const uint32_t nv = min((uint32_t)BS, M - base);  // valid lanes
  const uint32_t j = base + t;
  const bool valid = t < nv;
  const uint32_t key = valid ? keys[j] : 0xffffffffu;
  skey[t] = key;
  Xyzz<F> acc;
  if (valid) xyzz_load(acc, vals + (size_t)idx[j] * XW);
  else xyzz_set_inf(acc);
  __syncthreads();
  for (uint32_t d = 1; d < nv; d <<= 1) {
    const bool need = valid && t >= d && skey[t - d] == key;
    if (!__syncthreads_or(need)) break;
    xyzz_store(lv + (size_t)t * XW, acc);
    __syncthreads();
    if (need) {
      Xyzz<F> o;
      xyzz_load(o, lv + (size_t)(t - d) * XW);
      xyzz_add_red(acc, o);
    }
    __syncthreads();
  }
  if (!valid) return;
  const bool seg_last = t == nv - 1 || skey[t + 1] != key;
  if (!seg_last) return;
  const bool touches_start = skey[0] == key;
  const bool touches_end = t == nv - 1;
  const bool cont_in = touches_start && base > 0 && keys[base - 1] == key;
  const bool cont_out = touches_end && base + nv < M && keys[base + nv] == key;
  if (!cont_in && !cont_out) {
    xyzz_store(buckets + (size_t)key * XW, acc);
  } else {
    xyzz_store(ovals + (size_t)(touches_start ? 2 * blk : 2 * blk + 1) * XW, acc);
  }
  const uint32_t item_key = (cont_in || cont_out) ? key : nb;
  if (touches_start) okeys[2 * blk] = item_key;
  if (touches_end) okeys[2 * blk + 1] = touches_start ? nb : item_key;
}

// 5c''. quad-cooperative form of k_stitch_blk (G1, level 0): 64 compacted items per 256-thread
//      block, one QUAD per item, so every Hillis-Steele step is one xyzz_add_quad (5 product
//      latencies) instead of a one-lane full add (14): the stitch is latency-bound (a few steps
//      per block at any size), and at small inputs it was the largest phase (BLS12-381 2^10: 109 of
//      the stitch's 130 us in k_stitch_blk, profiles/r04d_*).  Same item / slot contract as
//      k_stitch_blk with BS = 64.
#ifndef ZK_STITCH_QUAD
#define ZK_STITCH_QUAD 1
#endif
constexpr int STITCH_QBS = 64;  // items per block of k_stitch_blk_q
template <class C>
__global__ void __launch_bounds__(256) k_stitch_blk_q(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ idx,
                                                      const uint32_t *__restrict__ vals,
                                                      const uint32_t *__restrict__ count, uint32_t nb,
                                                      uint32_t *__restrict__ buckets, uint32_t *__restrict__ okeys,
                                                      uint32_t *__restrict__ ovals, uint32_t nout) {
  using F = typename C::Fp;
  constexpr int XW = xyzz_words<F>();
  constexpr uint32_t BSQ = STITCH_QBS;
  __shared__ uint4 item_lds4[BSQ * XW / 4];  // [BSQ][XW] partial sums (16 KB: several blocks per CU)
  __shared__ uint32_t skey[BSQ];
  uint32_t *lv = reinterpret_cast<uint32_t *>(item_lds4);
  uint32_t *const park = nullptr;  // doubling fallback straight from the accumulator
  const uint32_t M = *count;
  const uint32_t tq = threadIdx.x >> 2, q = threadIdx.x & 3, blk = blockIdx.x;
  const uint32_t base = blk * BSQ;
  if (base >= M) {  // no items: clear this block's output slots
    if (threadIdx.x < 2 && 2 * blk + threadIdx.x < nout) okeys[2 * blk + threadIdx.x] = nb;
    return;
  }
  const uint32_t nv = min(BSQ, M - base);  // valid quads
  const uint32_t j = base + tq;
  const bool valid = tq < nv;  // quad-uniform
  const uint32_t key = valid ? keys[j] : 0xffffffffu;
  if (q == 0) skey[tq] = key;
  Xyzz<F> acc;
  if (valid) xyzz_load(acc, vals + (size_t)idx[j] * XW);
  else xyzz_set_inf(acc);
  __syncthreads();
  for (uint32_t d = 1; d < nv; d <<= 1) {
    const bool need = valid && tq >= d && skey[tq - d] == key;
    if (!__syncthreads_or(need)) break;
    xyzz_store_quad(lv + (size_t)tq * XW, acc, (int)q);
    __syncthreads();
    if (need) {
      Xyzz<F> o;
      xyzz_load(o, lv + (size_t)(tq - d) * XW);
      xyzz_add_quad(acc, o, park);
    }
    __syncthreads();
  }
  if (!valid) return;
  const bool seg_last = tq == nv - 1 || skey[tq + 1] != key;
  if (!seg_last) return;
  const bool touches_start = skey[0] == key;
  const bool touches_end = tq == nv - 1;
  const bool cont_in = touches_start && base > 0 && keys[base - 1] == key;
  const bool cont_out = touches_end && base + nv < M && keys[base + nv] == key;
  if (!cont_in && !cont_out) {
    xyzz_store_quad(buckets + (size_t)key * XW, acc, (int)q);
  } else {
    xyzz_store_quad(ovals + (size_t)(touches_start ? 2 * blk : 2 * blk + 1) * XW, acc, (int)q);
  }
  if (q == 0) {
    const uint32_t item_key = (cont_in || cont_out) ? key : nb;
    if (touches_start) okeys[2 * blk] = item_key;
    if (touches_end) okeys[2 * blk + 1] = touches_start ? nb : item_key;
  }
}

// 5c'. block stitch level straight on the item SLOTS (no global compaction): block b takes
//      slots [b BS, (b+1) BS), packs its valid items (key < nb) into LDS in slot order
//      (wavefront ballots + a block prefix), and sums them per key by a segmented TREE
//      reduction with compacted work: at step d (1, 2, 4, ...) item t adds item t + d when
//      t's offset r inside its key segment is a multiple of 2d and t + d is still in the
//      segment, so a segment of L items costs L - 1 additions (a Hillis-Steele scan: ~L log L)
//      and ends up summed in its FIRST item; the adding items of a step are listed compactly,
//      so a step costs ceil(cnt / 64) wavefront additions (writers, r = 0 mod 2d, and the items
//      read as t + d, r = d mod 2d, never coincide, so no barrier between reads and writes).
//      A segment that touches the block's first or last item may continue in the neighbour
//      blocks: it becomes an item of the next level (slot 2b, or 2b + 1 for the last segment
//      when it is not also the first); every other segment is a whole bucket run.  The final
//      level (one block) completes everything.  Compared with compaction by a device-wide
//      scan (k_item_flags + hipCUB + k_item_index before every level), one kernel per level.
template <class C, int BS>
__global__ void __launch_bounds__(BS) k_stitch_raw(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                   uint32_t nslots, uint32_t nb, int final_level,
                                                   uint32_t *__restrict__ buckets, uint32_t *__restrict__ okeys,
                                                   uint32_t *__restrict__ ovals) {
  using F = typename C::Fp;
  constexpr int XW = xyzz_words<F>();
  constexpr int NWAVE = BS / 64;
  // [BS][XW] item sums: 64 KB for BLS12-381 G1 (BS 256), plus skey / sstart / work: ~67.6 KB of
  // static LDS -- gfx950 has 160 KB per CU (the Makefile builds for gfx950 only)
  __shared__ uint4 tree_lds4[BS * XW / 4];
  uint32_t *lv = reinterpret_cast<uint32_t *>(tree_lds4);
  __shared__ uint32_t skey[BS], sstart[BS], work[BS];
  __shared__ uint32_t wcnt[NWAVE];
  const uint32_t t = threadIdx.x, blk = blockIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t j = blk * BS + t;
  const uint32_t kin = j < nslots ? keys[j] : nb;
  const bool vin = kin < nb;
  // pack the valid items: position = valid items before this slot in the block
  uint64_t bal = __ballot(vin);
  if (lane == 0) wcnt[wave] = (uint32_t)__popcll(bal);
  __syncthreads();
  uint32_t nv = 0, off = 0;
#pragma unroll
  for (int w = 0; w < NWAVE; w++) {
    off += (uint32_t)w < wave ? wcnt[w] : 0u;
    nv += wcnt[w];
  }
  if (nv == 0) {  // no items: this block's output slots stay empty
    if (!final_level && t < 2) okeys[2 * blk + t] = nb;
    return;
  }
  if (vin) {
    const uint32_t q = off + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
    skey[q] = kin;
    const uint4 *src = reinterpret_cast<const uint4 *>(vals + (size_t)j * XW);
    uint4 *dst = reinterpret_cast<uint4 *>(lv + (size_t)q * XW);
#pragma unroll
    for (int i = 0; i < XW / 4; i++) dst[i] = src[i];
  }
  __syncthreads();
  const bool valid = t < nv;
  const uint32_t key = valid ? skey[t] : 0xffffffffu - t;  // past nv: singleton segments
  // segment start of every item: a max-scan of the start positions
  uint32_t st = (t == 0 || (valid && skey[t - 1] != key) || !valid) ? t : 0u;
  sstart[t] = st;
  __syncthreads();
  for (uint32_t o = 1; o < (uint32_t)BS; o <<= 1) {
    const uint32_t v = t >= o ? sstart[t - o] : 0u;
    __syncthreads();
    st = max(st, v);
    sstart[t] = st;
    __syncthreads();
  }
  const uint32_t r = t - st;  // offset inside the segment
  for (uint32_t d = 1; d < nv; d <<= 1) {
    const bool need = valid && (r & (2 * d - 1)) == 0 && t + d < nv && skey[t + d] == key;
    bal = __ballot(need);
    if (lane == 0) wcnt[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t woff = 0, cnt = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; w++) {
      woff += (uint32_t)w < wave ? wcnt[w] : 0u;
      cnt += wcnt[w];
    }
    if (need) work[woff + (uint32_t)__popcll(bal & ((1ull << lane) - 1))] = t;
    __syncthreads();
    if (cnt == 0) break;  // every segment is summed (block-uniform)
    if (t < cnt) {        // compacted: wavefronts past cnt skip the addition
      const uint32_t a = work[t];
      Xyzz<F> acc, o;
      xyzz_load(acc, lv + (size_t)a * XW);
      xyzz_load(o, lv + (size_t)(a + d) * XW);
      xyzz_add_red(acc, o);
      xyzz_store(lv + (size_t)a * XW, acc);
    }
    __syncthreads();
  }
  if (!valid || r != 0) return;  // the segment's first item owns its sum
  const bool touches_start = t == 0;
  const bool touches_end = skey[nv - 1] == key;
  Xyzz<F> acc;
  xyzz_load(acc, lv + (size_t)t * XW);
  if (final_level || (!touches_start && !touches_end)) {
    xyzz_store(buckets + (size_t)key * XW, acc);
    return;
  }
  xyzz_store(ovals + (size_t)(touches_start ? 2 * blk : 2 * blk + 1) * XW, acc);
  if (touches_start) okeys[2 * blk] = key;
  if (touches_end) {
    if (touches_start) okeys[2 * blk + 1] = nb;
    else okeys[2 * blk + 1] = key;
  }
}

// 5a'. index compaction: the valid item slots as (key, slot index) pairs -- the XYZZ
//      payloads stay where they are and the stitch reads them through the index
static __global__ void __launch_bounds__(256) k_item_index(const uint32_t *__restrict__ ikeys,
                                                           const uint32_t *__restrict__ flags,
                                                           const uint32_t *__restrict__ pos, uint32_t nslots,
                                                           uint32_t *__restrict__ okeys, uint32_t *__restrict__ oidx,
                                                           uint32_t *__restrict__ ocount) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots) return;
  if (i == nslots - 1) *ocount = pos[i] + flags[i];
  if (!flags[i]) return;
  const uint32_t o = pos[i];
  okeys[o] = ikeys[i];
  oidx[o] = i;
}

// In-wavefront segmented point sum: the G lanes of an aligned segment (G a power of two
// <= 64) fold their accumulators with log2(G) cross-lane steps; lane 0 of the segment
// ends up with the segment's sum.  (Every lane executes every step, so the cost is
// log2(G) point adds of latency whatever the segment size.)
template <class F>
__device__ __forceinline__ Xyzz<F> xyzz_shfl_down(const Xyzz<F> &a, int off, int width) {
  Xyzz<F> r;
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    r.X.v[i] = (uint32_t)__shfl_down((int)a.X.v[i], off, width);
    r.Y.v[i] = (uint32_t)__shfl_down((int)a.Y.v[i], off, width);
    r.ZZ.v[i] = (uint32_t)__shfl_down((int)a.ZZ.v[i], off, width);
    r.ZZZ.v[i] = (uint32_t)__shfl_down((int)a.ZZZ.v[i], off, width);
  }
  return r;
}
template <class F>
__device__ __forceinline__ void seg_fold(Xyzz<F> &acc, int G) {
  for (int off = G >> 1; off >= 1; off >>= 1) {
    Xyzz<F> o = xyzz_shfl_down(acc, off, G);
    xyzz_add(acc, o);
  }
}

// Segment layout shared by the two reduction kernels: per window, segments of
// decreasing size G (aligned by construction), the window's lane block padded to a
// multiple of 64 so no wavefront spans two windows.
struct SegRegion {
  int count;  // segments in this region
  int G;      // lanes per segment
  int len;    // items per segment
};

// 6. digit split of the bucket weights.  Bucket m of a window (digit m + 1) has
//    m = m1 * 2^l0 + m0 (l0 + l1 = c - 1), so
//       sum_m (m+1) B_m = sum_v v Y0_v + 2^l0 sum_v v Y1_v + sum_v Y0_v,
//       Y0_v = sum_{m0 = v} B_m (2^l1 buckets),  Y1_v = sum_{m1 = v} B_m (2^l0 buckets).
//    Every Y is a PLAIN sum (no weights, no running-sum chain): G lanes per Y, each adds
//    len/G buckets, then an in-wavefront fold.  Region 0: the 2^l1 sums Y1 (longer
//    segments first), region 1: the 2^l0 sums Y0.  Output Y[w][y]: y < 2^l0 -> Y0_y,
//    else Y1_(y - 2^l0).
template <class C>
__global__ void __launch_bounds__(256) k_ysum(const uint32_t *__restrict__ buckets,
                                              const uint32_t *__restrict__ offsets,
                                              const uint8_t *__restrict__ filled, int W, int c, int l0,
                                              SegRegion r0, SegRegion r1, int wlanes,
                                              uint32_t *__restrict__ Y) {
  using F = typename C::Fp;
  const int l1 = c - 1 - l0;
  const int NY = (1 << l0) + (1 << l1);
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int w = g / wlanes, t = g % wlanes;  // W * wlanes is a multiple of 256 by launch
  const bool active = w < W;
  const int n0 = r0.count * r0.G;
  int G, len, seg, lane;
  bool hiY;  // Y1 (region 0) or Y0 (region 1)
  if (t < n0) { G = r0.G; len = r0.len; seg = t / G; lane = t % G; hiY = true; }
  else if (t < n0 + r1.count * r1.G) { G = r1.G; len = r1.len; seg = (t - n0) / G; lane = (t - n0) % G; hiY = false; }
  else { G = 1; len = 0; seg = 0; lane = 0; hiY = false; }  // padding lanes: no fold
  const uint32_t B = 1u << (c - 1);
  const int per = len / G;
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  if (active) {
    for (int k = 0; k < per; k++) {
      const int s = lane * per + k;
      const uint32_t m = hiY ? ((uint32_t)seg << l0) + s : ((uint32_t)s << l0) + seg;
      const uint32_t rank = (uint32_t)w * B + m;
      if (filled ? filled[rank] != 0 : offsets[rank + 1] > offsets[rank]) {  // empty buckets hold garbage
        Xyzz<F> bm;
        xyzz_load(bm, buckets + ((size_t)w * B + m) * xyzz_words<F>());
        xyzz_add(acc, bm);
      }
    }
  }
  seg_fold(acc, G);
  if (active && lane == 0 && len > 0) {
    const int y = hiY ? (1 << l0) + seg : seg;
    xyzz_store(Y + ((size_t)w * NY + y) * xyzz_words<F>(), acc);
  }
}

#ifndef ZK_YSUM_QUAD_FOLD
#define ZK_YSUM_QUAD_FOLD 1  // k_ysum2's block fold with quad-cooperative additions (G1)
#endif
// 6'. k_ysum2: block-level form of k_ysum, used when each region fills whole 256-lane
//     blocks (every shape from c = 12 up at the default QY).  Segment s of a block owns the
//     STRIDED lanes {s, s + S, s + 2S, ...} (S = 256 / G segments per block), so the fold
//     pairs lane t with lane t + h (h = 128 ... S): the upper half parks its partial in LDS
//     and drops out, the lower half adds it -- whole wavefronts leave the fold as h
//     shrinks, where k_ysum's in-wavefront fold keeps every lane adding at every step.
//     For G1 the fold's additions are quad-cooperative (xyzz_add_quad, 64 per round).
//     The next bucket's emptiness test (and, with PF, its data) is loaded one iteration
//     ahead: at one or two waves per SIMD nothing else hides those latencies.
#ifndef ZK_YSUM_WAVES
#define ZK_YSUM_WAVES 1  // waves per SIMD k_ysum2 is compiled for (A/B hook)
#endif
template <class C, bool PF>
__global__ void __launch_bounds__(256, ZK_YSUM_WAVES) k_ysum2(const uint32_t *__restrict__ buckets,
                                               const uint32_t *__restrict__ offsets,
                                               const uint8_t *__restrict__ filled, int W, int c, int l0,
                                               SegRegion r0, SegRegion r1, uint32_t *__restrict__ Y) {
  using F = typename C::Fp;
  constexpr int XW = xyzz_words<F>();
  // G1: the fold runs quad-cooperatively (2 x 64 KB of LDS for BLS12-381: the parked sums and
  // xyzz_add_quad's per-lane doubling fallback); Fp2 points keep the one-lane fold (LDS)
  constexpr bool QUAD_FOLD = ZK_YSUM_QUAD_FOLD && is_base_field<F>();
  __shared__ uint4 park4[(QUAD_FOLD ? 256 : 128) * XW / 4];
  __shared__ uint4 fold4[QUAD_FOLD ? 256 * XW / 4 : 1];
  uint32_t *park = reinterpret_cast<uint32_t *>(park4);
  uint32_t *fold = reinterpret_cast<uint32_t *>(fold4);
  const int l1 = c - 1 - l0;
  const int NY = (1 << l0) + (1 << l1);
  const int nb0 = r0.count * r0.G / 256, nb1 = r1.count * r1.G / 256;  // blocks per window and region
  const int w = blockIdx.x / (nb0 + nb1);
  int rb = blockIdx.x % (nb0 + nb1);
  const bool hiY = rb < nb0;  // Y1 (region 0) or Y0 (region 1)
  const SegRegion r = hiY ? r0 : r1;
  if (!hiY) rb -= nb0;
  const int G = r.G, S = 256 / G;
  const int t = threadIdx.x;
  const int seg = rb * S + t % S, part = t / S;
  const int per = r.len / G;
  const uint32_t B = 1u << (c - 1);
  const uint32_t *wb = buckets + (size_t)w * B * XW;
  auto bucket_m = [&](int s) -> uint32_t {
    return hiY ? ((uint32_t)seg << l0) + (uint32_t)s : ((uint32_t)s << l0) + (uint32_t)seg;
  };
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  auto nonempty = [&](uint32_t rank) -> bool {  // empty buckets hold garbage (never written)
    return filled ? filled[rank] != 0 : offsets[rank + 1] > offsets[rank];
  };
  uint32_t m = bucket_m(part * per);
  bool nfull = nonempty((uint32_t)w * B + m);
  Xyzz<F> nxt;
  if (PF) xyzz_load(nxt, wb + (size_t)m * XW);
  for (int k = 0; k < per; k++) {
    const bool full = nfull;
    const uint32_t mc = m;
    Xyzz<F> cur;
    if (PF) cur = nxt;
    if (k + 1 < per) {
      m = bucket_m(part * per + k + 1);
      nfull = nonempty((uint32_t)w * B + m);
      if (PF) xyzz_load(nxt, wb + (size_t)m * XW);
    }
    if (full) {
      if (!PF) xyzz_load(cur, wb + (size_t)mc * XW);
      xyzz_add_red(acc, cur);
    }
  }
  if constexpr (QUAD_FOLD) {
    // quad-cooperative fold: every lane parks its sum; level h adds slot a + h into slot a (a < h)
    // with 4 lanes per addition (xyzz_add_quad: 5 product latencies instead of 14), 64 additions
    // per round.  Slots read in a round (a, a + h) are never written in it (writes go to a < h).
    xyzz_store(fold + (size_t)t * XW, acc);
    __syncthreads();
    const int q = t >> 2;
    for (int h = 128; h >= S; h >>= 1) {
      for (int base = 0; base < h; base += 64) {
        const int a = base + q;
        Xyzz<F> x;
        if (a < h) {  // quad-uniform
          Xyzz<F> o;
          xyzz_load(x, fold + (size_t)a * XW);
          xyzz_load(o, fold + (size_t)(a + h) * XW);
          xyzz_add_quad(x, o, park + (size_t)t * XW);
        }
        __syncthreads();
        if (a < h && (t & 3) == 0) xyzz_store(fold + (size_t)a * XW, x);
      }
      __syncthreads();
    }
    if (t < S) {
      xyzz_load(acc, fold + (size_t)t * XW);
      const int y = hiY ? (1 << l0) + seg : seg;
      xyzz_store(Y + ((size_t)w * NY + y) * XW, acc);
    }
  } else {
    for (int h = 128; h >= S; h >>= 1) {
      if (t >= h && t < 2 * h) xyzz_store(park + (size_t)(t - h) * XW, acc);
      __syncthreads();
      if (t < h) {
        Xyzz<F> o;
        xyzz_load(o, park + (size_t)t * XW);
        xyzz_add_red(acc, o);
      }
      __syncthreads();
    }
    if (t < S) {
      const int y = hiY ? (1 << l0) + seg : seg;
      xyzz_store(Y + ((size_t)w * NY + y) * XW, acc);
    }
  }
}

// 6''. k_ysum3: k_ysum2 at TWO waves per SIMD, for the large windows (c = 20 at 2^23-2^26:
//      W * 2^c = 13.6M bucket additions, ~13 block rounds of k_ysum2 at one wave per SIMD, where
//      that kernel issues only ~0.6 of the VALU slots: nothing hides a lone wave's product and
//      load latencies).  The next bucket is gathered straight into LDS by global_load_lds while
//      the current addition runs (as in k_accum), so the prefetch costs no VGPRs (k_ysum2's
//      register prefetch holds 288); the block fold reuses the same LDS image after the loop
//      (one-lane additions: the fold is ~6 % of the additions at 16 buckets per lane).  64 KB of
//      LDS per block at BLS12-381: two blocks per CU.  G1 only.  (At BLS12-381 2^20 there are
//      65536 Y-sum lanes, one wave per SIMD in total, so this shape would only halve the lanes'
//      work and add fold levels: measured 0.36-0.39 vs 0.32 ms there, profiles/r03i_*.)
template <class C, int WAVES = 2>
__global__ void __launch_bounds__(256, WAVES) k_ysum3(const uint32_t *__restrict__ buckets,
                                                  const uint32_t *__restrict__ offsets,
                                                  const uint8_t *__restrict__ filled, int W, int c, int l0,
                                                  SegRegion r0, SegRegion r1, uint32_t *__restrict__ Y) {
  using F = typename C::Fp;
  constexpr int XW = xyzz_words<F>();
  constexpr int NCH = XW / 4;  // 16-B chunks per bucket
  __shared__ uint4 stage[4][NCH][64];
  static_assert(4 * NCH * 64 * 16 >= 128 * XW * 4, "the fold's park area fits the prefetch image");
  uint32_t *park = reinterpret_cast<uint32_t *>(&stage[0][0][0]);
  const int l1 = c - 1 - l0;
  const int NY = (1 << l0) + (1 << l1);
  const int nb0 = r0.count * r0.G / 256, nb1 = r1.count * r1.G / 256;  // blocks per window and region
  const int w = blockIdx.x / (nb0 + nb1);
  int rb = blockIdx.x % (nb0 + nb1);
  const bool hiY = rb < nb0;  // Y1 (region 0) or Y0 (region 1)
  const SegRegion r = hiY ? r0 : r1;
  if (!hiY) rb -= nb0;
  const int G = r.G, S = 256 / G;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int seg = rb * S + t % S, part = t / S;
  const int per = r.len / G;
  const uint32_t B = 1u << (c - 1);
  const uint32_t *wb = buckets + (size_t)w * B * XW;
  auto bucket_m = [&](int s) -> uint32_t {
    return hiY ? ((uint32_t)seg << l0) + (uint32_t)s : ((uint32_t)s << l0) + (uint32_t)seg;
  };
  auto nonempty = [&](uint32_t rank) -> bool {  // empty buckets hold garbage (never written)
    return filled ? filled[rank] != 0 : offsets[rank + 1] > offsets[rank];
  };
  auto prefetch = [&](uint32_t m) {
    const uint32_t *src = wb + (size_t)m * XW;
#pragma unroll
    for (int j = 0; j < NCH; j++)
      __builtin_amdgcn_global_load_lds((glb_void_t *)(src + 4 * j), (lds_void_t *)&stage[wave][j][0], 16, 0, 0);
  };
  auto read_bucket = [&](Xyzz<F> &P) {
    uint32_t wd[XW];
#pragma unroll
    for (int j = 0; j < NCH; j++) {
      const uint4 v = stage[wave][j][lane];
      wd[4 * j] = v.x;
      wd[4 * j + 1] = v.y;
      wd[4 * j + 2] = v.z;
      wd[4 * j + 3] = v.w;
    }
    xyzz_load(P, wd);
  };
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  uint32_t m = bucket_m(part * per);
  bool nfull = nonempty((uint32_t)w * B + m);
  prefetch(m);
  for (int k = 0; k < per; k++) {
    const bool full = nfull;
    Xyzz<F> cur;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the gather of bucket k has landed in LDS
    read_bucket(cur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS image read out before it is refilled
    if (k + 1 < per) {
      m = bucket_m(part * per + k + 1);
      nfull = nonempty((uint32_t)w * B + m);
      prefetch(m);
    }
    if (full) xyzz_add_red(acc, cur);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wavefront is done with its image: the fold reuses the LDS
  for (int h = 128; h >= S; h >>= 1) {
    if (t >= h && t < 2 * h) xyzz_store(park + (size_t)(t - h) * XW, acc);
    __syncthreads();
    if (t < h) {
      Xyzz<F> o;
      xyzz_load(o, park + (size_t)t * XW);
      xyzz_add_red(acc, o);
    }
    __syncthreads();
  }
  if (t < S) {
    const int y = hiY ? (1 << l0) + seg : seg;
    xyzz_store(Y + ((size_t)w * NY + y) * XW, acc);
  }
}

// 7. weighted Y sums by bit jobs: one 256-thread block per (window, job) = 64 quad lanes
//    (xyzz_add_quad: 4 physical lanes per addition).  Job 0 is the total sum_m B_m, taken
//    over the 2^l1 sums Y1 (the smaller set); job j in 1..l0 sums the Y0_v with bit j-1 of v
//    set, job j > l0 the Y1_v with bit j-1-l0 set (exponent j-1 either way).  Each quad adds
//    n/64 <= 2 items, then a block fold through LDS: depth log2(n) quad additions, where a
//    fold inside one wavefront (16 quads) would leave 8-16 items serial per quad.
template <class C>
__global__ void __launch_bounds__(256) k_jobsum_blk(const uint32_t *__restrict__ Y, int c, int l0,
                                                    uint64_t *__restrict__ out) {
  using F = typename C::Fp;
  constexpr int XW = xyzz_words<F>();
  __shared__ uint32_t park_lds[256 * XW];  // xyzz_add_quad's doubling fallback, per lane
  __shared__ uint4 fold4[32 * XW / 4];     // fold exchange, one slot per upper-half quad
  uint32_t *fold = reinterpret_cast<uint32_t *>(fold4);
  uint32_t *park = park_lds + threadIdx.x * XW;
  const int l1 = c - 1 - l0;
  const int NY = (1 << l0) + (1 << l1);
  const int w = blockIdx.x / c, j = blockIdx.x % c;
  const int t = threadIdx.x >> 2;  // quad (logical lane) 0..63
  const int d = (j == 0 || j > l0) ? 1 : 0;  // Y1 or Y0
  const int b = j == 0 ? -1 : (d ? j - 1 - l0 : j - 1);
  const int ld = d ? l1 : l0;
  const int n = b < 0 ? (1 << ld) : (1 << (ld - 1));
  const uint32_t *Yd = Y + ((size_t)w * NY + (d ? (1 << l0) : 0)) * XW;
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  for (int e = t; e < n; e += 64) {
    int v = e;
    if (b >= 0) {  // e-th index with bit b set
      const int lowmask = (1 << b) - 1;
      v = ((e & ~lowmask) << 1) | (1 << b) | (e & lowmask);
    }
    Xyzz<F> p;
    xyzz_load(p, Yd + (size_t)v * XW);
    xyzz_add_quad(acc, p, park);
  }
  // fold only over the quads that hold items (min(n, 64)): small windows have 8-32 items per job
  const int act = n < 64 ? n : 64;
  int h0 = 1;
  while (2 * h0 < act) h0 <<= 1;
  for (int h = act > 1 ? h0 : 0; h >= 1; h >>= 1) {
    if (t >= h && t < 2 * h && (threadIdx.x & 3) == 0) xyzz_store(fold + (size_t)(t - h) * XW, acc);
    __syncthreads();
    if (t < h) {
      Xyzz<F> o;
      xyzz_load(o, fold + (size_t)t * XW);
      xyzz_add_quad(acc, o, park);
    }
    __syncthreads();
  }
  // export: the 4 lanes of quad 0 hold the sum replicated; lane q writes coordinate q in the
  // canonical reference form (X, Y, ZZ, ZZZ of NP64 u64 each) for the host
  if (threadIdx.x < 4) {
    const int q = (int)threadIdx.x;
    Fe<F> v, r;
    fe_sel4(v, acc.X, acc.Y, acc.ZZ, acc.ZZZ, q);
    fe_to_ref(r, v);
    fe_store_ref(out + (((size_t)w * c + j) * 4 + q) * C::NP64, r);
  }
}

// ---------------------------------------------------------------------------
// Small inputs: bit jobs straight on the pairs, no buckets.
//   sum_i k_i P_i = sum_t 2^t Q_t,   Q_t = sum of the P_i whose scalar has bit t set
// Every step of the bucket pipeline is latency-bound at a few thousand pairs (a lone lane's
// point operation ~8 us, ~25 of them in a row through sort, accumulation, stitch, Y sums and
// job sums: BLS12-381 2^10 spent 0.38 ms on the device, profiles/r04l_*).  Here the chain is
// K = n / G mixed additions per lane plus a log-depth quad fold, and the host runs the usual
// Horner over the bits (its chain of ~255 doublings is the same as after the bucket pipeline).
// The work is nbits n predicated mixed additions -- 8-9x the bucket method's W n -- so the
// path only pays below a few thousand pairs (msm_bits_max).
//
constexpr int BITACC_MAX_K = 256;  // pairs per k_bitacc block (its LDS scalar staging)
// k_bitacc: block g = pairs [g K, g K + K), thread t = bit t (a wavefront covers 64 bits, so the
// point of step e is one uniform load for the whole block).  The K scalars are converted to
// integers (REDC when Montgomery) into LDS first; lane t adds P_e when bit t of k_e is set.
// Output: partial sum of bit t over the chunk at part[t G + g] (lazy XYZZ, like k_accum's flushes).
template <class C>
__global__ void __launch_bounds__(256, AccumOcc<typename C::Fp>::waves)
    k_bitacc(const uint64_t *__restrict__ scalars, int n, int stride, int loff, int nread, int mont, int nbits, int K,
             const uint32_t *__restrict__ points, uint32_t *__restrict__ part) {
  using F = typename C::Fp;
  constexpr int AW = aff_words<F>();
  __shared__ uint32_t sk[BITACC_MAX_K][9];  // integer scalars of the chunk (8 words, padded)
  const int t = threadIdx.x, g = blockIdx.x, G = gridDim.x;
  const int p0 = g * K, np = min(K, n - p0);
  for (int e = t; e < np; e += 256) {
    DigitStream<C> ds;
    ds.load(scalars, p0 + e, stride, loff, nread, mont);
#pragma unroll
    for (int j = 0; j < 8; j++) sk[e][j] = ds.k[j];
  }
  __syncthreads();
  if (t >= nbits) return;
  const int word = t >> 5;
  const uint32_t bit = (uint32_t)t & 31u;
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  for (int e = 0; e < np; e++) {
    if ((sk[e][word] >> bit) & 1u) {
      Aff<F> P;
      if (aff_load(P, points + (size_t)(p0 + e) * AW)) xyzz_acc_aff(acc, P);
    }
  }
  xyzz_store(part + ((size_t)t * G + g) * xyzz_words<F>(), acc);
}

// k_bitsum: one 256-thread block per bit t = 64 quad lanes (xyzz_add_quad): quad q adds the
// partials q, q + 64, ... of row t, then the block folds the active quads through LDS (depth
// log2 min(G, 64)); exports Q_t in the canonical reference form (X, Y, ZZ, ZZZ) for the host.
template <class C>
__global__ void __launch_bounds__(256) k_bitsum(const uint32_t *__restrict__ part, int G, uint64_t *__restrict__ out) {
  using F = typename C::Fp;
  constexpr int XW = xyzz_words<F>();
  __shared__ uint32_t park_lds[256 * XW];  // xyzz_add_quad's doubling fallback, per lane
  __shared__ uint4 fold4[32 * XW / 4];     // fold exchange, one slot per upper-half quad
  uint32_t *fold = reinterpret_cast<uint32_t *>(fold4);
  uint32_t *park = park_lds + threadIdx.x * XW;
  const int tb = blockIdx.x;
  const int q = threadIdx.x >> 2;  // quad (logical lane) 0..63
  const uint32_t *row = part + (size_t)tb * G * XW;
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  for (int e = q; e < G; e += 64) {
    Xyzz<F> p;
    xyzz_load(p, row + (size_t)e * XW);
    xyzz_add_quad(acc, p, park);
  }
  const int act = G < 64 ? G : 64;
  int h0 = 1;
  while (2 * h0 < act) h0 <<= 1;
  for (int h = act > 1 ? h0 : 0; h >= 1; h >>= 1) {
    if (q >= h && q < 2 * h && (threadIdx.x & 3) == 0) xyzz_store(fold + (size_t)(q - h) * XW, acc);
    __syncthreads();
    if (q < h) {
      Xyzz<F> o;
      xyzz_load(o, fold + (size_t)q * XW);
      xyzz_add_quad(acc, o, park);
    }
    __syncthreads();
  }
  if (threadIdx.x < 4) {
    const int l = (int)threadIdx.x;
    Fe<F> v, r;
    fe_sel4(v, acc.X, acc.Y, acc.ZZ, acc.ZZZ, l);
    fe_to_ref(r, v);
    fe_store_ref(out + ((size_t)tb * 4 + l) * C::NP64, r);
  }
}

// ---------------------------------------------------------------------------
// host orchestration

struct MsmShape {
  int n, c, W, B, l0, l1, NY, QY, J, CH;  // W: windows handled by one pass of the pipeline
  SegRegion r0, r1;
  int ylanes;  // lanes per window of k_ysum (multiple of 64)
  // two-level bucket sort: 2^fs fine buckets per coarse bin, nbins coarse bins per window,
  // level-1 workgroups of M entries (nwg per window)
  int fs, nbins, M, nwg;
  // level 1.5 (k_split): 2^s2 sub-bins per coarse bin (0: none), nwg2 workgroups per bin
  int s2 = 0, nwg2 = 1;
  size_t nmat2() const { return (size_t)W * nbins * ((size_t)1 << s2) * nwg2; }
  // point splits: the entries are sorted by (split, window, bucket), split h holding the pairs
  // [split_lo(h), split_lo(h + 1)); each split is accumulated by its own launch (host-input calls
  // start on the first split while the later splits' points still cross PCIe)
  int NS;
  size_t nmat() const { return (size_t)W * nbins * nwg; }  // level-1 count matrix of one split
  int split_lo(int h) const;
  int split_ch(int h) const;  // accumulation chunk length of split h
  int nsplit_max() const {  // points of the largest split
    int m = 0;
    for (int h = 0; h < NS; h++) m = std::max(m, split_lo(h + 1) - split_lo(h));
    return m;
  }
};

// Split weights of a host-input MSM (sixteenths): the first split is small so the device starts
// after 1/8 of the copies, the last one is small so little accumulation is left after the last
// copy lands, the middle ones are large so few splits pay the per-split sort / stitch.
// ZK_MSM_SPLIT_W="w0,w1,..." (experiment hook, read once): other weights / split counts (<= 8).
struct SplitCfg {
  int ns;
  int w[8];
};
static const SplitCfg &split_cfg() {
  static const SplitCfg cfg = [] {
    SplitCfg c{5, {2, 3, 4, 4, 3}};
    if (const char *e = getenv("ZK_MSM_SPLIT_W")) {
      SplitCfg d{0, {0}};
      for (const char *p = e; *p && d.ns < 8;) {
        char *end = nullptr;
        const long v = strtol(p, &end, 10);
        if (end == p || v <= 0) break;
        d.w[d.ns++] = (int)v;
        p = *end == ',' ? end + 1 : end;
      }
      if (d.ns >= 1) c = d;
    }
    return c;
  }();
  return cfg;
}
static const int *split_weights(int NS) {
  return NS == split_cfg().ns ? split_cfg().w : nullptr;  // nullptr: equal splits
}
inline int MsmShape::split_lo(int h) const {
  const int *w = split_weights(NS);
  if (!w) return (int)((int64_t)n * h / NS);
  int acc = 0, tot = 0;
  for (int k = 0; k < NS; k++) {
    tot += w[k];
    if (k < h) acc += w[k];
  }
  return (int)((int64_t)n * acc / tot);
}

static int ilog2(unsigned x) { int r = 0; while ((1u << (r + 1)) <= x) r++; return r; }

// Shape of one pipeline pass over W windows of n scalars.  The constants were swept on
// MI355X (profiles/r01_*, profiles/r02h_qy_qa_sweep.txt): Y sums take 16 buckets per lane at
// scale (8: ysum 0.37 -> 0.48 ms, 4: 0.66 ms at BLS12-381 2^20), the accumulation 64 sorted entries per lane (128 from 2^25
// entries on, profiles/r01_v7_ch_sweep.txt).
#define ZK_MSM_SPLITS_MAX 8  // most splits of a host-input MSM pipeline (copy / sort / accumulation overlap)
// Splits of a host-input MSM whose windows fit one pipeline pass: 5 weighted splits (2, 3, 4, 4, 3
// sixteenths, split_weights) from 2^19 pairs, 2 from 2^17, else 1 (BLS12-381 2^20 through the
// reference symbol: 6.3-6.4 ms unsplit, 5.4-5.5 ms in two splits, 4.8-4.9 ms in four equal ones,
// profiles/r03e_split_e2e.txt; the round-4 copy / sort / conversion streams: profiles/r04*_e2e*)
static int msm_splits(int n, bool host_inputs, bool one_pass) {
  if (!host_inputs || !one_pass) return 1;
  if (n >= (1 << 19)) return split_cfg().ns;
  if (n >= (1 << 17)) return split_cfg().ns < 2 ? split_cfg().ns : 2;
  return 1;
}
#ifndef ZK_YSUM_LANES
#define ZK_YSUM_LANES 65536  // Y-sum lanes at most (one wave per SIMD of 256 CUs)
#endif
#ifndef ZK_YSUM_PF
#define ZK_YSUM_PF 1  // k_ysum2 loads the next bucket one iteration ahead
#endif
#ifndef ZK_YSUM_PF_G2
#define ZK_YSUM_PF_G2 1  // the same for Fp2 points (A/B hook)
#endif
// Y sums by k_ysum3 (two waves per SIMD, LDS prefetch) when the lanes fill several rounds of one
// wave per SIMD (ZK_YSUM3_LANES, default 4 x 65536: c = 20 from 2^23 pairs).  Mode -1: that rule,
// 0 / 1: always k_ysum2 / k_ysum3 (block-level shapes); set by the environment ZK_YSUM3 (A/B hook)
// or zkg_msm_set_ysum_mode (test hook)
inline std::atomic<int> &ysum_mode() {
  static std::atomic<int> v{[] {
    const char *e = getenv("ZK_YSUM3");
    return e ? (atoi(e) != 0 ? 1 : 0) : -1;
  }()};
  return v;
}
// G2 Y sums through k_ysum3<C, 1> (LDS prefetch) instead of k_ysum2 (register prefetch): default on
// for BLS12-381 G2 only (its k_ysum2 spills 247 VGPRs; 1.211 -> 1.126 ms at 2^20, MSM 12.06 -> 11.99
// ms; BN254 G2 0.498 -> 0.512 ms, off; profiles/r06f_g2lds*).  ZK_YSUM_G2_LDS=1 / 0 forces either
// (A/B hook, read once).
template <class F>
inline bool ysum_g2_lds() {
  static const int env = [] {
    const char *e = getenv("ZK_YSUM_G2_LDS");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  return env >= 0 ? env == 1 : F::N >= 28;
}
inline bool ysum3_on(size_t lanes) {
  static const size_t min_lanes = [] {
    const char *e = getenv("ZK_YSUM3_LANES");
    return e ? (size_t)atoll(e) : (size_t)4 * 65536;
  }();
  const int mode = ysum_mode().load();
  return mode >= 0 ? mode != 0 : lanes >= min_lanes;
}
// buckets per Y-sum lane at scale (a power of two; ZK_YSUM_QY overrides it, A/B hook, read once)
inline int ysum_qy_max() {
  static const int v = [] {
    const char *e = getenv("ZK_YSUM_QY");
    const int q = e ? atoi(e) : 16;
    return (q >= 1 && q <= 256 && (q & (q - 1)) == 0) ? q : 16;
  }();
  return v;
}
static MsmShape make_shape(int n, int c, int W, int NS = 1) {
  MsmShape s;
  s.n = n;
  s.c = c;
  s.W = W;
  s.NS = NS;
  s.B = 1 << (c - 1);
  s.l0 = c / 2;  // l0 + l1 = c - 1, l0 >= l1
  s.l1 = c - 1 - s.l0;
  s.NY = (1 << s.l0) + (1 << s.l1);
  auto pow2 = [](int v) { int r = 1; while (2 * r <= v) r *= 2; return r; };  // segments need powers of 2
  // buckets per lane in the Y sums: 16 at scale, fewer when there are few buckets, so the
  // sums keep at most ~64K lanes (2 W B bucket adds): one wave per SIMD, each issuing its
  // own chain (more lanes share the SIMDs and only lengthen every fold step; BLS12-381
  // 2^16: ysum 0.21 -> ~0.15 ms with QY 2 -> 4, profiles/r02y_msm_small_ab.txt)
  {
    const size_t adds = 2 * (size_t)s.W * (size_t)s.B;
    int q = (int)((adds + ZK_YSUM_LANES - 1) / ZK_YSUM_LANES);  // rounded up: at most ZK_YSUM_LANES lanes
    q = q < 1 ? 1 : (q > ysum_qy_max() ? ysum_qy_max() : q);
    s.QY = pow2(q) < q ? 2 * pow2(q) : pow2(q);  }
  auto clampG = [](int g) { return g < 1 ? 1 : (g > 64 ? 64 : g); };
  s.r0 = SegRegion{1 << s.l1, clampG((1 << s.l0) / s.QY), 1 << s.l0};  // Y1 sums
  s.r1 = SegRegion{1 << s.l0, clampG((1 << s.l1) / s.QY), 1 << s.l1};  // Y0 sums
  s.ylanes = (s.r0.count * s.r0.G + s.r1.count * s.r1.G + 63) & ~63;
  s.J = c;
  {
    const int lb = c - 1;  // log2 B
    s.fs = lb > 8 ? lb - 8 : 0;
    s.nbins = 1 << (lb - s.fs);
    // ~2048 level-1 workgroups over the pass, at least 2048 entries each
    size_t M = ((size_t)W * n + 2047) / 2048;
    M = (M + 255) & ~(size_t)255;
    s.M = (int)(M < 2048 ? 2048 : M);
    s.nwg = (int)(((size_t)s.nsplit_max() + s.M - 1) / s.M);
    // sub-bins when an average coarse bin exceeds half of level 2's LDS staging AND has >= 1024
    // fine buckets to scatter to (c >= 19: 2^25-2^26 at the default window; BLS12-381 2^26 sort
    // 31.6 -> 15.6 ms).  With c = 16's 128 fine buckets per bin the direct scatter stays cheaper
    // than the extra pass (2^21-2^24: +0.2 to +1.4 ms, profiles/r04x_*).  ZK_SORT_SPLIT=0 turns
    // level 1.5 off (A/B hook, read once)
    static const bool split_on = [] {
      const char *e = getenv("ZK_SORT_SPLIT");
      return !(e && e[0] == '0');
    }();
    const size_t per_bin = (size_t)s.nsplit_max() / s.nbins;
    const size_t half_cap = (size_t)fine_stage_cap(s.fs) / 2;
    while (split_on && s.fs >= 10 && s.s2 < s.fs && s.s2 < 8 && (per_bin >> s.s2) > half_cap) s.s2++;
    if (s.s2) {
      const size_t w2 = per_bin / 16384;  // ~16K entries per level-1.5 workgroup
      s.nwg2 = (int)(w2 < 1 ? 1 : (w2 > 64 ? 64 : w2));
    }
  }
  // entries per thread in the level-0 accumulation: 64 at scale (~2^17+ lanes), fewer for
  // small inputs so the serial chain per lane stays short (a lone lane's madd ~12 us), and at
  // least 8 above 2^12 points (window x chunk sweep, profiles/r03l_small_window_chunk_sweep.txt;
  // a floor at the average bucket run, n / B, measured worse: profiles/r03k_chunk_rule_sweep.txt)
  s.CH = s.split_ch(0);
  return s;
}

// The chunk rule is applied to every split's own entry count (each launch keeps ~2^17 lanes = 2
// waves per SIMD, or 2^18 at CH 64), so a small split does not run its accumulation at one wave per
// SIMD (round 3 sized every split's chunks from the largest split).
inline int MsmShape::split_ch(int h) const {
  const size_t ent = (size_t)W * (size_t)(split_lo(h + 1) - split_lo(h));  // entries of this launch
  const size_t ch = ent >> 17, lo = n > 4096 ? 8 : 4;
  int r = ch >= 64 ? 64 : (ch <= lo ? (int)lo : (int)ch);
  if (ent >= ((size_t)1 << 25)) r = 128;
  if (const char *e = getenv("ZK_MSM_CH")) {  // experiment / test hook: fixed chunk length
    const int v = atoi(e);
    if (v > 0) r = v;
  }
  return r;
}

// items per workgroup of the block stitch: 128 for the wide G2 points, so the LDS exchange
// buffer stays at 64 KB
template <class F>
constexpr int stitch_bs() { return xyzz_words<F>() > 64 ? 128 : 256; }
// items per block of the level-0 stitch (the quad-cooperative kernel's 64 for G1)
template <class F>
constexpr int stitch_bs0() { return (ZK_STITCH_QUAD && is_base_field<F>()) ? STITCH_QBS : stitch_bs<F>(); }

static size_t stitch_slots0(const MsmShape &s) {  // item slots of the largest split's accumulation
  size_t m = 0;
  for (int h = 0; h < s.NS; h++) {
    const size_t ch = (size_t)s.split_ch(h);
    m = std::max(m, 2 * (((size_t)s.W * (s.split_lo(h + 1) - s.split_lo(h)) + ch - 1) / ch));
  }
  return m;
}
static size_t stitch_slots1(const MsmShape &s, int bs) { return 2 * ((stitch_slots0(s) + bs - 1) / bs) + 2; }

// sorted entries of one pipeline pass: passes of several windows are kept at <= 2^30 entries
// (memory per pass, swept sizes); a single window of n points is always one pass, so a pass
// holds at most n < 2^31 entries (the C ABI's int) -- every entry index, offset and point
// index (with the sign in bit 31) fits a u32, and hipCUB only scans the count matrix and
// the item flags (far below 2^31 entries)
constexpr size_t MSM_MAX_GROUP_ENTRIES = (size_t)1 << 30;
constexpr size_t MSM_MAX_PASS_ENTRIES = ((size_t)1 << 31) - 1;
// test hook (zkg_msm_set_group_limit): a smaller cap, so tests reach the multi-group path
// at small sizes; 0 restores the default
inline std::atomic<size_t> &msm_group_limit() {
  static std::atomic<size_t> v{MSM_MAX_GROUP_ENTRIES};
  return v;
}

// device bytes of the per-pass buffers
template <class C>
static size_t group_bytes(const MsmShape &s) {
  using F = typename C::Fp;
  const size_t xw = xyzz_words<F>() * 4;  // bytes per XYZZ
  const size_t nb = (size_t)s.W * s.B;
  const size_t maxent = (size_t)s.W * s.n;
  const size_t ns0 = stitch_slots0(s), ns1 = stitch_slots1(s, stitch_bs0<F>());
  size_t cub = 0, cub2 = 0;
  ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)(s.nmat() + 1)));
  ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub2, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)ns0));
  if (s.s2) {
    size_t cub3 = 0;
    ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub3, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)(s.nmat2() + 1)));
    if (cub3 > cub2) cub2 = cub3;
  }
  size_t bytes = 0;
  auto add = [&](size_t b) { bytes += (b + 255) & ~size_t(255); };
  add(maxent * 4 * 3);                    // digits, level-1 values, list
  add(maxent * 2);                        // level-1 fine indices
  add((s.nmat() + 1) * 4 * 2);            // level-1 counts, their scan
  if (s.s2) {
    add(maxent * 2);                      // level-1.5 fine indices (values reuse the digits' buffer)
    add((s.nmat2() + 1) * 4 * 2);         // level-1.5 counts, their scan
  }
  add(s.NS * (nb + 1) * 4);               // offsets (every split)
  add(nb);                                // filled flags (split pipelines)
  add(ns0 * (xw + 4) + ns0 * 16 + 64);    // level-0 items, compacted keys + index, flags, pos, count
  add(ns1 * (xw + 4) * 2);                // stitch ping-pong
  add(nb * xw);                           // buckets
  add((size_t)s.W * s.NY * xw);           // Y
  add(cub > cub2 ? cub : cub2);
  if (s.NS > 1) add(cub > cub2 ? cub : cub2);  // the sort stream's own scan scratch
  return bytes + (1 << 20);
}

// window groups (pipeline passes) of the most recent msm_run, for tests of the degrade path
inline std::atomic<int> &msm_last_groups() {
  static std::atomic<int> v{0};
  return v;
}

// Opt-in phase profile (zkg_msm_profile(1)): HIP events between the phases of every call,
// printed to stderr with the host-side finish time.  Off by default.
inline std::atomic<int> &msm_profile_flag() {
  static std::atomic<int> on{0};
  return on;
}
struct PhaseProf {
  bool on = false;
  hipStream_t st = nullptr;
  std::vector<std::pair<const char *, hipEvent_t>> ev;
  explicit PhaseProf(hipStream_t s) : st(s) {
    on = msm_profile_flag().load() != 0;
    mark("start");
  }
  void mark(const char *name) {
    if (!on) return;
    hipEvent_t e;
    ZK_CHECK(hipEventCreate(&e));
    ZK_CHECK(hipEventRecord(e, st));
    ev.emplace_back(name, e);
  }
  void report(double host_ms) {
    if (!on) return;
    ZK_CHECK(hipStreamSynchronize(st));
    fprintf(stderr, "[zk msm]");
    for (size_t i = 1; i < ev.size(); i++) {
      float ms = 0;
      ZK_CHECK(hipEventElapsedTime(&ms, ev[i - 1].second, ev[i].second));
      fprintf(stderr, " %s=%.3f", ev[i].first, ms);
    }
    fprintf(stderr, " host_finish=%.3f ms\n", host_ms);
    for (auto &e : ev) ZK_CHECK(hipEventDestroy(e.second));
    ev.clear();
  }
};

// Where the scalars of one pipeline run come from: row i holds `stride` u64 limbs, the
// scalar is limbs [loff, loff + nread) (nread <= 4) -- Montgomery Fr or a plain integer
struct ScalarSlice {
  const uint64_t *data;
  int stride, loff, nread;
  bool mont;
};

// One pass of the device pipeline over windows [wbase, wbase + s.W): digits, bucket sort,
// accumulation, stitch, Y sums, job sums, export; the (window, job) sums land in the pinned
// host buffer h (reference-form XYZZ, window-major).  launch() enqueues everything on the
// pass's stream without a host round trip; finish() waits for it.  With NS point splits every
// split is sorted into its own list region and accumulated on its own (split pipelines, for
// host inputs that arrive split by split).
template <class C>
struct GroupPass {
  using F = typename C::Fp;
  static constexpr int STITCH_BS = stitch_bs<F>();
  Device &dev;
  MsmShape s;
  ScalarSlice sc;
  int wbase, timer_slot;
  const uint32_t *pts_int;
  uint64_t *h;
  PhaseProf *prof;
  hipStream_t st;
  size_t nb, xw, maxent, ns0, ns1, cub = 0;
  uint32_t *list, *dig, *tmpv, *cnt, *coff, *offsets, *ikeys0, *ivals0, *ckeys, *cidx, *flags, *pos, *ccount;
  uint16_t *tmpf, *tmpf2 = nullptr;
  uint32_t *cnt2 = nullptr, *coff2 = nullptr;
  uint32_t *okA, *ovA, *okB, *ovB, *buckets, *Y;
  void *cubtmp;
  uint8_t *filled = nullptr;  // split pipelines: bucket b holds a sum from an earlier split
  // host inputs: the sorts run on their own stream (sst, with their own scan scratch) beside the
  // previous split's accumulation, and the points of split h (reference form, pts_ref) are
  // converted on the main stream right before its accumulation -- the copy stream carries
  // copies only
  hipStream_t sst = nullptr;
  void *cubtmp_sort = nullptr;
  const uint64_t *pts_ref = nullptr;
  std::vector<hipEvent_t> sorted_ev;
  // sort-ahead (msm_run, large device-resident inputs): the pass was sorted on another stream,
  // which records this event; launch() waits for it instead of sorting
  hipEvent_t presorted = nullptr;
  // stitch state (level ping-pong)
  const uint32_t *inK, *inV;
  size_t slots;
  uint32_t *outK, *outV, *altK, *altV;

  GroupPass(Device &d, const MsmShape &shape, const ScalarSlice &scal, int wb, const uint32_t *pts, uint64_t *hh,
            PhaseProf *pr, hipStream_t stream, int tslot)
      : dev(d), s(shape), sc(scal), wbase(wb), timer_slot(tslot), pts_int(pts), h(hh), prof(pr), st(stream) {
    const int n = s.n;
    nb = (size_t)s.W * s.B;
    xw = xyzz_words<F>();
    maxent = (size_t)s.W * n;
    ZK_REQUIRE(maxent <= MSM_MAX_PASS_ENTRIES, "msm: window group exceeds the sort capacity (internal sizing bug)");
    list = dev.arena.take<uint32_t>(maxent);  // bucket-ordered (point index | sign)
    dig = dev.arena.take<uint32_t>(maxent);   // |digit| | sign per (window, point)
    tmpv = dev.arena.take<uint32_t>(maxent);  // level-1 order: values
    tmpf = dev.arena.take<uint16_t>(maxent);  // level-1 order: fine bucket within the coarse bin
    cnt = dev.arena.take<uint32_t>(s.nmat() + 1);
    coff = dev.arena.take<uint32_t>(s.nmat() + 1);
    if (s.s2) {
      tmpf2 = dev.arena.take<uint16_t>(maxent);
      cnt2 = dev.arena.take<uint32_t>(s.nmat2() + 1);
      coff2 = dev.arena.take<uint32_t>(s.nmat2() + 1);
    }
    offsets = dev.arena.take<uint32_t>((size_t)s.NS * (nb + 1));  // split h: offsets + h (nb + 1)
    if (s.NS > 1) filled = dev.arena.take<uint8_t>(nb);
    ns0 = stitch_slots0(s);
    ns1 = stitch_slots1(s, stitch_bs0<F>());
    ikeys0 = dev.arena.take<uint32_t>(ns0);
    ivals0 = dev.arena.take<uint32_t>(ns0 * xw);
    ckeys = dev.arena.take<uint32_t>(ns0);
    cidx = dev.arena.take<uint32_t>(ns0);
    flags = dev.arena.take<uint32_t>(ns0);
    pos = dev.arena.take<uint32_t>(ns0);
    ccount = dev.arena.take<uint32_t>(16);
    okA = dev.arena.take<uint32_t>(ns1);
    ovA = dev.arena.take<uint32_t>(ns1 * xw);
    okB = dev.arena.take<uint32_t>(ns1);
    ovB = dev.arena.take<uint32_t>(ns1 * xw);
    buckets = dev.arena.take<uint32_t>(nb * xw);
    Y = dev.arena.take<uint32_t>((size_t)s.W * s.NY * xw);
    size_t cub2 = 0;
    ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub, cnt, coff, (int)(s.nmat() + 1), st));
    ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub2, flags, pos, (int)ns0, st));
    if (cub2 > cub) cub = cub2;
    if (s.s2) {
      size_t cub3 = 0;
      ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub3, cnt2, coff2, (int)(s.nmat2() + 1), st));
      if (cub3 > cub) cub = cub3;
    }
    cubtmp = dev.arena.take<char>(cub);
    if (s.NS > 1) cubtmp_sort = dev.arena.take<char>(cub);
  }
  void mark(const char *what) {  // the phase profile follows the first group's stream
    if (prof && wbase == 0) prof->mark(what);
  }

  // bucket sort of split sp's points [lo, hi): digits, level-1 count / scan / scatter, level 2;
  // its entries go to the list region [W lo, W hi), its offsets to offsets + sp (nb + 1)
  void sort(int sp, hipStream_t st, void *cubtmp) {
    const int n = s.n, c = s.c;
    const int lo = s.split_lo(sp), hi = s.split_lo(sp + 1);
    const uint32_t base = (uint32_t)((size_t)s.W * lo);
    hipLaunchKernelGGL(k_digits<C>, dim3(div_up(hi - lo, 256)), dim3(256), 0, st, sc.data, n, lo, hi, sc.stride,
                       sc.loff, sc.nread, sc.mont ? 1 : 0, c, wbase, s.W, dig);
    ZK_CHECK(hipGetLastError());
    if (st == this->st) mark("digits");
    const dim3 grid((unsigned)s.nwg, (unsigned)s.W);
    hipLaunchKernelGGL(k_coarse<false>, grid, dim3(256), 0, st, dig, n, lo, hi, s.M, s.fs, s.nbins, cnt, tmpv + base,
                       tmpf + base);
    ZK_CHECK(hipGetLastError());
    size_t cb = cub;
    ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(cubtmp, cb, cnt, coff, (int)(s.nmat() + 1), st));
    hipLaunchKernelGGL(k_coarse<true>, grid, dim3(256), 0, st, dig, n, lo, hi, s.M, s.fs, s.nbins, coff, tmpv + base,
                       tmpf + base);
    ZK_CHECK(hipGetLastError());
    // level 1.5 when the coarse bins outgrow level 2's staging: sub-bins of this split's region
    // (values into the digits' buffer, dead after level 1; the sorts of later splits follow on the
    // same stream, so their digits are written only after this split's level 2 has read it)
    const uint32_t *fv = tmpv + base, *fcoff = coff;
    const uint16_t *ff = tmpf + base;
    int fnwg = s.nwg, fs = s.fs;
    uint32_t nq = (uint32_t)(s.W * s.nbins);
    if (s.s2) {
      const int nsub = 1 << s.s2, s2sh = s.fs - s.s2;
      const dim3 g2((unsigned)s.nwg2, nq);
      hipLaunchKernelGGL(k_split<false>, g2, dim3(256), 0, st, coff, s.nwg, s2sh, nsub, cnt2, tmpv + base, tmpf + base,
                         dig + base, tmpf2 + base);
      ZK_CHECK(hipGetLastError());
      size_t cb2 = cub;
      ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(cubtmp, cb2, cnt2, coff2, (int)(s.nmat2() + 1), st));
      hipLaunchKernelGGL(k_split<true>, g2, dim3(256), 0, st, coff, s.nwg, s2sh, nsub, coff2, tmpv + base, tmpf + base,
                         dig + base, tmpf2 + base);
      ZK_CHECK(hipGetLastError());
      fv = dig + base;
      ff = tmpf2 + base;
      fcoff = coff2;
      fnwg = s.nwg2;
      fs = s2sh;
      nq *= (uint32_t)nsub;
    }
    const int cap = fine_stage_cap(fs);
    const int lds = (4 << fs) + 4 * cap;
    if ((size_t)(hi - lo) * s.W >= (size_t)nq * 4096) {  // bins of >= 4096 entries: the wide workgroup
      ZK_CHECK(hipFuncSetAttribute((const void *)k_fine<1024, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   lds));
      hipLaunchKernelGGL((k_fine<1024, 4, true>), dim3(nq), dim3(1024), lds, st, fcoff, fnwg, nq, fs, cap, fv, ff,
                         list + base, offsets + (size_t)sp * (nb + 1), base);
    } else {
      ZK_CHECK(hipFuncSetAttribute((const void *)k_fine<256, 1, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   lds));
      hipLaunchKernelGGL((k_fine<256, 1, false>), dim3(nq), dim3(256), lds, st, fcoff, fnwg, nq, fs, cap, fv, ff,
                         list + base, offsets + (size_t)sp * (nb + 1), base);
    }
    ZK_CHECK(hipGetLastError());
    if (st == this->st) mark("sort");
  }

  // accumulation of split sp: list range [offsets[sp nb], offsets[(sp+1) nb]); a run that starts
  // in a lane's chunk begins from the earlier splits' bucket sum (filled)
  // host inputs: split h's scalars / points are on the device once the copy thread has recorded
  // wait_sc[h] / wait_pt[h] (ready flags: an event must be recorded, in host order, before a
  // stream waits on it)
  std::vector<hipEvent_t> wait_sc, wait_pt;
  const std::atomic<int> *ready_sc = nullptr, *ready_pt = nullptr;
  void wait_for(hipStream_t on, const std::vector<hipEvent_t> &ev, const std::atomic<int> *ready, int sp) {
    if (sp >= (int)ev.size() || !ev[sp]) return;
    if (ready)
      while (!ready[sp].load(std::memory_order_acquire)) std::this_thread::yield();
    ZK_CHECK(hipStreamWaitEvent(on, ev[sp], 0));
  }
  // host inputs: split sp's points (landed in pts_ref) -> internal form, on the main stream
  void convert(int sp) {
    const int lo = s.split_lo(sp), hi = s.split_lo(sp + 1);
    if (hi <= lo) return;
    hipLaunchKernelGGL(k_points_int<C>, dim3(div_up(hi - lo, 256)), dim3(256), 0, st,
                       pts_ref + (size_t)lo * 2 * C::NP64, hi - lo, const_cast<uint32_t *>(pts_int) + (size_t)lo * aff_words<F>());
    ZK_CHECK(hipGetLastError());
  }
  int ch0 = 0;  // chunk length of the accumulation whose items the stitch is summing
  void accumulate(int sp) {
    if (sp == 0) timer_begin(dev, timer_slot, st);
    const size_t npts = (size_t)s.split_lo(sp + 1) - (size_t)s.split_lo(sp);
    const int CH = s.split_ch(sp);
    ch0 = CH;
    const size_t nsl = 2 * (((size_t)s.W * npts + CH - 1) / CH);  // <= ns0
    // upper bound on the chunk count; threads past the range's end only clear their item slots
    hipLaunchKernelGGL(k_accum<C>, dim3(div_up(nsl / 2, 256)), dim3(256), 0, st, pts_int, list,
                       offsets + (size_t)sp * (nb + 1), (uint32_t)nb, CH, (uint32_t)s.W, (uint32_t)s.B, buckets,
                       ikeys0, ivals0, (uint32_t)nsl, (const uint8_t *)(sp > 0 ? filled : nullptr));
    ZK_CHECK(hipGetLastError());
    if (sp == s.NS - 1) timer_end(dev, timer_slot, st);
    mark("accum");
    inK = ikeys0;
    inV = ivals0;
    slots = nsl;
    level = 0;
    outK = okA; outV = ovA; altK = okB; altV = ovB;
  }
  void fill_mark(int sp) {
    hipLaunchKernelGGL(k_fill_mark, dim3(div_up(nb, 256)), dim3(256), 0, st, offsets + (size_t)sp * (nb + 1),
                       (uint32_t)nb, sp == 0 ? 1 : 0, filled);
    ZK_CHECK(hipGetLastError());
  }

  // stitch level: compact the partial items, sum them per bucket (k_stitch_blk); true when
  // every item completed at this level
  int level = 0;
  bool stitch_level() {
    const bool raw = ZK_STITCH_RAW && level++ > 0;
    // the quad-cooperative level-0 kernel wins where its blocks fit about one round on the chip:
    // few item slots (small inputs) or long chunks (CH 64: runs mostly complete inside a lane or
    // merged in-wave, so few items survive compaction); with many items (2^16-2^18, CH 10-32)
    // the one-lane kernel's 4x fewer blocks win (BLS12-381 2^16: 0.196 vs 0.220 ms stitch,
    // 2^10: 0.150 vs 0.094, 2^20: 0.052 vs 0.041; profiles/r04f_*)
    const bool quad0 = stitch_bs0<F>() == STITCH_QBS && (ns0 <= 65536 || ch0 >= 64);
    const int bs = raw ? STITCH_BS : (quad0 ? STITCH_QBS : STITCH_BS);  // items per block at this level
    const bool final_level = slots <= (size_t)bs;  // all items fit one block: everything completes
    const size_t nout = final_level ? 2 : 2 * ((slots + bs - 1) / bs);
    if (raw) {  // one kernel per level, straight on the slots
      hipLaunchKernelGGL((k_stitch_raw<C, STITCH_BS>), dim3((unsigned)((slots + STITCH_BS - 1) / STITCH_BS)),
                         dim3(STITCH_BS), 0, st, inK, inV, (uint32_t)slots, (uint32_t)nb, final_level ? 1 : 0,
                         buckets, outK, outV);
      ZK_CHECK(hipGetLastError());
    } else {  // device-wide compaction of the valid slots, then the Hillis-Steele block stitch
      hipLaunchKernelGGL(k_item_flags, dim3(div_up(slots, 256)), dim3(256), 0, st, inK, (const uint32_t *)nullptr,
                         (uint32_t)slots, (uint32_t)nb, flags);
      ZK_CHECK(hipGetLastError());
      size_t cb = cub;
      ZK_CHECK(hipcub::DeviceScan::ExclusiveSum(cubtmp, cb, flags, pos, (int)slots, st));
      hipLaunchKernelGGL(k_item_index, dim3(div_up(slots, 256)), dim3(256), 0, st, inK, flags, pos, (uint32_t)slots,
                         ckeys, cidx, ccount);
      ZK_CHECK(hipGetLastError());
      bool launched = false;
      if constexpr (stitch_bs0<F>() == STITCH_QBS) {
        if (quad0) {
          hipLaunchKernelGGL(k_stitch_blk_q<C>, dim3((unsigned)(nout / 2)), dim3(256), 0, st, ckeys, cidx, inV, ccount,
                             (uint32_t)nb, buckets, outK, outV, (uint32_t)nout);
          launched = true;
        }
      }
      if (!launched)
        hipLaunchKernelGGL((k_stitch_blk<C, STITCH_BS>), dim3((unsigned)(nout / 2)), dim3(STITCH_BS), 0, st, ckeys,
                           cidx, inV, ccount, (uint32_t)nb, (uint32_t)s.W, (uint32_t)s.B, buckets, outK, outV,
                           (uint32_t)nout);
      ZK_CHECK(hipGetLastError());
    }
    inK = outK; inV = outV; slots = nout;
    uint32_t *tk = outK, *tv = outV;
    outK = altK; outV = altV; altK = tk; altV = tv;
    return final_level;
  }

  // Y sums, job sums, export and the copy back to the host
  void reduce_tail() {
    const int c = s.c;
    const int n0 = s.r0.count * s.r0.G, n1 = s.r1.count * s.r1.G;
    if (n0 % 256 == 0 && n1 % 256 == 0) {  // block-level Y sums (every shape from c = 12 up)
      const unsigned nblk = (unsigned)(s.W * (n0 + n1) / 256);
      bool two_waves = false;  // k_ysum3 (G1 only: not instantiated for Fp2 points)
      if constexpr (is_base_field<F>()) {
        two_waves = ysum3_on((size_t)nblk * 256);
        if (two_waves)
          hipLaunchKernelGGL((k_ysum3<C>), dim3(nblk), dim3(256), 0, st, buckets, offsets, (const uint8_t *)filled,
                             s.W, c, s.l0, s.r0, s.r1, Y);
      } else if (ysum_g2_lds<F>()) {
        // Fp2 (round 6, A/B): the LDS-gather form at one wave per SIMD -- the register prefetch of
        // k_ysum2 holds a whole Fp2 XYZZ bucket (112 / 72 VGPRs), and BLS12-381's k_ysum2 spills
        // 247 VGPRs to scratch at 512 + 256 AGPRs; the LDS image is 128 / 80 KB per block
        two_waves = true;
        hipLaunchKernelGGL((k_ysum3<C, 1>), dim3(nblk), dim3(256), 0, st, buckets, offsets, (const uint8_t *)filled,
                           s.W, c, s.l0, s.r0, s.r1, Y);
      }
      if (!two_waves)
        hipLaunchKernelGGL((k_ysum2<C, is_base_field<F>() ? ZK_YSUM_PF != 0 : ZK_YSUM_PF_G2 != 0>), dim3(nblk),
                           dim3(256), 0, st, buckets, offsets,
                           (const uint8_t *)filled, s.W, c, s.l0, s.r0, s.r1, Y);
    } else {  // small shapes: in-wavefront segments
      const size_t lanes = (size_t)s.W * s.ylanes;
      hipLaunchKernelGGL(k_ysum<C>, dim3(div_up(lanes, 256)), dim3(256), 0, st, buckets, offsets,
                         (const uint8_t *)filled, s.W, c, s.l0, s.r0, s.r1, s.ylanes, Y);
    }
    ZK_CHECK(hipGetLastError());
    mark("ysum");
    // the job sums land straight in the pinned host buffer (mapped at the same address on the
    // device): no copy, and no copy-engine start-up after the last kernel
    hipLaunchKernelGGL(k_jobsum_blk<C>, dim3((unsigned)(s.W * c)), dim3(256), 0, st, Y, c, s.l0, h);
    ZK_CHECK(hipGetLastError());
    mark("jobsum");
  }

  // Everything is enqueued without a host round trip.  The stitch levels are deterministic: a
  // level of S item slots leaves 2 ceil(S / STITCH_BS) slots, and the level whose slots fit one
  // block completes every run whatever the scalars (skewed inputs only make the runs longer),
  // so all levels are launched up front (3 at BLS12-381 2^20, 4 at 2^26); with split pipelines
  // the next split starts from complete buckets without the host looking at any count.
  void launch() {
    for (int sp = 0; sp < s.NS; sp++) {
      if (presorted) {  // one split (msm_run's sort-ahead shape)
        ZK_CHECK(hipStreamWaitEvent(st, presorted, 0));
      } else if (sst) {  // split sp's sort on the sort stream, beside split sp-1's accumulation
        wait_for(sst, wait_sc, ready_sc, sp);
        sort(sp, sst, cubtmp_sort);
        ZK_CHECK(hipEventRecord(sorted_ev[sp], sst));
      } else {
        wait_for(st, wait_sc, ready_sc, sp);
        sort(sp, st, cubtmp);
      }
      wait_for(st, wait_pt, ready_pt, sp);
      if (pts_ref) convert(sp);
      if (sst) ZK_CHECK(hipStreamWaitEvent(st, sorted_ev[sp], 0));
      accumulate(sp);
      for (bool final_level = false; !final_level;) final_level = stitch_level();
      if (s.NS > 1) fill_mark(sp);
    }
    mark("stitch");
    reduce_tail();
  }
  void finish() {
    stream_wait(dev, st);
    mark("export");
  }
};

// host: combine the per-(window, job) sums (XYZZ, canonical reference form; job order
// of k_jobsum: total, U_{0,0..l0-1}, U_{1,0..l1-1}):
//   V_w = sum_j 2^(e_j) P_{w,j}, e_j = 0 (total), j - 1 (bit jobs)   [Horner over c - 1 exponents]
//   result = sum_w 2^(c w) V_w                                        [Horner over the windows]
// The V_w are independent: the host pool computes them, top window first, WHILE the calling
// thread runs the cross-window chain of c (W - 1) doublings (Jacobian, 2M + 5S each),
// waiting for each V_w only when the chain reaches it.  On one host core a point op costs
// ~0.4 us against ~20 us for a lone GPU lane, which is why this tail stays on the host.
// bits > 0: the small-input layout instead (k_bitsum): `bits` sums Q_t, t = 0 .. bits-1, in
// windows of c: job j of window w is Q_{c w + j} with exponent j.
template <class C>
static void finish_host(int c, int W, const uint64_t *exported, zkh::Xyzz<typename HostOf<C>::Fp> &out,
                        int bits = 0) {
  using HF = typename HostOf<C>::Fp;
  const int NP = C::NP64;
  const int J = c, E = bits ? c : c - 1;  // local exponents 0 .. E-1
  std::vector<zkh::Jac<HF>> V(W);
  std::unique_ptr<std::atomic<int>[]> ready(new std::atomic<int>[W]);
  for (int w = 0; w < W; w++) ready[w].store(0, std::memory_order_relaxed);
  // windows are claimed top first from one counter, by the pool's workers and by the calling
  // thread whenever the chain reaches a window nobody has finished: the chain never waits for a
  // worker's wake-up (~50 us), and a window is never computed twice
  std::atomic<int> next_win{0};
  auto window = [&](int i) {
    const int w = W - 1 - i;
    std::vector<zkh::Xyzz<HF>> Z(E);
    for (auto &z : Z) zkh::xyzz_set_inf(z);
    for (int j = 0; j < J; j++) {
      if (bits && c * w + j >= bits) break;
      const uint64_t *q = exported + ((size_t)w * J + j) * 4 * NP;
      zkh::Xyzz<HF> p;
      memcpy(p.X.v, q + 0 * NP, NP * 8);
      memcpy(p.Y.v, q + 1 * NP, NP * 8);
      memcpy(p.ZZ.v, q + 2 * NP, NP * 8);
      memcpy(p.ZZZ.v, q + 3 * NP, NP * 8);
      if (zkh::xyzz_is_inf(p)) continue;
      const int e = bits ? j : (j == 0 ? 0 : j - 1);
      zkh::xyzz_add(Z[e], Z[e], p);
    }
    zkh::Xyzz<HF> acc;
    zkh::xyzz_set_inf(acc);
    for (int e = E - 1; e >= 0; e--) {
      zkh::xyzz_dbl(acc, acc);
      zkh::xyzz_add(acc, acc, Z[e]);
    }
    zkh::xyzz_to_jac(V[w], acc);
    ready[w].store(1, std::memory_order_release);
  };
  zkh::Jac<HF> acc;
  zkh::jac_set_inf(acc);
  auto claim = [&]() -> bool {  // computes the next unclaimed window; false when none is left
    const int i = next_win.fetch_add(1);
    if (i >= W) return false;
    window(i);
    return true;
  };
  auto chain = [&] {
    for (int w = W - 1; w >= 0; w--) {
      for (int k = 0; k < c; k++) zkh::jac_dbl(acc, acc);
      while (!ready[w].load(std::memory_order_acquire))
        if (!claim()) std::this_thread::yield();
      zkh::jac_add(acc, acc, V[w]);
    }
  };
  const int nthreads = W < 8 ? W : 8;
  host_parallel_for_main(nthreads, [&](int) { while (claim()) {} }, chain);
  zkh::jac_to_xyzz(out, acc);
}

// Largest n that takes the bit-job path (default-window calls).  ZK_MSM_BITS_MAX overrides it
// (experiment / A-B hook, read once; 0 = always the bucket pipeline).
#ifndef ZK_MSM_BITS_MAX
#define ZK_MSM_BITS_MAX 4096
#endif
inline int msm_bits_max() {
  static const int v = [] {
    const char *e = getenv("ZK_MSM_BITS_MAX");
    return e ? atoi(e) : ZK_MSM_BITS_MAX;
  }();
  return v;
}
// chunks of the bit-job accumulation: ~256 blocks (one wavefront per SIMD for the 4 x 64 bits)
// so a lane's chain is K = n / 256 mixed additions; ZK_MSM_BITS_G overrides the block count
inline int msm_bits_groups(int n) {
  static const int g = [] {
    const char *e = getenv("ZK_MSM_BITS_G");
    const int v = e ? atoi(e) : 256;
    return v >= 1 ? v : 256;
  }();
  int K = (n + g - 1) / g;
  if (K > BITACC_MAX_K) K = BITACC_MAX_K;  // whatever the hooks say: k_bitacc's LDS holds 256 scalars
  return (n + K - 1) / K;
}

// The small-input path (k_bitacc / k_bitsum above): points to internal form, bit-job partial
// sums, per-bit sums exported to the host, Horner over the bits in windows of 8 on the host.
template <class C>
static void msm_run_bits(Device &dev, int n, const ScalarSlice &sc_in, const uint64_t *points, bool host_inputs,
                         int nbits, zkh::Xyzz<typename HostOf<C>::Fp> &out) {
  using F = typename C::Fp;
  constexpr int XW = xyzz_words<F>();
  ZK_REQUIRE(nbits >= 1 && nbits <= 256, "msm: bit-job path takes at most 256-bit scalars (internal)");
  const int G = msm_bits_groups(n), K = (n + G - 1) / G;
  ZK_REQUIRE(K >= 1 && K <= BITACC_MAX_K, "msm: bit-job chunk larger than k_bitacc's LDS staging (internal)");
  hipStream_t st = dev.stream;
  const size_t sc_bytes = host_inputs ? (size_t)n * sc_in.stride * 8 : 0;
  const size_t pt_bytes = host_inputs ? (size_t)n * 2 * C::NP64 * 8 : 0;
  const size_t int_bytes = (size_t)n * aff_words<F>() * 4;
  const size_t part_bytes = (size_t)nbits * G * XW * 4;
  const size_t exp_bytes = (size_t)nbits * 4 * C::NP64 * 8;
  const size_t need = sc_bytes + pt_bytes + int_bytes + part_bytes + 4 * 256;
  if (!dev.arena.try_reserve(need)) {
    ZK_CHECK(hipStreamSynchronize(st));
    ntt_release(dev);
    ZK_REQUIRE(dev.arena.try_reserve(need), "msm: out of device memory");
  }
  dev.arena.reset();
  msm_last_groups().store(1);
  PhaseProf prof(st);
  ScalarSlice sc = sc_in;
  const uint64_t *pts_ref = points;
  if (host_inputs) {
    uint64_t *a = dev.arena.take<uint64_t>((size_t)n * sc_in.stride);
    uint64_t *b = dev.arena.take<uint64_t>((size_t)n * 2 * C::NP64);
    ZK_CHECK(hipMemcpyAsync(a, sc_in.data, sc_bytes, hipMemcpyHostToDevice, st));
    ZK_CHECK(hipMemcpyAsync(b, points, pt_bytes, hipMemcpyHostToDevice, st));
    sc.data = a;
    pts_ref = b;
  }
  uint32_t *pts_int = dev.arena.take<uint32_t>((size_t)n * aff_words<F>());
  uint32_t *part = dev.arena.take<uint32_t>((size_t)nbits * G * XW);
  uint64_t *h = reinterpret_cast<uint64_t *>(dev.host_staging(exp_bytes + 64));  // k_bitsum writes here
  hipLaunchKernelGGL(k_points_int<C>, dim3(div_up(n, 256)), dim3(256), 0, st, pts_ref, n, pts_int);
  ZK_CHECK(hipGetLastError());
  prof.mark("points");
  timer_begin(dev, 0, st);
  hipLaunchKernelGGL(k_bitacc<C>, dim3((unsigned)G), dim3(256), 0, st, sc.data, n, sc.stride, sc.loff, sc.nread,
                     sc.mont ? 1 : 0, nbits, K, pts_int, part);
  ZK_CHECK(hipGetLastError());
  timer_end(dev, 0, st);
  prof.mark("bitacc");
  hipLaunchKernelGGL(k_bitsum<C>, dim3((unsigned)nbits), dim3(256), 0, st, part, G, h);
  ZK_CHECK(hipGetLastError());
  prof.mark("bitsum");
  stream_wait(dev, st);
  prof.mark("export");
  timer_collect(dev);
  const auto t0 = std::chrono::steady_clock::now();
  constexpr int BW = 8;  // host Horner windows over the bits
  finish_host<C>(BW, (nbits + BW - 1) / BW, h, out, nbits);
  prof.report(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

// Sort-ahead: device-resident inputs of at least 2^ZK_MSM_AHEAD_MIN pairs (default 23; read once,
// A/B hook) whose windows fit one pass run as TWO window groups whose bucket sorts both go to the
// context's sort stream: group A's beside the point conversion, group B's beside group A's
// accumulation.  Window groups are independent sums, so unlike point splits this adds no
// additions.  It pays only where k_accum leaves VGPRs free for the sort's wavefronts: the 254-bit
// madd at three waves per SIMD (153 VGPRs) -- BN128 2^24 26.97 -> 26.35 ms -- while the 381-bit
// one fills the register file at two (2 x 254): there the sort waits for accumulation waves to
// retire and the accumulation grows by what the sort saved (BLS12-381 2^23 22.53 / 22.63 ms, 2^24
// 39.94 / 39.99, profiles/r05x_sort_ahead.txt).  Below 2^23 the halved Y-sum / job-sum / stitch
// launches (latency-bound at c = 16) cost about what the hidden sort saves.
inline int msm_ahead_default() {
  static const int v = [] {
    const char *e = getenv("ZK_MSM_AHEAD_MIN");
    return e ? atoi(e) : 23;
  }();
  return v;
}
inline std::atomic<int> &msm_ahead_min() {  // zkg_msm_set_ahead_min (test hook): < 0 the default
  static std::atomic<int> v{-1};
  return v;
}
// (Sorting ONE group on the sort stream beside the point conversion measured no better: BLS12-381
// 2^20 3.565 vs 3.506 ms, 2^24 39.23 vs 39.34 ms, profiles/r05x_sort_ahead.txt.)
template <class C>
static bool msm_ahead(int n, bool host_inputs, int W, int Wg) {
  if (host_inputs || Wg != W || W < 2) return false;
  const int set = msm_ahead_min().load();  // the test hook applies to every field
  const int lg = set >= 0 ? set : (AccumOcc<typename C::Fp>::waves >= 3 ? msm_ahead_default() : 0);
  return lg > 0 && lg < 31 && (size_t)n >= ((size_t)1 << lg);
}

// Run the device pipeline for one scalar slice.  points are DEVICE pointers (or host
// pointers when host_inputs, in which case they are staged, with the scalars).
// Result: sum_i k_i P_i in host XYZZ (reference Montgomery form).
template <class C>
static void msm_run(Device &dev, int n, const ScalarSlice &sc_in, const uint64_t *points, bool host_inputs,
                    int window, zkh::Xyzz<typename HostOf<C>::Fp> &out) {
  using F = typename C::Fp;
  if (n <= 0) {
    zkh::xyzz_set_inf(out);
    return;
  }
  const bool explicit_window = window >= 4 && window <= 24;
  const int bits = sc_in.mont ? HostOf<C>::Fr::BITS : 64 * sc_in.nread;
  const int c = explicit_window ? window
                                : (is_base_field<F>() ? msm_default_window_bits(n, bits) : msm_default_window(n));
  // small inputs with the default window: bit jobs, no buckets (an explicit window -- the
  // reference's _variable entry -- always runs the bucket method it names)
  if (!explicit_window && n <= msm_bits_max()) {
    msm_run_bits<C>(dev, n, sc_in, points, host_inputs, bits, out);
    return;
  }
  // Signed digits need floor(bits/c) + 1 windows: the top window then holds at most c-1
  // bits plus the carry, i.e. a digit <= 2^(c-1) = B, so no carry leaves it.
  const int W = bits / c + 1;
  // window groups: one pipeline pass sorts at most msm_group_limit() entries (2^30 by default)
  // or one window (n < 2^31 entries, MSM_MAX_PASS_ENTRIES)
  int Wg = (int)std::min<size_t>((size_t)W, std::max<size_t>(1, msm_group_limit().load() / (size_t)n));
  hipStream_t st = dev.stream;

  const size_t sc_bytes = host_inputs ? (size_t)n * sc_in.stride * 8 : 0;
  const size_t pt_bytes = host_inputs ? (size_t)n * 2 * C::NP64 * 8 : 0;
  const size_t int_bytes = (size_t)n * aff_words<F>() * 4;
  // Working set: when the device cannot hold it, drop this context's cached NTT twiddles, then
  // halve the windows per pass (the result does not depend on the grouping) down to one window
  // before giving up -- instead of aborting the caller's process on the first failed hipMalloc.
  bool dropped_twiddles = false;
  // Host inputs in one pipeline pass: the pairs are split msm_splits() ways, split h is sorted
  // and accumulated as soon as its scalars and points have landed while the next split's cross PCIe
  auto splits = [&](int wg) { return msm_splits(n, host_inputs, wg == W); };
  MsmShape s = make_shape(n, c, Wg, splits(Wg));
  const int Wa = (W + 1) / 2;
  const bool ahead = msm_ahead<C>(n, host_inputs, W, Wg) &&
                     dev.arena.try_reserve(int_bytes + 3 * 256 + group_bytes<C>(make_shape(n, c, Wa, 1)) +
                                           group_bytes<C>(make_shape(n, c, W - Wa, 1)));
  while (!ahead && !dev.arena.try_reserve(sc_bytes + pt_bytes + int_bytes + 3 * 256 + group_bytes<C>(s))) {
    if (!dropped_twiddles) {
      ZK_CHECK(hipStreamSynchronize(st));
      ntt_release(dev);
      dropped_twiddles = true;
      continue;
    }
    ZK_REQUIRE(Wg > 1, "msm: out of device memory (one window per pass does not fit)");
    Wg = (Wg + 1) / 2;
    s = make_shape(n, c, Wg, splits(Wg));
  }
  const int NS = s.NS;
  msm_last_groups().store(ahead ? 2 : (W + Wg - 1) / Wg);
  dev.arena.reset();
  ScalarSlice sc = sc_in;
  uint32_t *pts_int = nullptr;
  PhaseProf prof(st);
  bool inputs_on_aux = false;
  std::atomic<int> ready_sc[ZK_MSM_SPLITS_MAX], ready_pt[ZK_MSM_SPLITS_MAX];
  std::string copy_err;  // an Error of the copy thread (recoverable error mode), rethrown after join
  std::mutex copy_mu;
  std::vector<std::thread> copier_v;  // the copy thread, joined on every exit (JoinAll)
  JoinAll join_copier{copier_v};
  uint64_t *pts_ref = nullptr;  // host inputs: the device copy of the caller's (reference-form) points
  if (host_inputs) {
    uint64_t *a = dev.arena.take<uint64_t>((size_t)n * sc_in.stride);
    uint64_t *b = dev.arena.take<uint64_t>((size_t)n * 2 * C::NP64);
    pts_int = dev.arena.take<uint32_t>((size_t)n * aff_words<F>());
    sc.data = a;
    pts_ref = b;
    // Caller memory is pageable; the runtime's pageable path runs at PCIe rate on MI355X hosts
    // (56 GB/s measured, tools/microbench/copy_bw.hip), a pinned bounce buffer only adds a host
    // copy -- but a pageable copy returns only once it is staged, so the copies are issued by a
    // thread of their own on the context's second stream, split by split (scalars, then points),
    // each recording an event; that stream carries nothing but copies.  The calling thread
    // enqueues split h's sort (on the sort stream) behind its scalars, and its point conversion
    // and accumulation (main stream) behind its points, so split h is accumulated while split h+1
    // still crosses PCIe.  (Round 3 converted the points on the copy stream: every conversion then
    // delayed the next copy, and ran beside an accumulation at a tenth of its speed --
    // profiles/r04b_e2e_trace.txt.)
    hipStream_t st2 = dev.aux_stream();
    for (int h = 0; h < 3 * NS; h++) dev.split_event(h);  // created here, before the thread uses them
    for (int h = 0; h < NS; h++) {
      ready_sc[h].store(0, std::memory_order_relaxed);
      ready_pt[h].store(0, std::memory_order_relaxed);
    }
    const int stride = sc_in.stride;
    const uint64_t *sc_host = sc_in.data;
    const MsmShape shp = s;
    copier_v.emplace_back([&dev, st2, NS, shp, a, b, stride, sc_host, points, &ready_sc, &ready_pt, &copy_err,
                           &copy_mu] {
      catch_into(&copy_err, &copy_mu, [&] {
      ZK_CHECK(hipSetDevice(dev.id));
      for (int h = 0; h < NS; h++) {
        const int lo = shp.split_lo(h), hi = shp.split_lo(h + 1);
        ZK_CHECK(hipMemcpyAsync(a + (size_t)lo * stride, sc_host + (size_t)lo * stride,
                                (size_t)(hi - lo) * stride * 8, hipMemcpyHostToDevice, st2));
        ZK_CHECK(hipEventRecord(dev.split_event(3 * h), st2));
        ready_sc[h].store(1, std::memory_order_release);
        const size_t off = (size_t)lo * 2 * C::NP64;
        ZK_CHECK(hipMemcpyAsync(b + off, points + off, (size_t)(hi - lo) * 2 * C::NP64 * 8, hipMemcpyHostToDevice, st2));
        ZK_CHECK(hipEventRecord(dev.split_event(3 * h + 1), st2));
        ready_pt[h].store(1, std::memory_order_release);
      }
      });
      for (int h = 0; h < NS; h++) {  // after an error too: the waiting pipeline must not spin forever
        ready_sc[h].store(1, std::memory_order_release);
        ready_pt[h].store(1, std::memory_order_release);
      }
    });
    inputs_on_aux = true;
  } else {
    pts_int = dev.arena.take<uint32_t>((size_t)n * aff_words<F>());
    if (ahead) ZK_CHECK(hipEventRecord(dev.split_event(0), st));  // the sorts start behind the caller's work
    hipLaunchKernelGGL(k_points_int<C>, dim3(div_up(n, 256)), dim3(256), 0, st, points, n, pts_int);
    ZK_CHECK(hipGetLastError());
  }
  prof.mark("points");
  const size_t mark = dev.arena.used();
  const size_t per_w = (size_t)c * 4 * C::NP64;  // exported u64 per window
  uint64_t *h = reinterpret_cast<uint64_t *>(dev.host_staging((size_t)W * per_w * 8 + 64));
  if (ahead) {
    GroupPass<C> pa(dev, make_shape(n, c, Wa, 1), sc, 0, pts_int, h, &prof, st, 0);
    GroupPass<C> pb(dev, make_shape(n, c, W - Wa, 1), sc, Wa, pts_int, h + (size_t)Wa * per_w, &prof, st, 1);
    hipStream_t sst = dev.aux2_stream();
    ZK_CHECK(hipStreamWaitEvent(sst, dev.split_event(0), 0));
    pa.sort(0, sst, pa.cubtmp);
    ZK_CHECK(hipEventRecord(dev.split_event(1), sst));
    pb.sort(0, sst, pb.cubtmp);
    ZK_CHECK(hipEventRecord(dev.split_event(2), sst));
    pa.presorted = dev.split_event(1);
    pb.presorted = dev.split_event(2);
    pa.launch();
    pb.launch();  // waits for B's sort: every sort-stream kernel is complete before pb.finish()
    pb.finish();
    timer_collect(dev);
    const auto t0 = std::chrono::steady_clock::now();
    finish_host<C>(c, W, h, out);
    prof.report(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    return;
  }
  // Window groups run one after the other on the device's stream.  (Running two groups
  // concurrently on two streams -- one's sort and latency-bound tail beside the other's
  // accumulation -- was measured and does not pay: the two accumulations overlap each
  // other instead, profiles/r02t_pipelined_groups_ab.txt.)
  for (int wbase = 0; wbase < W; wbase += Wg) {
    dev.arena.rewind(mark);
    const MsmShape sg = (wbase + Wg <= W) ? s : make_shape(n, c, W - wbase);
    GroupPass<C> pass(dev, sg, sc, wbase, pts_int, h + (size_t)wbase * per_w, &prof, st, wbase == 0 ? 0 : -1);
    if (inputs_on_aux) {  // joined by the first group: later groups follow on the same stream
      // (only a single-pass shape is split, so the first group has the splits of the copies)
      ZK_REQUIRE(sg.NS == NS, "msm: split pipeline shape mismatch (internal)");
      for (int h = 0; h < NS; h++) {
        pass.wait_sc.push_back(dev.split_event(3 * h));
        pass.wait_pt.push_back(dev.split_event(3 * h + 1));
        pass.sorted_ev.push_back(dev.split_event(3 * h + 2));
      }
      pass.ready_sc = ready_sc;
      pass.ready_pt = ready_pt;
      pass.pts_ref = pts_ref;
      // ZK_MSM_SORT_INLINE=1 (A/B hook, read once): every split's sort on the main stream, in line
      static const bool sort_inline = [] {
        const char *e = getenv("ZK_MSM_SORT_INLINE");
        return e && e[0] == '1';
      }();
      if (NS > 1 && !sort_inline) pass.sst = dev.aux2_stream();
    }
    inputs_on_aux = false;
    pass.launch();
    for (auto &t : copier_v)
      if (t.joinable()) t.join();  // every copy is issued (the stream order does the rest)
    pass.finish();
    rethrow_first(copy_err);
  }
  timer_collect(dev);
  const auto t0 = std::chrono::steady_clock::now();
  finish_host<C>(c, W, h, out);
  prof.report(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

// ---------------------------------------------------------------------------
// public (C++) entry point used by the C ABI layer

// Device bytes of one msm_run's working set (what its arena reserves) with the W windows in
// `groups` passes -- exposed for memory planning and the degrade-path tests.
template <class C>
size_t msm_workspace_bytes(int n, int nl, bool mont, bool host_inputs, int window, int groups) {
  using F = typename C::Fp;
  if (n <= 0) return 0;
  const int nread = nl < 4 ? nl : 4;
  const int nbits = mont ? HostOf<C>::Fr::BITS : 64 * nread;
  if (!(window >= 4 && window <= 24) && n <= msm_bits_max()) {  // the bit-job path (msm_run_bits)
    const size_t io = host_inputs ? (size_t)n * nl * 8 + (size_t)n * 2 * C::NP64 * 8 : 0;
    return io + (size_t)n * aff_words<F>() * 4 + (size_t)nbits * msm_bits_groups(n) * xyzz_words<F>() * 4 + 4 * 256;
  }
  const int c = (window >= 4 && window <= 24)
                    ? window
                    : (is_base_field<F>() ? msm_default_window_bits(n, nbits) : msm_default_window(n));
  const int W = nbits / c + 1;
  const int g = groups < 1 ? 1 : (groups > W ? W : groups);
  const int Wg = (W + g - 1) / g;
  const size_t sc_bytes = host_inputs ? (size_t)n * nl * 8 : 0;
  const size_t pt_bytes = host_inputs ? (size_t)n * 2 * C::NP64 * 8 : 0;
  const size_t int_bytes = (size_t)n * aff_words<F>() * 4;
  const int NS = msm_splits(n, host_inputs, Wg == W);
  if (msm_ahead<C>(n, host_inputs, W, Wg)) {
    const int Wa = (W + 1) / 2;
    return int_bytes + 3 * 256 + group_bytes<C>(make_shape(n, c, Wa, 1)) + group_bytes<C>(make_shape(n, c, W - Wa, 1));
  }
  return sc_bytes + pt_bytes + int_bytes + 3 * 256 + group_bytes<C>(make_shape(n, c, Wg, NS));
}

// One complete MSM on one device context (caller holds dev.mu): every scalar slice.
template <class C>
static void msm_xyzz(Device &dev, int n, const uint64_t *scalars, int nl, const uint64_t *points, bool host_inputs,
                     bool mont, int window, zkh::Xyzz<typename HostOf<C>::Fp> &acc) {
  using HF = typename HostOf<C>::Fp;
  if (mont || nl <= 4) {
    // Montgomery coefficients: the reference converts the first 4 limbs of each row
    // (Fr_mont_to_std reads 4 limbs, G1_proj.c:637-641); for expo_nlimbs != 4 its result
    // is undefined (it reads past the row / leaves limbs uninitialised), here the value of
    // the row's first min(nl, 4) limbs is used
    msm_run<C>(dev, n, ScalarSlice{scalars, nl, 0, nl < 4 ? nl : 4, mont}, points, host_inputs, window, acc);
  } else {
    // standard scalars wider than 256 bits, used verbatim like the reference
    // (G1_proj.c:511,552): k = sum_j k_j 2^(256 j) over 4-limb slices, one device MSM per
    // slice, combined by Horner on the host (256 doublings per slice)
    zkh::xyzz_set_inf(acc);
    const int nsl = (nl + 3) / 4;
    for (int j = nsl - 1; j >= 0; j--) {
      for (int k = 0; k < 256; k++) zkh::xyzz_dbl(acc, acc);
      const int nread = nl - 4 * j < 4 ? nl - 4 * j : 4;
      zkh::Xyzz<HF> r;
      msm_run<C>(dev, n, ScalarSlice{scalars, nl, 4 * j, nread, false}, points, host_inputs, window, r);
      zkh::xyzz_add(acc, acc, r);
    }
  }
}

template <class C>
void msm_g1(int n, const uint64_t *scalars, int nl, const uint64_t *points, bool host_inputs, bool mont,
            int window, uint64_t *out_proj) {
  using HF = typename HostOf<C>::Fp;
  ZK_REQUIRE(nl >= 1, "msm: expo_nlimbs must be >= 1");
  zkh::Xyzz<HF> acc;
  const std::vector<int> set = host_inputs ? device_set() : std::vector<int>();
  const int G = (int)set.size();
  if (G > 1 && n > 0) {
    // Host buffers with a device set (zkg_set_devices / ZKG_DEVICES): contiguous chunks
    // [n k / G, n (k+1) / G), one host thread per listed device (one context per occurrence of
    // a device id), each copying and computing only its chunk over its own PCIe link; the
    // partial sums are added in list order.  The affine result equals the unsharded one (a
    // group sum), and the reference's own call is a single chunk (G1_proj.c:630-644).
    std::vector<zkh::Xyzz<HF>> part(G);
    std::vector<std::thread> th;
    std::string err;
    std::mutex emu;
    {
    JoinAll join_all{th};
    for (int k = 0; k < G; k++) {
      const size_t lo = (size_t)n * k / G, hi = (size_t)n * (k + 1) / G;
      int slot = 0;
      for (int j = 0; j < k; j++) slot += set[j] == set[k];
      zkh::xyzz_set_inf(part[k]);
      if (hi == lo) continue;
      th.emplace_back([&, k, lo, hi, slot] {
        catch_into(&err, &emu, [&] {
          ZK_CHECK(hipSetDevice(set[k]));
          Device &d = device_context(set[k], slot);
          std::lock_guard<std::mutex> lock(d.mu);
          msm_xyzz<C>(d, (int)(hi - lo), scalars + lo * nl, nl, points + lo * 2 * C::NP64, true, mont, window,
                      part[k]);
        });
      });
    }
    }  // joined
    rethrow_first(err);
    zkh::xyzz_set_inf(acc);
    for (int k = 0; k < G; k++) zkh::xyzz_add(acc, acc, part[k]);
  } else if (G == 1) {  // a one-entry set pins the host-buffer MSM to that device
    DeviceGuard on(set[0]);
    Device &dev = current_device();
    std::lock_guard<std::mutex> lock(dev.mu);
    msm_xyzz<C>(dev, n, scalars, nl, points, host_inputs, mont, window, acc);
  } else {
    Device &dev = current_device();
    std::lock_guard<std::mutex> lock(dev.mu);
    msm_xyzz<C>(dev, n, scalars, nl, points, host_inputs, mont, window, acc);
  }
  zkh::Proj<HF> p;
  zkh::xyzz_to_proj(p, acc);
  memcpy(out_proj + 0 * C::NP64, p.X.v, C::NP64 * 8);
  memcpy(out_proj + 1 * C::NP64, p.Y.v, C::NP64 * 8);
  memcpy(out_proj + 2 * C::NP64, p.Z.v, C::NP64 * 8);
}

}  // namespace zk
