// zk_ntt.hip -- forward / inverse NTT over the scalar field Fr (BN128, BLS12-381).
//
// Replaces <C>_poly_mont_ntt_forward / _inverse (bls12_381_poly_mont.c:418-463 and
// :472-522; bn128_poly_mont.c same lines).  The reference computes
//   forward:  tgt[k] = sum_j src[j] * gen^(j k)                 (recursive radix-2 DIT)
//   inverse:  tgt[j] = (1/N) * sum_k src[k] * gen^(-j k)       (recursive DIF, x 1/2 per level)
// with natural-order input and output, N = 2^m.  Both are exact field computations
// with canonical outputs, so any correct schedule reproduces them bit for bit.
//
// GPU schedule (MI355X-first): N = R_0 * R_1 * ... * R_{P-1}, R_p = 2^r_p <= 256, i.e.
// P = ceil(m/8) HBM passes (3 at 2^24); m <= 11 runs as one workgroup-sized pass.
// Pass p performs, inside LDS, R_p-point DFTs along digit p (stride S_p =
// R_{p+1}...R_{P-1}) for a tile of G consecutive columns (coalesced 128-B row segments),
// as radix-4 rounds (two radix-2 DIT stages per LDS round trip), then multiplies output
// k_p by the inter-pass twiddle w^(T_p * k_p * lo) (T_p = R_0...R_{p-1}, lo = the column
// below digit p) read from a precomputed per-pass table.  The last pass writes each
// output straight to its natural index k = sum_q k_q T_q (no bit-reversal pass).
// Inverse: w -> w^-1 and the 1/N factor folded into pass 0's twiddle table.
// Twiddle tables are built on the device once per (curve, m, gen, direction) and cached.
#include <algorithm>
#include <atomic>
#include <map>
#include <thread>
#include <tuple>
#include <vector>
#include "zk_field.hpp"
#include "zk_host.hpp"
#include "zk_runtime.hpp"
#include "zk_ntt.hpp"

namespace zk {

// Two pass-kernel widths: 256 threads over 1024-element tiles (36 KB of LDS, 4 workgroups
// per CU) for DFTs of up to 2^8 points, and 1024 threads over 4096-element tiles (144 KB: one
// workgroup per CU) for the 2^9..2^12-point DFTs of the two-pass schedule (2^17..2^24).
constexpr int NTT_THREADS = 256;
constexpr int NTT_TILE = 1024;  // elements per workgroup tile for multi-pass transforms
constexpr int NTT_THREADS_BIG = 1024;
constexpr int NTT_TILE_BIG = 4096;
// Inner twiddles are read from a global (L1/L2-resident, a few KB) internal-limb table with
// 48-B rows (3 x 16-B loads) rather than staged in LDS: the 1024-element tile alone is
// 36 KB, so dropping the 4.6 KB twiddle copy lets 4 instead of 3 workgroups share a CU.
constexpr int ITW_STRIDE = 12;

// ---------------------------------------------------------------------------- tables

// w^e from the two-level tables (internal form, stored packed canonical)
template <class F>
__device__ __forceinline__ void tw2(Fe<F> &w, const uint64_t *__restrict__ tlo, const uint64_t *__restrict__ thi,
                                    int h, uint32_t e) {
  Fe<F> a, b;
  fe_load_ref(a, tlo + (size_t)(e & ((1u << h) - 1)) * F::N64);
  fe_load_ref(b, thi + (size_t)(e >> h) * F::N64);
  fe_mul(w, a, b);
}

// tlo[i] = w^i (i < 2^h), thi[i] = w^(i 2^h) (i < 2^(m-h)); pows = reference-form w^(2^b)
template <class F>
__global__ void k_tw_tables(uint64_t *__restrict__ tlo, uint64_t *__restrict__ thi, int h, int m,
                            const uint64_t *__restrict__ pows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int nlo = 1 << h, nhi = 1 << (m - h);
  for (int which = 0; which < 2; which++) {
    const int cnt = which ? nhi : nlo;
    if (i >= cnt) continue;
    const int base = which ? h : 0, nb = which ? m - h : h;
    Fe<F> acc;
    fe_one(acc);
    for (int b = 0; b < nb; b++)
      if ((i >> b) & 1) {
        Fe<F> p, q, t;
        fe_load_ref(q, pows + (size_t)(b + base) * F::N64);
        fe_to_int(p, q);
        fe_mul(t, acc, p);
        acc = t;
      }
    fe_store_ref((which ? thi : tlo) + (size_t)i * F::N64, acc);
  }
}

// per-pass table: tab[k*S + lo] = w^(T k lo) (* scale, if given), k < R, lo < S
template <class F>
__global__ void k_tw_pass(uint64_t *__restrict__ tab, int R, int S, uint32_t T, const uint64_t *__restrict__ tlo,
                          const uint64_t *__restrict__ thi, int h, const uint64_t *__restrict__ scale) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)R * S) return;
  const uint32_t k = (uint32_t)(idx / S), lo = (uint32_t)(idx % S);
  Fe<F> w;
  tw2(w, tlo, thi, h, T * k * lo);
  if (scale) {
    Fe<F> s, t, u;
    fe_load_ref(s, scale);
    fe_to_int(t, s);
    fe_mul(u, w, t);
    w = u;
  }
  fe_store_ref(tab + idx * F::N64, w);
}

// inner twiddles of an R-point DFT: itw[j] = w_R^j = w^(j N/R), j < R/2
template <class F>
__global__ void k_tw_inner(uint64_t *__restrict__ itw, int m, int r, const uint64_t *__restrict__ tlo,
                           const uint64_t *__restrict__ thi, int h) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (1 << r) / 2) return;
  Fe<F> w;
  tw2(w, tlo, thi, h, (uint32_t)j << (m - r));
  fe_store_ref(itw + (size_t)j * F::N64, w);
}

// the same table in internal limbs, ITW_STRIDE u32 per entry (exactly what fe_load_ref gives)
template <class F>
__global__ void k_tw_inner_int(uint32_t *__restrict__ itw_i, const uint64_t *__restrict__ itw, int n) {
  static_assert(F::N <= ITW_STRIDE, "inner twiddle rows hold F::N limbs");
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  Fe<F> w;
  fe_load_ref(w, itw + (size_t)j * F::N64);
#pragma unroll
  for (int q = 0; q < ITW_STRIDE; q++) itw_i[(size_t)j * ITW_STRIDE + q] = q < F::N ? w.v[q] : 0u;
}

// ---------------------------------------------------------------------------- pass kernel

// LDS slot of tile element I: an XOR swizzle of the low 6 index bits by bits 6..11, so that
// every access pattern of the pass (bit-reversed loads, the radix-4 rounds at every stride,
// G-interleaved stores) hits 64 distinct banks with 9-word elements, for the 1024-element
// tiles (R = 2^8, G = 4) and every 4096-element tile shape (R = 2^9..2^12) -- checked by brute
// force over the wave access patterns (tools/ntt_lds_banks.py); the plain layout had 4-16-way
// conflicts (rocprofv3 SQ_LDS_BANK_CONFLICT was 80 % of the LDS-active cycles,
// profiles/r02o_ntt_lds.txt)
__device__ __forceinline__ uint32_t lds_slot(uint32_t I) {
  const uint32_t m1 = (I >> 6) & 3, m2 = (I >> 8) & 3, m3 = (I >> 10) & 3;
  const uint32_t x = m1 ^ m2, y = x ^ m3;
  return I ^ (m1 | (x << 2) | (y << 4));
}

// value < 2^(64 N64) with normalised limbs -> N64 u64 words, as is (no canonicalisation)
template <class F>
__device__ __forceinline__ void fe_store_packed(uint64_t *__restrict__ p, const Fe<F> &a) {
  uint32_t w[F::NW];
  fe_pack(w, a);
  uint4 *q = reinterpret_cast<uint4 *>(p);
#pragma unroll
  for (int i = 0; i < F::NW / 4; i++) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

template <class F>
__device__ __forceinline__ void lds_get(Fe<F> &x, const uint32_t *p) {
#pragma unroll
  for (int q = 0; q < F::N; q++) x.v[q] = p[q];
}
template <class F>
__device__ __forceinline__ void lds_put(uint32_t *p, const Fe<F> &x) {
#pragma unroll
  for (int q = 0; q < F::N; q++) p[q] = x.v[q];
}

// in-LDS DIT over G instances of R points (bit-reversed input order -> natural order).
// Lazy butterflies (zk_field.hpp "lazy ops"): x = a + t, y = a + 4p - t with no carries
// or reductions; limbs are renormalised once per radix-4 round when written back to LDS.
// Value bound: inputs < 2p (canonical input, or the previous pass's product output), every
// stage adds < 4p, so after R = 2^8 points (8 stages) values are < 34p, well inside fe_mul's
// input range (R'/p > 68) and fe_reduce_small's (< 64p): the products of the next stage and
// the pass's closing product (twiddle / scale) or reduction bring them back below 2p.  (The
// 4096-point tiles add 12 stages: < 50p.)  Limb bound: normalised (< 2^29) at round entry, < 2^31.4 at round exit.
// Every radix 2^1..2^12, both Fr fields, every closing step (table twiddle, on-the-fly twiddle
// = a product of two canonical entries < 1.02p, 1/N scale, fe_reduce_small) and the inter-pass
// fixed point (values < 1.72p between passes) are checked by tools/lazy_bounds.py.
template <class F, int NT>
__device__ __forceinline__ void lds_dft(uint32_t *data, const uint32_t *__restrict__ itw, int r, int G) {
  constexpr int NW = F::N;
  const int R = 1 << r;
  const int tid = threadIdx.x;
  int s = 0;
  if (r >= 2) {  // first radix-4 round: twiddles w_2^0 = w_4^0 = 1, only w_4^1 is non-trivial
    const int q4 = R >> 2;
    Fe<F> w3;
    lds_get(w3, itw + (size_t)(R / 4) * ITW_STRIDE);  // w_4 = w_R^(R/4)
    for (int u = tid; u < G * q4; u += NT) {
      const int g = u / q4, j = u % q4;
      const int i0 = g * R + j * 4;
      Fe<F> a0, a1, a2, a3, b0, b1, b3, t;
      lds_get(a0, data + (size_t)lds_slot(i0) * NW);
      lds_get(a1, data + (size_t)lds_slot(i0 + 1) * NW);
      lds_get(a2, data + (size_t)lds_slot(i0 + 2) * NW);
      lds_get(a3, data + (size_t)lds_slot(i0 + 3) * NW);
      fe_add_lazy(b0, a0, a1);
      fe_sub_lazy(b1, a0, a1);
      fe_sub_lazy(b3, a2, a3);
      fe_mul(t, b3, w3);
      Fe<F> s23;
      fe_add_lazy(s23, a2, a3);
      fe_add_lazy(a0, b0, s23);
      fe_sub_lazy<F, 4, 2>(a2, b0, s23);  // s23 limbs <= 2 (2^RB - 1): borrow 2
      fe_add_lazy(a1, b1, t);
      fe_sub_lazy(a3, b1, t);
      fe_norm(a0);
      fe_norm(a1);
      fe_norm(a2);
      fe_norm(a3);
      lds_put(data + (size_t)lds_slot(i0) * NW, a0);
      lds_put(data + (size_t)lds_slot(i0 + 1) * NW, a1);
      lds_put(data + (size_t)lds_slot(i0 + 2) * NW, a2);
      lds_put(data + (size_t)lds_slot(i0 + 3) * NW, a3);
    }
    __syncthreads();
    s = 2;
  }
  for (; s + 1 < r; s += 2) {  // radix-4 rounds: stages s and s+1
    const int half = 1 << s;
    const int q4 = R >> 2;
    for (int u = tid; u < G * q4; u += NT) {
      const int g = u / q4, j = u % q4;
      const int blk = j >> s, off = j & (half - 1);
      const int i0 = g * R + blk * 4 * half + off;
      Fe<F> a0, a1, a2, a3, w1, w2, w3, t;
      lds_get(a0, data + (size_t)lds_slot(i0) * NW);
      lds_get(a1, data + (size_t)lds_slot(i0 + half) * NW);
      lds_get(a2, data + (size_t)lds_slot(i0 + 2 * half) * NW);
      lds_get(a3, data + (size_t)lds_slot(i0 + 3 * half) * NW);
      lds_get(w1, itw + (size_t)(off * (R / (2 * half))) * ITW_STRIDE);           // w_{2h}^off
      lds_get(w2, itw + (size_t)(off * (R / (4 * half))) * ITW_STRIDE);           // w_{4h}^off
      lds_get(w3, itw + (size_t)((off + half) * (R / (4 * half))) * ITW_STRIDE);  // w_{4h}^(off+h)
      // stage s
      Fe<F> b0, b1, b2, b3;
      fe_mul(t, a1, w1);
      fe_add_lazy(b0, a0, t);
      fe_sub_lazy(b1, a0, t);
      fe_mul(t, a3, w1);
      fe_add_lazy(b2, a2, t);
      fe_sub_lazy(b3, a2, t);
      // stage s+1
      fe_mul(t, b2, w2);
      fe_add_lazy(a0, b0, t);
      fe_sub_lazy(a2, b0, t);
      fe_mul(t, b3, w3);
      fe_add_lazy(a1, b1, t);
      fe_sub_lazy(a3, b1, t);
      fe_norm(a0);
      fe_norm(a1);
      fe_norm(a2);
      fe_norm(a3);
      lds_put(data + (size_t)lds_slot(i0) * NW, a0);
      lds_put(data + (size_t)lds_slot(i0 + half) * NW, a1);
      lds_put(data + (size_t)lds_slot(i0 + 2 * half) * NW, a2);
      lds_put(data + (size_t)lds_slot(i0 + 3 * half) * NW, a3);
    }
    __syncthreads();
  }
  if (s < r) {  // odd r: one radix-2 stage left
    const int half = 1 << s;
    const int q2 = R >> 1;
    for (int u = tid; u < G * q2; u += NT) {
      const int g = u / q2, j = u % q2;
      const int blk = j >> s, off = j & (half - 1);
      const int i0 = g * R + blk * 2 * half + off;
      Fe<F> a, b, w, t, x, y;
      lds_get(a, data + (size_t)lds_slot(i0) * NW);
      lds_get(b, data + (size_t)lds_slot(i0 + half) * NW);
      lds_get(w, itw + (size_t)(off * (R / (2 * half))) * ITW_STRIDE);
      fe_mul(t, b, w);
      fe_add_lazy(x, a, t);
      fe_sub_lazy(y, a, t);
      fe_norm(x);
      fe_norm(y);
      lds_put(data + (size_t)lds_slot(i0) * NW, x);
      lds_put(data + (size_t)lds_slot(i0 + half) * NW, y);
    }
    __syncthreads();
  }
}

struct PassArgs {
  int m, r, S, T, last, G, P;
  int h;    // split of the two-level power tables (tlo: 2^h entries)
  int otf;  // non-last pass: inter-pass twiddles computed from tlo/thi instead of a table
  int dig[8];  // log2 radix of every pass
};

// Inter-pass twiddle tables hold R_p * S_p entries (32 B each); a pass whose table would
// exceed 2^25 entries (1 GiB) computes its twiddles on the fly from the two-level tables
// (one more product per element) instead.  At 2^24 pass 0's table is the whole
// transform's size (512 MiB) and still pays: the pass is VALU-bound, and computing the
// twiddles measured 0.08 ms slower per transform than streaming them (profiles/r02p_*).
#ifndef ZK_NTT_TABLE_MAX
#define ZK_NTT_TABLE_MAX ((size_t)1 << 25)
#endif
static std::atomic<size_t> g_ntt_table_max{0};  // test hook (ntt_set_table_max); 0 = the default
void ntt_set_table_max(size_t entries) { g_ntt_table_max.store(entries); }
static size_t ntt_table_max() {
  const size_t v = g_ntt_table_max.load();
  return v ? v : ZK_NTT_TABLE_MAX;
}

// One pass.  Block = one tile of G instances x R elements.
//   non-last pass: instance (hi, lo), lo in [0, S); element k at hi*R*S + k*S + lo
//                  tile = G consecutive lo for one hi; output * tab[k*S + lo]
//   last pass    : S == 1; instance = position prefix (k_0..k_{P-2}); element k at inst*R + k;
//                  tile = G instances with consecutive k_0; output to natural index
template <class F, int NT>
__global__ void __launch_bounds__(NT) k_ntt_pass(const uint64_t *__restrict__ src, uint64_t *__restrict__ dst,
                                                          PassArgs a, const uint32_t *__restrict__ itw_i,
                                                          const uint64_t *__restrict__ tab,
                                                          const uint64_t *__restrict__ scale,
                                                          const uint64_t *__restrict__ tlo,
                                                          const uint64_t *__restrict__ thi) {
  extern __shared__ uint32_t lds[];
  constexpr int NW = F::N;
  const int r = a.r, G = a.G, S = a.S;
  const int R = 1 << r;
  uint32_t *data = lds;                          // [G][R] elements
  const uint32_t *itw = (const uint32_t *)__builtin_assume_aligned(itw_i, 16);  // [R/2] inner twiddles
  const int tid = threadIdx.x;
  const int tile = blockIdx.x;

  // instance geometry of this tile
  size_t hi_base = 0;  // non-last: hi * R * S + lo0
  size_t pos_base = 0, nat_base = 0;  // last: position / natural index of instance k_0 = k0base
  int k0base = 0, k0stride_pos = 0;
  if (!a.last) {
    const int ntl = S / G;
    hi_base = (size_t)(tile / ntl) * R * S + (size_t)(tile % ntl) * G;
  } else if (a.P > 1) {
    const int R0 = 1 << a.dig[0];
    const int ntile0 = R0 / G;
    k0base = (tile % ntile0) * G;
    int rem = tile / ntile0;
    size_t Sq = (size_t)1 << a.m;
    size_t Tq = (size_t)R0;
    for (int q = 0; q < a.P - 1; q++) {
      Sq >>= a.dig[q];
      if (q == 0) {
        k0stride_pos = (int)(Sq >> r);  // position stride of k_0, in units of R
      } else {
        const int kq = rem & ((1 << a.dig[q]) - 1);
        rem >>= a.dig[q];
        pos_base += (size_t)kq * Sq;
        nat_base += (size_t)kq * Tq;
        Tq <<= a.dig[q];
      }
    }
  }

  // load: element (g, k) -> LDS slot g*R + bitrev_r(k)
  const int nel = G * R;
  for (int e = tid; e < nel; e += NT) {
    int g, k;
    size_t addr;
    if (!a.last) {
      g = e % G;
      k = e / G;
      addr = hi_base + (size_t)k * S + g;
    } else {
      g = e / R;
      k = e % R;
      addr = pos_base + ((size_t)(k0base + g) * k0stride_pos) * R + k;
      if (a.P == 1) addr = k;
    }
    Fe<F> x;
    fe_load_ref(x, src + addr * F::N64);
    const int kr = r ? (int)(__builtin_bitreverse32((uint32_t)k) >> (32 - r)) : 0;
    lds_put(data + (size_t)lds_slot((uint32_t)(g * R + kr)) * NW, x);
  }
  __syncthreads();

  lds_dft<F, NT>(data, itw, r, G);

  // Output: one loop per closing mode (uniform per launch), so every mode is its own loop in
  // the ISA (tools/ntt_isa_model.py prices each pass from these loops)
  //   non-last pass: x * w, w from the pass's table or (otf) tw2; stored packed, not canonical
  //                  (a product is < 2p < 2^256; the next pass only multiplies and adds it)
  //   last pass:     the lazily grown value (< 50p) back below 2p, as fe_store_ref's
  //                  canonicalisation needs -- by the product with the scale (1/N) when an
  //                  inverse's scale has no table to ride on, else by a product-free reduction
  auto out_addr = [&](int g, int k) -> size_t {
    if (!a.last) return hi_base + (size_t)k * S + g;
    return (a.P == 1) ? (size_t)k : nat_base + (size_t)(k0base + g) + (size_t)k * a.T;
  };
  if (!a.last && !a.otf) {
    for (int e = tid; e < nel; e += NT) {
      const int g = e % G, k = e / G;  // consecutive threads -> consecutive g (coalesced)
      Fe<F> x, w, y;
      lds_get(x, data + (size_t)lds_slot((uint32_t)(g * R + k)) * NW);
      const size_t addr = out_addr(g, k);
      fe_load_ref(w, tab + ((size_t)k * S + (addr % S)) * F::N64);
      fe_mul(y, x, w);
      fe_store_packed(dst + addr * F::N64, y);
    }
  } else if (!a.last) {
    for (int e = tid; e < nel; e += NT) {
      const int g = e % G, k = e / G;
      Fe<F> x, w, y;
      lds_get(x, data + (size_t)lds_slot((uint32_t)(g * R + k)) * NW);
      const size_t addr = out_addr(g, k);
      tw2(w, tlo, thi, a.h, (uint32_t)a.T * (uint32_t)k * (uint32_t)(addr % S));
      fe_mul(y, x, w);
      fe_store_packed(dst + addr * F::N64, y);
    }
  } else if (scale) {
    Fe<F> sc, t;
    fe_load_ref(t, scale);
    fe_to_int(sc, t);
    for (int e = tid; e < nel; e += NT) {
      const int g = e % G, k = e / G;
      Fe<F> x, y;
      lds_get(x, data + (size_t)lds_slot((uint32_t)(g * R + k)) * NW);
      fe_mul(y, x, sc);
      fe_store_ref(dst + out_addr(g, k) * F::N64, y);
    }
  } else {
    for (int e = tid; e < nel; e += NT) {
      const int g = e % G, k = e / G;
      Fe<F> x;
      lds_get(x, data + (size_t)lds_slot((uint32_t)(g * R + k)) * NW);
      fe_reduce_small(x);
      fe_store_ref(dst + out_addr(g, k) * F::N64, x);
    }
  }
}

// ---------------------------------------------------------------------------- host side

// Pass split.  Default: three-or-more passes of <= 2^8-point DFTs on 1024-element tiles,
// except 2^20 = 2^10 x 2^10, which runs as two passes on 4096-element tiles (G = 4 columns:
// 128-B row segments, 256 tiles per pass): 0.128 vs 0.144 ms (profiles/r02am_ntt_two_pass.txt).
// Two passes lose elsewhere: below 2^20 a pass has fewer than 256 tiles (2^18: 0.101 vs
// 0.057 ms), above it the column pass gets G <= 2 columns, i.e. 32- or 64-B row segments
// (2^22: 0.575 vs 0.556 ms; 2^24 = 2^12 x 2^12: 2.65 vs 2.09 ms, 2.42 ms with the 4 workgroups
// sharing each 128-B line placed on one XCD).  Test hook zkg_ntt_set_max_radix: 12 forces the
// two-pass split for every 2^17..2^24, 8 forbids it, 0 restores the default.
static std::atomic<int> g_ntt_max_radix{0};
void ntt_set_max_radix(int r) { g_ntt_max_radix.store(r == 8 || r == 12 ? r : 0); }

static void split_digits(int m, std::vector<int> &d) {
  d.clear();
  if (m == 0) { d.push_back(0); return; }
  if (m <= 11) { d.push_back(m); return; }  // one workgroup-sized DFT
  const int mode = g_ntt_max_radix.load();
  if ((mode == 12 && m >= 17 && m <= 24) || (mode == 0 && m == 20)) {  // two passes, 2^9..2^12 points each
    d.push_back((m + 1) / 2);
    d.push_back(m / 2);
    return;
  }
  const int P = (m + 7) / 8;
  const int base = m / P, extra = m % P;
  for (int p = 0; p < P; p++) d.push_back(base + (p < extra ? 1 : 0));
}

// cached twiddle set for one (curve, m, gen, direction)
struct TwSet {
  uint64_t *mem = nullptr;       // one allocation
  std::vector<uint64_t *> inner; // per pass: R_p/2 inner twiddles
  std::vector<uint32_t *> inner_i; // the same, internal limbs, ITW_STRIDE u32 per entry
  std::vector<uint64_t *> tab;   // per non-last pass: R_p * S_p table
  uint64_t *scale = nullptr;     // 1/N (reference form) for the last pass of an inverse, unless a table holds it
  uint64_t *tlo = nullptr, *thi = nullptr;  // two-level power tables (2^h and 2^(m-h) entries)
  int h = 0;
  size_t bytes = 0;
  uint64_t last_use = 0;
};
// (context uid, m | first radix << 8, direction, generator, table cap)
typedef std::tuple<int, int, int, uint64_t, uint64_t, uint64_t, uint64_t, size_t> TwKey;
static std::map<TwKey, TwSet> g_tw;  // entries of context d are only touched under d's mutex
static std::mutex g_tw_mu;          // guards the map structure itself
static uint64_t g_tw_clock = 0;
static const size_t TW_CACHE_LIMIT = (size_t)8 << 30;

template <class Cfg>
static TwSet &twiddles(Device &dev, int curve, int m, const uint64_t *gen_mont, bool inverse,
                       const std::vector<int> &dig) {
  using F = typename Cfg::Fd;
  using HF = typename Cfg::Fh;
  // the tables depend on the pass split too (the test hook can change it between calls)
  const size_t table_max = ntt_table_max();
  TwKey key(dev.uid * 2 + curve, m | (dig[0] << 8), inverse, gen_mont[0], gen_mont[1], gen_mont[2], gen_mont[3],
            table_max);
  std::lock_guard<std::mutex> lock(g_tw_mu);
  auto it = g_tw.find(key);
  if (it != g_tw.end()) {
    it->second.last_use = ++g_tw_clock;
    return it->second;
  }
  const size_t N = (size_t)1 << m;
  const int P = (int)dig.size();
  const int h = m / 2;
  const size_t el = F::N64;
  // host: w (or w^-1), its 2^b powers, 1/N
  zkh::Fe<HF> g;
  memcpy(g.v, gen_mont, sizeof g.v);
  if (inverse) zkh::inv(g, g);
  std::vector<uint64_t> pows((size_t)(m > 0 ? m : 1) * HF::N, 0);
  {
    zkh::Fe<HF> p = g;
    for (int b = 0; b < m; b++) {
      memcpy(&pows[(size_t)b * HF::N], p.v, sizeof p.v);
      zkh::sqr(p, p);
    }
  }
  zkh::Fe<HF> ninv;
  {
    zkh::Fe<HF> nn;
    zkh::set_zero(nn);
    nn.v[0] = (uint64_t)1 << m;
    zkh::to_mont(nn, nn);
    zkh::inv(ninv, nn);
  }
  // sizes
  size_t words = ((size_t)1 << h) * el + ((size_t)1 << (m - h)) * el + pows.size() + 2 * el;
  size_t S = N, T = 1;
  std::vector<size_t> tab_words(P, 0);
  for (int p = 0; p < P; p++) {
    S >>= dig[p];
    words += ((size_t)1 << dig[p]) / 2 * el + el;
    words += ((size_t)1 << dig[p]) / 2 * (ITW_STRIDE / 2) + 2;
    if (p < P - 1 && ((size_t)1 << dig[p]) * S <= table_max) {
      tab_words[p] = ((size_t)1 << dig[p]) * S * el;
      words += tab_words[p];
    }
    T <<= dig[p];
  }
  // evict least-recently used sets of this context beyond the cache limit (and, when the
  // device is out of memory, until the new set fits)
  auto evict_one = [&]() -> bool {
    auto victim = g_tw.end();
    for (auto i2 = g_tw.begin(); i2 != g_tw.end(); ++i2)
      if (std::get<0>(i2->first) / 2 == dev.uid &&
          (victim == g_tw.end() || i2->second.last_use < victim->second.last_use))
        victim = i2;
    if (victim == g_tw.end()) return false;
    ZK_CHECK(hipStreamSynchronize(dev.stream));
    ZK_CHECK(hipFree(victim->second.mem));
    g_tw.erase(victim);
    return true;
  };
  for (;;) {
    size_t total = words * 8;
    for (auto &kv : g_tw)
      if (std::get<0>(kv.first) / 2 == dev.uid) total += kv.second.bytes;
    if (total <= TW_CACHE_LIMIT || !evict_one()) break;
  }
  TwSet ts;
  ts.bytes = words * 8;
  while (hipMalloc(&ts.mem, ts.bytes) != hipSuccess) {
    (void)hipGetLastError();
    ZK_REQUIRE(evict_one(), "ntt: out of device memory for the twiddle tables");
  }
  uint64_t *cur = ts.mem;
  auto take = [&](size_t w) { uint64_t *p = cur; cur += (w + 1) & ~size_t(1); return p; };
  uint64_t *tlo = take(((size_t)1 << h) * el);
  uint64_t *thi = take(((size_t)1 << (m - h)) * el);
  uint64_t *d_pows = take(pows.size());
  uint64_t *d_ninv = take(el);
  hipStream_t st = dev.stream;
  ZK_CHECK(hipMemcpyAsync(d_pows, pows.data(), pows.size() * 8, hipMemcpyHostToDevice, st));
  ZK_CHECK(hipMemcpyAsync(d_ninv, ninv.v, el * 8, hipMemcpyHostToDevice, st));
  {
    const int nt = 1 << (h > m - h ? h : m - h);
    hipLaunchKernelGGL(k_tw_tables<F>, dim3(div_up(nt, 256)), dim3(256), 0, st, tlo, thi, h, m, d_pows);
    ZK_CHECK(hipGetLastError());
  }
  S = N;
  T = 1;
  for (int p = 0; p < P; p++) {
    const int r = dig[p];
    S >>= r;
    uint64_t *inner = take(((size_t)1 << r) / 2 * el + el);
    if (r > 0) {
      hipLaunchKernelGGL(k_tw_inner<F>, dim3(div_up(((size_t)1 << r) / 2, 256)), dim3(256), 0, st, inner, m, r, tlo,
                         thi, h);
      ZK_CHECK(hipGetLastError());
    }
    ts.inner.push_back(inner);
    uint32_t *inner_i = (uint32_t *)take(((size_t)1 << r) / 2 * (ITW_STRIDE / 2) + 2);
    if (r > 0) {
      hipLaunchKernelGGL(k_tw_inner_int<F>, dim3(div_up(((size_t)1 << r) / 2, 256)), dim3(256), 0, st, inner_i, inner,
                         (1 << r) / 2);
      ZK_CHECK(hipGetLastError());
    }
    ts.inner_i.push_back(inner_i);
    if (p < P - 1 && tab_words[p]) {
      uint64_t *tab = take(tab_words[p]);
      const size_t cnt = ((size_t)1 << r) * S;
      hipLaunchKernelGGL(k_tw_pass<F>, dim3(div_up(cnt, 256)), dim3(256), 0, st, tab, 1 << r, (int)S, (uint32_t)T,
                         tlo, thi, h, (inverse && p == 0) ? d_ninv : nullptr);
      ZK_CHECK(hipGetLastError());
      ts.tab.push_back(tab);
    } else {
      ts.tab.push_back(nullptr);
    }
    T <<= r;
  }
  // the inverse's 1/N rides on pass 0's table when there is one, else on the last pass's
  // closing product
  ts.scale = (inverse && (P == 1 || !tab_words[0])) ? d_ninv : nullptr;
  ts.tlo = tlo;
  ts.thi = thi;
  ts.h = h;
  ts.last_use = ++g_tw_clock;
  return g_tw.emplace(key, ts).first->second;
}

struct CfgBN { using Fd = BN_Fr; using Fh = zkh::BN_Fr; };
struct CfgBLS { using Fd = BLS_Fr; using Fh = zkh::BLS_Fr; };

// Host I/O spread over a device set (zkg_set_devices): the transform runs on the first listed
// device; chunk k of the input / output crosses PCIe through listed device k (its own link) and
// moves between device k and the compute device over xGMI (peer copies; a plain device-to-device
// copy when both are the same GPU).  One host thread per helper drives its copies, so the links
// run concurrently.
struct Spread {
  std::vector<Device *> helpers;  // listed devices 1 .. G-1 (contexts, locked by the caller)
  int G = 1;
};

static void enable_peer(int a, int b) {
  if (a == b) return;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) {
    (void)hipGetLastError();
    return;
  }
  DeviceGuard on(a);
  const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
  if (e != hipSuccess) (void)hipGetLastError();  // already enabled
}

// chunk k of n bytes (k = 0 .. G-1), 4 KiB aligned boundaries
static void spread_chunk(size_t n, int G, int k, size_t &off, size_t &len) {
  const size_t a = (n / G * k) & ~(size_t)4095, b = k + 1 == G ? n : ((n / G * (k + 1)) & ~(size_t)4095);
  off = a;
  len = b - a;
}

// host -> device-0 buffer `d` (bytes), chunk 0 by dev0's own stream (caller's thread)
static void spread_in(Device &dev0, const Spread &sp, uint64_t *d, const uint64_t *h, size_t bytes) {
  std::vector<std::thread> th;
  std::string err;
  std::mutex emu;
  {
  JoinAll join_all{th};
  for (int k = 1; k < sp.G; k++) {
    th.emplace_back([&, k] { catch_into(&err, &emu, [&] {
      Device &hk = *sp.helpers[k - 1];
      size_t off, len;
      spread_chunk(bytes, sp.G, k, off, len);
      if (!len) return;
      ZK_CHECK(hipSetDevice(hk.id));
      uint64_t *buf = hk.arena.take<uint64_t>(len / 8);
      ZK_CHECK(hipMemcpyAsync(buf, (const char *)h + off, len, hipMemcpyHostToDevice, hk.stream));
      if (hk.id == dev0.id) ZK_CHECK(hipMemcpyAsync((char *)d + off, buf, len, hipMemcpyDeviceToDevice, hk.stream));
      else ZK_CHECK(hipMemcpyPeerAsync((char *)d + off, dev0.id, buf, hk.id, len, hk.stream));
      ZK_CHECK(hipStreamSynchronize(hk.stream));
    }); });
  }
  size_t off, len;
  spread_chunk(bytes, sp.G, 0, off, len);
  ZK_CHECK(hipMemcpyAsync((char *)d + off, (const char *)h + off, len, hipMemcpyHostToDevice, dev0.stream));
  }  // joined
  rethrow_first(err);
  ZK_CHECK(hipSetDevice(dev0.id));
}

// device-0 buffer `d` -> host (dev0's stream is idle: the passes have completed)
static void spread_out(Device &dev0, const Spread &sp, uint64_t *h, const uint64_t *d, size_t bytes) {
  std::vector<std::thread> th;
  std::string err;
  std::mutex emu;
  {
  JoinAll join_all{th};
  for (int k = 1; k < sp.G; k++) {
    th.emplace_back([&, k] { catch_into(&err, &emu, [&] {
      Device &hk = *sp.helpers[k - 1];
      size_t off, len;
      spread_chunk(bytes, sp.G, k, off, len);
      if (!len) return;
      ZK_CHECK(hipSetDevice(hk.id));
      hk.arena.reset();
      uint64_t *buf = hk.arena.take<uint64_t>(len / 8);
      if (hk.id == dev0.id) ZK_CHECK(hipMemcpyAsync(buf, (const char *)d + off, len, hipMemcpyDeviceToDevice, hk.stream));
      else ZK_CHECK(hipMemcpyPeerAsync(buf, hk.id, (const char *)d + off, dev0.id, len, hk.stream));
      ZK_CHECK(hipMemcpyAsync((char *)h + off, buf, len, hipMemcpyDeviceToHost, hk.stream));
      ZK_CHECK(hipStreamSynchronize(hk.stream));
    }); });
  }
  size_t off, len;
  spread_chunk(bytes, sp.G, 0, off, len);
  ZK_CHECK(hipMemcpyAsync((char *)h + off, (const char *)d + off, len, hipMemcpyDeviceToHost, dev0.stream));
  }  // joined
  rethrow_first(err);
  ZK_CHECK(hipSetDevice(dev0.id));
}

template <class Cfg>
static void ntt_run(Device &dev, int curve, int m, const uint64_t *gen_mont, const uint64_t *src, uint64_t *dst,
                    bool host_io, bool inverse, const Spread *sp = nullptr) {
  using F = typename Cfg::Fd;
  const size_t N = (size_t)1 << m;
  hipStream_t st = dev.stream;
  std::vector<int> dig;
  split_digits(m, dig);
  const int P = (int)dig.size();
  TwSet &tw = twiddles<Cfg>(dev, curve, m, gen_mont, inverse, dig);

  const size_t elbytes = (size_t)F::N64 * 8;
  size_t need = N * elbytes + (1 << 20);
  if (host_io) need += 2 * N * elbytes;
  if (!dev.arena.try_reserve(need)) {  // out of memory: drop the other cached twiddle sets
    {
      std::lock_guard<std::mutex> lock(g_tw_mu);
      ZK_CHECK(hipStreamSynchronize(dev.stream));
      for (auto it = g_tw.begin(); it != g_tw.end();) {
        if (std::get<0>(it->first) / 2 == dev.uid && &it->second != &tw) {
          ZK_CHECK(hipFree(it->second.mem));
          it = g_tw.erase(it);
        } else {
          ++it;
        }
      }
    }
    dev.arena.reserve(need);
  }
  dev.arena.reset();
  const uint64_t *d_src = src;
  uint64_t *d_dst = dst;
  if (host_io) {
    uint64_t *a = dev.arena.take<uint64_t>(N * F::N64);
    d_src = a;
    d_dst = dev.arena.take<uint64_t>(N * F::N64);
    if (sp) {
      for (Device *hk : sp->helpers) {  // chunk staging on every helper
        size_t off, len, mx = 0;
        for (int k = 0; k < sp->G; k++) {
          spread_chunk(N * elbytes, sp->G, k, off, len);
          mx = std::max(mx, len);
        }
        ZK_CHECK(hipSetDevice(hk->id));
        hk->arena.reserve(mx + 4096);
        hk->arena.reset();
      }
      ZK_CHECK(hipSetDevice(dev.id));
      spread_in(dev, *sp, a, src, N * elbytes);
    } else {
      ZK_CHECK(hipMemcpyAsync(a, src, N * elbytes, hipMemcpyHostToDevice, st));
    }
  }
  uint64_t *scratch = dev.arena.take<uint64_t>(N * F::N64);

  size_t S = N, T = 1;
  const uint64_t *in = d_src;
  PassArgs pa;
  pa.m = m;
  pa.P = P;
  for (int p = 0; p < P && p < 8; p++) pa.dig[p] = dig[p];
  for (int p = 0; p < P; p++) {
    const int r = dig[p];
    const int R = 1 << r;
    S >>= r;
    const int last = (p == P - 1);
    uint64_t *out = last ? d_dst : scratch;
    const bool big = r > 8;  // 2^9..2^12-point DFTs: 1024 threads over 4096-element tiles
    const int tile = big ? NTT_TILE_BIG : NTT_TILE;
    int G;
    if (P == 1) {
      G = 1;
    } else if (!last) {
      G = tile / R;
      if ((size_t)G > S) G = (int)S;
    } else {
      G = tile / R;
      if (G > (1 << dig[0])) G = 1 << dig[0];
    }
    const size_t ntiles = N / ((size_t)R * G);
    const size_t lds = (size_t)G * R * F::N * 4;
    pa.r = r;
    pa.S = (int)S;
    pa.T = (int)T;
    pa.last = last;
    pa.G = G;
    pa.h = tw.h;
    pa.otf = (!last && !tw.tab[p]) ? 1 : 0;
    const void *kfn = big ? (const void *)k_ntt_pass<F, NTT_THREADS_BIG> : (const void *)k_ntt_pass<F, NTT_THREADS>;
    ZK_CHECK(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (p == 0) timer_begin(dev);
    if (big)
      hipLaunchKernelGGL((k_ntt_pass<F, NTT_THREADS_BIG>), dim3((unsigned)ntiles), dim3(NTT_THREADS_BIG), lds, st, in,
                         out, pa, tw.inner_i[p], tw.tab[p], last ? tw.scale : nullptr, tw.tlo, tw.thi);
    else
      hipLaunchKernelGGL((k_ntt_pass<F, NTT_THREADS>), dim3((unsigned)ntiles), dim3(NTT_THREADS), lds, st, in, out,
                         pa, tw.inner_i[p], tw.tab[p], last ? tw.scale : nullptr, tw.tlo, tw.thi);
    ZK_CHECK(hipGetLastError());
    if (last) timer_end(dev);
    in = out;
    T <<= r;
  }
  if (host_io) {
    if (sp) {
      stream_wait(dev, st);
      spread_out(dev, *sp, dst, d_dst, N * elbytes);
    } else {
      copy_to_host(dev, st, dst, d_dst, N * elbytes);  // pinned pieces + 8 host threads (zk_runtime.hpp)
    }
  }
  stream_wait(dev, st);
  timer_collect(dev);
}

void ntt_release(Device &dev) {
  std::lock_guard<std::mutex> lock(g_tw_mu);
  for (auto it = g_tw.begin(); it != g_tw.end();) {
    if (std::get<0>(it->first) / 2 == dev.uid) {
      ZK_CHECK(hipFree(it->second.mem));
      it = g_tw.erase(it);
    } else {
      ++it;
    }
  }
}

void ntt(int curve, int m, const uint64_t *gen_mont, const uint64_t *src, uint64_t *dst, bool host_io,
         bool inverse) {
  ZK_REQUIRE(m >= 0 && m <= 30, "ntt: log2 size out of range (0..30)");
  std::vector<int> set = host_io && m >= 16 ? device_set() : std::vector<int>();
  int cur = 0;
  ZK_CHECK(hipGetDevice(&cur));
  if (!set.empty()) {
    // compute on the calling thread's device when the set lists it (one thread or rank per GPU
    // keeps its transforms on its own GPU), else on the first listed device
    const auto it = std::find(set.begin(), set.end(), cur);
    if (it != set.end()) std::rotate(set.begin(), it, set.end());
  }
  if (set.size() == 1 && set[0] != cur) {  // a one-entry set pins the transform to that device
    DeviceGuard on(set[0]);
    Device &dev = current_device();
    std::lock_guard<std::mutex> lock(dev.mu);
    if (curve == 0) ntt_run<CfgBN>(dev, curve, m, gen_mont, src, dst, host_io, inverse);
    else ntt_run<CfgBLS>(dev, curve, m, gen_mont, src, dst, host_io, inverse);
    return;
  }
  if (set.size() > 1) {
    // compute on the first device of the (rotated) set, host I/O spread over every listed one;
    // the contexts are locked in uid order (concurrent calls with other sets cannot deadlock)
    const int G = (int)set.size();
    std::vector<Device *> ctx(G);
    for (int k = 0; k < G; k++) {
      int slot = 0;
      for (int j = 0; j < k; j++) slot += set[j] == set[k];
      ctx[k] = &device_context(set[k], slot);
    }
    std::vector<Device *> order = ctx;
    std::sort(order.begin(), order.end(), [](Device *a, Device *b) { return a->uid < b->uid; });
    std::vector<std::unique_lock<std::mutex>> locks;
    for (Device *d : order) locks.emplace_back(d->mu);
    Spread sp;
    sp.G = G;
    sp.helpers.assign(ctx.begin() + 1, ctx.end());
    for (int k = 1; k < G; k++) {
      enable_peer(set[0], set[k]);
      enable_peer(set[k], set[0]);
    }
    DeviceGuard on(set[0]);
    if (curve == 0) ntt_run<CfgBN>(*ctx[0], curve, m, gen_mont, src, dst, host_io, inverse, &sp);
    else ntt_run<CfgBLS>(*ctx[0], curve, m, gen_mont, src, dst, host_io, inverse, &sp);
    return;
  }
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  if (curve == 0) ntt_run<CfgBN>(dev, curve, m, gen_mont, src, dst, host_io, inverse);
  else ntt_run<CfgBLS>(dev, curve, m, gen_mont, src, dst, host_io, inverse);
}

}  // namespace zk
