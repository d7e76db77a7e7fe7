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
// P <= 4 HBM passes (3 at 2^24).  Pass p performs, inside LDS, 2^r_p-point DFTs along
// digit p (stride S_p = R_{p+1}...R_{P-1}) for a tile of G consecutive columns (coalesced
// 256-B row segments), then multiplies output k_p by the inter-pass twiddle
// w^(T_p * k_p * lo), T_p = R_0...R_{p-1}, lo = the column index below digit p.  The last
// pass writes each output straight to its natural index k = sum_q k_q T_q (so no
// separate bit-reversal pass).  Derivation in DESIGN.md.  Twiddles: w^e for e < N
// comes from two small tables (w^(e mod 2^h), w^(2^h * (e >> h))), L2-resident.
#include "zk_field.hpp"
#include "zk_host.hpp"
#include "zk_runtime.hpp"
#include "zk_ntt.hpp"

namespace zk {

constexpr int NTT_TILE = 2048;  // elements per workgroup tile (R * G)
constexpr int NTT_THREADS = 256;

struct PassDesc {
  int r;       // log2 radix of this pass
  int S;       // stride of digit p, in elements
  int T;       // product of earlier radices
  int last;    // 1 for the final pass
};

template <class F>
__device__ __forceinline__ void twiddle(Fe<F> &w, const uint64_t *__restrict__ tlo, const uint64_t *__restrict__ thi,
                                        int h, uint32_t e) {
  // tables hold internal-form powers, stored packed (canonical, N64 u64 words)
  Fe<F> a, b;
  fe_load_ref(a, tlo + (size_t)(e & ((1u << h) - 1)) * F::N64);
  fe_load_ref(b, thi + (size_t)(e >> h) * F::N64);
  fe_mul(w, a, b);
}

// One pass.  Block = one tile of G instances x R elements.
//   non-last pass: instance (hi, lo) with lo in [0, S); element k at hi*R*S + k*S + lo
//                  tile = G consecutive lo for one hi
//   last pass    : S == 1; instance = position prefix; element k at inst*R + k;
//                  tile = G instances with consecutive digit k_0 (stride S_0/R in inst)
//                  output to natural index natbase(inst) + k * T
template <class F>
__global__ void __launch_bounds__(NTT_THREADS) k_ntt_pass(const uint64_t *__restrict__ src, uint64_t *__restrict__ dst,
                                                          int m, int r, int S, int T, int last, int G,
                                                          const int *__restrict__ digits_r, int P,
                                                          const uint64_t *__restrict__ tlo,
                                                          const uint64_t *__restrict__ thi, int h,
                                                          const uint64_t *__restrict__ scale) {
  extern __shared__ uint32_t lds[];
  constexpr int NW = F::N;  // u32 words per element
  const int R = 1 << r;
  const int halfR = R >> 1;
  uint32_t *data = lds;                          // [G][R] elements
  uint32_t *itw = lds + (size_t)G * R * NW;      // [R/2] inner twiddles w_R^j
  const int tid = threadIdx.x;
  const uint32_t N = 1u << m;

  // inner twiddles: w_R^j = w_N^(j * N/R)
  for (int j = tid; j < halfR; j += NTT_THREADS) {
    Fe<F> w;
    twiddle(w, tlo, thi, h, (uint32_t)j * (N >> r));
#pragma unroll
    for (int q = 0; q < NW; q++) itw[j * NW + q] = w.v[q];
  }

  // tile -> instance mapping
  const int tile = blockIdx.x;
  size_t in_base[1];  // silence unused warnings on some compilers
  (void)in_base;

  // load: element (g, k) -> LDS slot g*R + bitrev(k)
  const int nel = G * R;
  for (int e = tid; e < nel; e += NTT_THREADS) {
    int g, k;
    size_t addr;
    if (!last) {
      g = e % G;
      k = e / G;
      const int ntile_lo = S / G;  // S multiple of G
      const int hi = tile / ntile_lo;
      const int lo = (tile % ntile_lo) * G + g;
      addr = (size_t)hi * R * S + (size_t)k * S + lo;
    } else {
      g = e / R;
      k = e % R;
      // instance index: digits (k_0, ..., k_{P-2}); tile covers G consecutive k_0
      const int R0 = 1 << digits_r[0];
      const int ntile0 = R0 / G;
      const int k0 = (tile % ntile0) * G + g;
      const int rest = tile / ntile0;  // enumerates k_1..k_{P-2}
      // position prefix (in units of R_last): k_0 * S_0/R + sum_{1<=q<P-1} k_q * S_q/R
      size_t pos = 0;
      int rem = rest;
      size_t Sq = (size_t)N;  // S_q * R_q running
      for (int q = 0; q < P - 1; q++) {
        Sq >>= digits_r[q];
        int kq;
        if (q == 0) kq = k0;
        else { kq = rem & ((1 << digits_r[q]) - 1); rem >>= digits_r[q]; }
        pos += (size_t)kq * Sq;
      }
      addr = pos + k;
    }
    Fe<F> x;
    fe_load_ref(x, src + addr * F::N64);
    const int kr = r ? (int)(__builtin_bitreverse32((uint32_t)k) >> (32 - r)) : 0;
    uint32_t *d = data + ((size_t)g * R + kr) * NW;
#pragma unroll
    for (int q = 0; q < NW; q++) d[q] = x.v[q];
  }
  __syncthreads();

  // radix-2 DIT stages in LDS
  for (int s = 0; s < r; s++) {
    const int half = 1 << s;
    const int tstep = halfR >> s;  // w_{2half}^j = w_R^(j * R/(2 half))
    for (int bf = tid; bf < G * halfR; bf += NTT_THREADS) {
      const int g = bf / halfR;
      const int j = bf % halfR;
      const int blk = j >> s;
      const int off = j & (half - 1);
      const int i0 = g * R + blk * 2 * half + off;
      const int i1 = i0 + half;
      Fe<F> a, b, w, t;
#pragma unroll
      for (int q = 0; q < NW; q++) {
        a.v[q] = data[i0 * NW + q];
        b.v[q] = data[i1 * NW + q];
        w.v[q] = itw[(off * tstep) * NW + q];
      }
      fe_mul(t, b, w);
      Fe<F> u, v;
      fe_add(u, a, t);
      fe_sub(v, a, t);
#pragma unroll
      for (int q = 0; q < NW; q++) {
        data[i0 * NW + q] = u.v[q];
        data[i1 * NW + q] = v.v[q];
      }
    }
    __syncthreads();
  }

  // store (with inter-pass twiddle, or to natural positions on the last pass)
  Fe<F> sc;
  if (last && scale) {
    Fe<F> t;
    fe_load_ref(t, scale);
    fe_to_int(sc, t);
  }
  for (int e = tid; e < nel; e += NTT_THREADS) {
    int g = e % G, k = e / G;  // consecutive threads -> consecutive g (coalesced)
    Fe<F> x;
    const uint32_t *d = data + ((size_t)g * R + k) * NW;
#pragma unroll
    for (int q = 0; q < NW; q++) x.v[q] = d[q];
    size_t addr;
    if (!last) {
      const int ntile_lo = S / G;
      const int hi = tile / ntile_lo;
      const int lo = (tile % ntile_lo) * G + g;
      addr = (size_t)hi * R * S + (size_t)k * S + lo;
      if (lo != 0 && k != 0) {
        Fe<F> w, y;
        twiddle(w, tlo, thi, h, (uint32_t)((size_t)T * k * lo));
        fe_mul(y, x, w);
        x = y;
      }
    } else {
      const int R0 = 1 << digits_r[0];
      const int ntile0 = R0 / G;
      const int k0 = (tile % ntile0) * G + g;
      const int rest = tile / ntile0;
      // natural index: k_0 + sum_{1<=q<P-1} k_q T_q + k * T_last
      size_t nat = (size_t)k0;
      int rem = rest;
      size_t Tq = (size_t)R0;
      for (int q = 1; q < P - 1; q++) {
        int kq = rem & ((1 << digits_r[q]) - 1);
        rem >>= digits_r[q];
        nat += (size_t)kq * Tq;
        Tq <<= digits_r[q];
      }
      addr = nat + (size_t)k * T;
      if (P == 1) addr = k;
      if (scale) {
        Fe<F> y;
        fe_mul(y, x, sc);
        x = y;
      }
    }
    fe_store_ref(dst + addr * F::N64, x);
  }
}

// twiddle tables: tlo[i] = w^i (i < 2^h), thi[i] = w^(i * 2^h) (i < 2^(m-h))
template <class F>
__global__ void k_tw_tables(uint64_t *__restrict__ tlo, uint64_t *__restrict__ thi, int h, int m,
                            const uint64_t *__restrict__ pows /* w^(2^b), b < m */) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int nlo = 1 << h, nhi = 1 << (m - h);
  if (i < nlo) {
    Fe<F> acc;
    fe_one(acc);
    for (int b = 0; b < h; b++)
      if ((i >> b) & 1) {
        Fe<F> p, q, t;
        fe_load_ref(q, pows + (size_t)b * F::N64);
        fe_to_int(p, q);
        fe_mul(t, acc, p);
        acc = t;
      }
    fe_store_ref(tlo + (size_t)i * F::N64, acc);
  }
  if (i < nhi) {
    Fe<F> acc;
    fe_one(acc);
    for (int b = 0; b < m - h; b++)
      if ((i >> b) & 1) {
        Fe<F> p, q, t;
        fe_load_ref(q, pows + (size_t)(b + h) * F::N64);
        fe_to_int(p, q);
        fe_mul(t, acc, p);
        acc = t;
      }
    fe_store_ref(thi + (size_t)i * F::N64, acc);
  }
}

// ---------------------------------------------------------------------------
// host side

static void split_digits(int m, std::vector<int> &d) {
  d.clear();
  if (m == 0) { d.push_back(0); return; }
  int P = (m + 7) / 8;
  if (m <= 11) P = 1;  // one workgroup-sized DFT
  int base = m / P, extra = m % P;
  for (int p = 0; p < P; p++) d.push_back(base + (p < extra ? 1 : 0));
}

template <class Cfg>
static void ntt_run(Device &dev, int m, const uint64_t *gen_mont, const uint64_t *src, uint64_t *dst,
                    bool host_io, bool inverse) {
  using F = typename Cfg::Fd;   // device field
  using HF = typename Cfg::Fh;  // host field
  const size_t N = (size_t)1 << m;
  hipStream_t st = dev.stream;

  // host: w (forward) or w^-1 (inverse), its 2^b powers, and 1/N
  zkh::Fe<HF> g;
  memcpy(g.v, gen_mont, sizeof g.v);
  if (inverse) zkh::inv(g, g);
  std::vector<uint64_t> pows((size_t)(m > 0 ? m : 1) * HF::N);
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
    // N in standard form -> Montgomery -> inverse
    if (m < 64) nn.v[0] = (uint64_t)1 << m;
    zkh::to_mont(nn, nn);
    zkh::inv(ninv, nn);
  }

  std::vector<int> dig;
  split_digits(m, dig);
  const int P = (int)dig.size();
  const int h = m / 2;

  const size_t elbytes = (size_t)F::N64 * 8;
  size_t need = 0;
  auto acc = [&](size_t b) { need += (b + 255) & ~size_t(255); };
  if (host_io) { acc(N * elbytes); acc(N * elbytes); }
  acc(N * elbytes);                              // scratch
  acc(((size_t)1 << h) * elbytes);
  acc(((size_t)1 << (m - h)) * elbytes);
  acc(pows.size() * 8);
  acc(elbytes);
  acc(64 * sizeof(int));
  dev.arena.reserve(need + (1 << 20));
  dev.arena.reset();

  const uint64_t *d_src = src;
  uint64_t *d_dst = dst;
  if (host_io) {
    uint64_t *a = dev.arena.take<uint64_t>(N * F::N64);
    ZK_CHECK(hipMemcpyAsync(a, src, N * elbytes, hipMemcpyHostToDevice, st));
    d_src = a;
    d_dst = dev.arena.take<uint64_t>(N * F::N64);
  }
  uint64_t *scratch = dev.arena.take<uint64_t>(N * F::N64);
  uint64_t *tlo = dev.arena.take<uint64_t>(((size_t)1 << h) * F::N64);
  uint64_t *thi = dev.arena.take<uint64_t>(((size_t)1 << (m - h)) * F::N64);
  uint64_t *d_pows = dev.arena.take<uint64_t>(pows.size());
  uint64_t *d_scale = dev.arena.take<uint64_t>(F::N64);
  int *d_dig = dev.arena.take<int>(64);
  ZK_CHECK(hipMemcpyAsync(d_pows, pows.data(), pows.size() * 8, hipMemcpyHostToDevice, st));
  ZK_CHECK(hipMemcpyAsync(d_scale, ninv.v, elbytes, hipMemcpyHostToDevice, st));
  ZK_CHECK(hipMemcpyAsync(d_dig, dig.data(), dig.size() * sizeof(int), hipMemcpyHostToDevice, st));
  {
    const int nt = 1 << (h > m - h ? h : m - h);
    hipLaunchKernelGGL(k_tw_tables<F>, dim3(div_up(nt, 256)), dim3(256), 0, st, tlo, thi, h, m, d_pows);
    ZK_CHECK(hipGetLastError());
  }

  // pass chain: src -> scratch -> (in place) ... -> dst
  KernelTimer &kt = dominant_timer();
  size_t S = N;
  size_t T = 1;
  const uint64_t *in = d_src;
  for (int p = 0; p < P; p++) {
    const int r = dig[p];
    const int R = 1 << r;
    S >>= r;
    const int last = (p == P - 1);
    uint64_t *out = last ? d_dst : scratch;
    int G;
    size_t ntiles;
    if (!last) {
      G = NTT_TILE / R;
      if ((size_t)G > S) G = (int)S;
      ntiles = N / ((size_t)R * G);
    } else {
      const int R0 = 1 << dig[0];
      G = (P == 1) ? 1 : NTT_TILE / R;
      if (G > R0) G = R0;
      if (P == 1) G = 1;
      ntiles = N / ((size_t)R * G);
    }
    const size_t lds = ((size_t)G * R + R / 2) * F::N * 4;
    if (kt.enabled && p == 0) ZK_CHECK(hipEventRecord(kt.ev0, st));
    hipLaunchKernelGGL(k_ntt_pass<F>, dim3((unsigned)ntiles), dim3(NTT_THREADS), lds, st, in, out, m, r, (int)S,
                       (int)T, last, G, d_dig, P, tlo, thi, h, (last && inverse) ? d_scale : nullptr);
    ZK_CHECK(hipGetLastError());
    if (kt.enabled && last) ZK_CHECK(hipEventRecord(kt.ev1, st));
    in = out;
    T <<= r;
  }
  if (host_io) ZK_CHECK(hipMemcpyAsync(dst, d_dst, N * elbytes, hipMemcpyDeviceToHost, st));
  ZK_CHECK(hipStreamSynchronize(st));
  if (kt.enabled) {
    float ms = 0;
    ZK_CHECK(hipEventElapsedTime(&ms, kt.ev0, kt.ev1));
    kt.total_ms += ms;
    kt.launches++;
  }
}

struct CfgBN { using Fd = BN_Fr; using Fh = zkh::BN_Fr; };
struct CfgBLS { using Fd = BLS_Fr; using Fh = zkh::BLS_Fr; };

void ntt(int curve, int m, const uint64_t *gen_mont, const uint64_t *src, uint64_t *dst, bool host_io,
         bool inverse) {
  ZK_REQUIRE(m >= 0 && m <= 30, "ntt: log2 size out of range (0..30)");
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  if (curve == 0) ntt_run<CfgBN>(dev, m, gen_mont, src, dst, host_io, inverse);
  else ntt_run<CfgBLS>(dev, m, gen_mont, src, dst, host_io, inverse);
}

}  // namespace zk
