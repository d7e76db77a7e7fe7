// zk_gen.cpp -- deterministic synthetic inputs (the benchmark's "synthetic data").
//
// Specification (re-implemented independently in oracle/zk_oracle.c and checked equal
// by tests/test_generator.py):
//   splitmix64(s):  s += 0x9E3779B97F4A7C15; z = s; z = (z^(z>>30))*0xBF58476D1CE4E5B9;
//                   z = (z^(z>>27))*0x94D049BB133111EB; return z^(z>>31)
//   stream(seed,i): state = seed ^ (0xD1B54A32D192ED03 * (i+1))
//   rand_below(F):  draw n64 words (LSW first), mask the top word to the bit length of p,
//                   retry until < p                       (uniform canonical element)
//   field element i of a vector (NTT input, MSM scalar in Montgomery form):
//                   rand_below(Fr, stream(seed, i))
//   points:         a = rand_below(Fr, stream(seed ^ 0xA0761D6478BD642F, 0)),
//                   b = rand_below(Fr, stream(seed ^ 0xE7037ED1A0B428DB, 0))  (as integers)
//                   P_i = (a + i*b) * G1   in affine Montgomery (x || y; infinity = 0xFF..)
// Points P_i = P_0 + i*H are in the order-r subgroup, like a KZG SRS.
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <thread>
#include <vector>
#include "zk_host.hpp"
#include "zk_gen.hpp"

namespace zkg {

using namespace zkh;

static inline uint64_t splitmix64(uint64_t &s) {
  s += 0x9E3779B97F4A7C15ull;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline uint64_t stream_state(uint64_t seed, uint64_t i) { return seed ^ (0xD1B54A32D192ED03ull * (i + 1)); }

template <class F>
static void rand_below(uint64_t *w, uint64_t state) {
  const int topbits = F::BITS - 64 * (F::N - 1);
  const uint64_t mask = topbits >= 64 ? ~0ull : ((1ull << topbits) - 1);
  for (;;) {
    for (int i = 0; i < F::N; i++) w[i] = splitmix64(state);
    w[F::N - 1] &= mask;
    if (!geq_p<F>(w)) return;
  }
}

template <class F>
void gen_field(uint64_t seed, int64_t start, int64_t count, uint64_t *out) {
  for (int64_t k = 0; k < count; k++) rand_below<F>(out + (size_t)k * F::N, stream_state(seed, (uint64_t)(start + k)));
}

static unsigned host_threads() {
  unsigned n = std::thread::hardware_concurrency();
  if (n == 0) n = 1;
  if (n > 16) n = 16;  // the GPU box grants ~16 host cores per GPU
  return n;
}

template <class Fp, class Fr>
void gen_points(uint64_t seed, int64_t start, int64_t count, uint64_t *out, const uint64_t *gx, const uint64_t *gy,
                const uint64_t *b3v) {
  Fe<Fp> b3;
  memcpy(b3.v, b3v, sizeof b3.v);
  Proj<Fp> G;
  memcpy(G.X.v, gx, sizeof G.X.v);
  memcpy(G.Y.v, gy, sizeof G.Y.v);
  set_one(G.Z);
  uint64_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  rand_below<Fr>(a, stream_state(seed ^ 0xA0761D6478BD642Full, 0));
  rand_below<Fr>(b, stream_state(seed ^ 0xE7037ED1A0B428DBull, 0));
  Proj<Fp> P0, H;
  proj_scale(P0, G, a, 4, b3);
  proj_scale(H, G, b, 4, b3);

  const int64_t CHUNK = 4096;
  const int64_t nchunks = (count + CHUNK - 1) / CHUNK;
  auto work = [&](int64_t c0, int64_t c1) {
    std::vector<Proj<Fp>> pts(CHUNK);
    std::vector<Fe<Fp>> pref(CHUNK);
    for (int64_t ch = c0; ch < c1; ch++) {
      const int64_t i0 = start + ch * CHUNK;
      const int64_t n = std::min<int64_t>(CHUNK, start + count - i0);
      // P_{i0} = P0 + i0*H
      uint64_t k[1] = {(uint64_t)i0};
      Proj<Fp> cur;
      proj_scale(cur, H, k, 1, b3);
      proj_add(cur, cur, P0, b3);
      for (int64_t j = 0; j < n; j++) {
        pts[j] = cur;
        proj_add(cur, cur, H, b3);
      }
      // batch inversion of Z (Montgomery's trick); zero Z = infinity is skipped
      Fe<Fp> acc;
      set_one(acc);
      for (int64_t j = 0; j < n; j++) {
        pref[j] = acc;
        if (!is_zero(pts[j].Z)) mul(acc, acc, pts[j].Z);
      }
      Fe<Fp> ia;
      inv(ia, acc);
      for (int64_t j = n - 1; j >= 0; j--) {
        uint64_t *o = out + (size_t)(i0 - start + j) * 2 * Fp::N;
        if (is_zero(pts[j].Z)) {
          memset(o, 0xff, 2 * Fp::N * 8);
          continue;
        }
        Fe<Fp> zi, x, y;
        mul(zi, ia, pref[j]);        // 1/Z_j
        mul(ia, ia, pts[j].Z);       // drop Z_j from the running inverse
        mul(x, pts[j].X, zi);
        mul(y, pts[j].Y, zi);
        memcpy(o, x.v, Fp::N * 8);
        memcpy(o + Fp::N, y.v, Fp::N * 8);
      }
    }
  };
  const unsigned nt = (unsigned)std::min<int64_t>(host_threads(), std::max<int64_t>(1, nchunks));
  if (nt <= 1) {
    work(0, nchunks);
  } else {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++) {
      int64_t c0 = nchunks * t / nt, c1 = nchunks * (t + 1) / nt;
      th.emplace_back(work, c0, c1);
    }
    for (auto &x : th) x.join();
  }
}

template void gen_field<BN_Fr>(uint64_t, int64_t, int64_t, uint64_t *);
template void gen_field<BLS_Fr>(uint64_t, int64_t, int64_t, uint64_t *);
template void gen_points<BN_Fp, BN_Fr>(uint64_t, int64_t, int64_t, uint64_t *, const uint64_t *, const uint64_t *,
                                       const uint64_t *);
template void gen_points<BLS_Fp, BLS_Fr>(uint64_t, int64_t, int64_t, uint64_t *, const uint64_t *,
                                         const uint64_t *, const uint64_t *);

}  // namespace zkg
