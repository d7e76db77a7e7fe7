// Static A/B of the 381-bit device product (CPU only, ISA counts):
//   schoolbook interleaved REDC (zk_field.hpp fe_mul) vs one signed Karatsuba level (7 + 7 limbs)
//   on the a*b part with the same interleaved REDC fed the assembled column sums.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 --save-temps -c kara_isa.hip
//   python tools/isa_count.py kara_isa-hip-amdgcn-amd-amdhsa-gfx950.s k_school ; ... k_kara
// Both kernels run a chain of 8 dependent products per loop iteration (operands normalised).
#include "../../zikkurat-algebra_amd/csrc/zk_field.hpp"
using namespace zk;
using F = BLS_Fp;

// one Karatsuba level: z0 = a_lo b_lo, z2 = a_hi b_hi, z1' = (a_lo - a_hi)(b_hi - b_lo) (signed),
// a b = z0 + (z0 + z2 + z1') 2^(7 RB) + z2 2^(14 RB); columns assembled as 64-bit sums, then the
// product-scanning REDC of fe_mul with column k of a b injected into its accumulator
__device__ __forceinline__ void fe_mul_kara(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  constexpr int N = 14, H = 7;
  int32_t da[H], db[H];
#pragma unroll
  for (int i = 0; i < H; i++) {
    da[i] = (int32_t)a.v[i] - (int32_t)a.v[i + H];
    db[i] = (int32_t)b.v[i + H] - (int32_t)b.v[i];
  }
  uint64_t z0[2 * H - 1], z2[2 * H - 1], mid[2 * H - 1];
#pragma unroll
  for (int k = 0; k < 2 * H - 1; k++) {
    uint64_t s0 = 0, s2 = 0;
#pragma unroll
    for (int i = 0; i < H; i++) {
      const int j = k - i;
      if (j < 0 || j >= H) continue;
      s0 += (uint64_t)a.v[i] * b.v[j];
      s2 += (uint64_t)a.v[i + H] * b.v[j + H];
    }
    z0[k] = s0;
    z2[k] = s2;
    int64_t s1 = (int64_t)(s0 + s2);
#pragma unroll
    for (int i = 0; i < H; i++) {
      const int j = k - i;
      if (j < 0 || j >= H) continue;
      s1 += (int64_t)da[i] * db[j];
    }
    mid[k] = (uint64_t)s1;
  }
  uint32_t m[N], o[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint64_t t = 0;
    if (k < 2 * H - 1) t += z0[k];
    if (k >= H && k - H < 2 * H - 1) t += mid[k - H];
    if (k >= 2 * H && k - 2 * H < 2 * H - 1) t += z2[k - 2 * H];
    acc += t;
    if (k < N) {
#pragma unroll
      for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * F::p(k - i);
      m[k] = ((uint32_t)acc * F::MINV) & F::MASK;
      acc += (uint64_t)m[k] * F::p(0);
      acc >>= F::RB;
    } else {
#pragma unroll
      for (int i = k - N + 1; i < N; i++) acc += (uint64_t)m[i] * F::p(k - i);
      o[k - N] = (uint32_t)acc & F::MASK;
      acc >>= F::RB;
    }
  }
  o[N - 1] = (uint32_t)acc;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = o[i];
}

template <int KARA>
__global__ void k_chain(uint32_t *buf, int iters) {
  Fe<F> a, b;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < F::N; i++) { a.v[i] = buf[t * 28 + i]; b.v[i] = buf[t * 28 + 14 + i]; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
      Fe<F> c;
      if (KARA) fe_mul_kara(c, a, b); else fe_mul(c, a, b);
      a = c;
    }
  }
#pragma unroll
  for (int i = 0; i < F::N; i++) buf[t * 28 + i] = a.v[i];
}
template __global__ void k_chain<0>(uint32_t *, int);
template __global__ void k_chain<1>(uint32_t *, int);
