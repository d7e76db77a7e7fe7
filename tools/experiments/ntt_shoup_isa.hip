// ISA cost of a constant-multiplier (Shoup) product against the Montgomery product the NTT uses
// (verdict r05 item 4).  Compile-only experiment:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 --save-temps -c tools/experiments/ntt_shoup_isa.hip
//   python tools/isa_count.py ntt_shoup_isa-hip-amdgcn-amd-amdhsa-gfx950.s k_mont   (and k_shoup)
// Both kernels run the same loop: x <- x * w_i for a twiddle stream w_i (a butterfly's product),
// x lazily below 34p on input as in the NTT passes.
//   k_mont : fe_mul (product scanning, interleaved REDC by R' = 2^261), twiddle w R' (9 limbs)
//   k_shoup: r = x W - q p with q = floor(x W' / 2^261) from the high columns of x W' (W' =
//            floor(W 2^261 / p), precomputed per twiddle: 9 more limbs), columns 0..8 of x W and
//            of q p only (r < 4p fits 261 bits), the high half from columns 8..16 (column 8 a guard,
//            lower columns dropped: q short by at most 2).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../zikkurat-algebra_amd/csrc/zk_field.hpp"

using namespace zk;
using F = BLS_Fr;

template <class FF>
__device__ __forceinline__ void fe_mul_shoup(Fe<FF> &r, const Fe<FF> &a, const Fe<FF> &W, const Fe<FF> &Wp) {
  constexpr int N = FF::N;
  // high half of a * Wp: columns 8 .. 16, column 8 as the guard (its carry into column 9)
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i <= 8; i++) acc += (uint64_t)a.v[i] * Wp.v[8 - i];
  acc >>= FF::RB;
  uint32_t q[N];
#pragma unroll
  for (int k = N; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = k - N + 1; i < N; i++) acc += (uint64_t)a.v[i] * Wp.v[k - i];
    q[k - N] = (uint32_t)acc & FF::MASK;
    acc >>= FF::RB;
  }
  q[N - 1] = (uint32_t)acc;
  // low columns of a W - q p (signed column sums; the result < 4p < 2^261)
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < N; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) {
      c += (int64_t)((uint64_t)a.v[i] * W.v[k - i]);
      c -= (int64_t)((uint64_t)q[i] * FF::p(k - i));
    }
    r.v[k] = (k < N - 1) ? ((uint32_t)c & FF::MASK) : (uint32_t)c & ((1u << 29) - 1);
    c >>= FF::RB;
  }
}

__global__ void k_mont(const uint32_t *__restrict__ tw, uint32_t *__restrict__ out, int n) {
  Fe<F> x;
#pragma unroll
  for (int i = 0; i < F::N; i++) x.v[i] = out[threadIdx.x * 16 + i];
  for (int it = 0; it < n; it++) {
    Fe<F> w, t;
#pragma unroll
    for (int i = 0; i < F::N; i++) w.v[i] = tw[it * 16 + i];
    fe_mul(t, x, w);
    x = t;
  }
#pragma unroll
  for (int i = 0; i < F::N; i++) out[threadIdx.x * 16 + i] = x.v[i];
}

__global__ void k_shoup(const uint32_t *__restrict__ tw, uint32_t *__restrict__ out, int n) {
  Fe<F> x;
#pragma unroll
  for (int i = 0; i < F::N; i++) x.v[i] = out[threadIdx.x * 16 + i];
  for (int it = 0; it < n; it++) {
    Fe<F> w, wp, t;
#pragma unroll
    for (int i = 0; i < F::N; i++) {
      w.v[i] = tw[it * 32 + i];
      wp.v[i] = tw[it * 32 + 16 + i];
    }
    fe_mul_shoup(t, x, w, wp);
    x = t;
  }
#pragma unroll
  for (int i = 0; i < F::N; i++) out[threadIdx.x * 16 + i] = x.v[i];
}
