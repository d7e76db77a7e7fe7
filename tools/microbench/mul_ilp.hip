// mul_ilp.hip -- does a 381-bit product with two independent mad chains (even/odd
// column halves) beat the single-accumulator product when only 1-2 waves share a SIMD?
// Occupancy is pinned with dynamic LDS.  Build+run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -I../../zikkurat-algebra_amd/csrc mul_ilp.hip -o /tmp/mi && /tmp/mi
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include "zk_field.hpp"
using namespace zk;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// product scanning with two accumulators per column (terms split by parity of i)
template <class F>
__device__ __forceinline__ void fe_mul_ilp(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  constexpr int N = F::N;
  uint32_t m[N], o[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < N; k++) {
    uint64_t e = 0, f = 0;
#pragma unroll
    for (int i = 0; i < k; i++) {
      if (i & 1) { f += (uint64_t)a.v[i] * b.v[k - i]; f += (uint64_t)m[i] * F::p(k - i); }
      else { e += (uint64_t)a.v[i] * b.v[k - i]; e += (uint64_t)m[i] * F::p(k - i); }
    }
    acc += e;
    acc += f;
    acc += (uint64_t)a.v[k] * b.v[0];
    m[k] = ((uint32_t)acc * F::MINV) & F::MASK;
    acc += (uint64_t)m[k] * F::p(0);
    acc >>= F::RB;
  }
#pragma unroll
  for (int k = N; k < 2 * N - 1; k++) {
    uint64_t e = 0, f = 0;
#pragma unroll
    for (int i = k - N + 1; i < N; i++) {
      if (i & 1) { f += (uint64_t)a.v[i] * b.v[k - i]; f += (uint64_t)m[i] * F::p(k - i); }
      else { e += (uint64_t)a.v[i] * b.v[k - i]; e += (uint64_t)m[i] * F::p(k - i); }
    }
    acc += e;
    acc += f;
    o[k - N] = (uint32_t)acc & F::MASK;
    acc >>= F::RB;
  }
  o[N - 1] = (uint32_t)acc;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = o[i];
}

template <class F, int MODE, int CHAINS>
__global__ void __launch_bounds__(256) k_chain(const uint32_t *in, uint32_t *out, int iters) {
  extern __shared__ uint32_t lds[];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<F> x[CHAINS], y;
#pragma unroll
  for (int c = 0; c < CHAINS; c++)
#pragma unroll
    for (int i = 0; i < F::N; i++) x[c].v[i] = in[(t * 3 + i + 11 * c) & 1023] & F::MASK;
#pragma unroll
  for (int i = 0; i < F::N; i++) y.v[i] = in[(t * 7 + i + 3) & 1023] & F::MASK;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) x[c].v[F::N - 1] &= 0xffff;
  y.v[F::N - 1] &= 0xffff;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) {
      if (MODE == 0) fe_mul(x[c], x[c], y);
      else fe_mul_ilp(x[c], x[c], y);
    }
  }
  uint32_t z = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) z ^= x[c].v[0];
  if (z == 0x12345) lds[threadIdx.x] = z;
  out[t] = z;
}

template <class F, int MODE, int CHAINS>
static void run(const char *name, int waves_per_simd) {
  // 256-thread blocks = 4 waves = 1 per SIMD; blocks per CU = waves_per_simd (via LDS)
  const int cus = 256, blocks = cus * waves_per_simd * 8, threads = 256, iters = 32;
  const size_t lds = (160 * 1024) / waves_per_simd - 1024;
  uint32_t *in, *out;
  CK(hipMalloc(&in, 4096));
  CK(hipMalloc(&out, (size_t)blocks * threads * 4));
  std::vector<uint32_t> h(1024);
  uint32_t s = 1;
  for (auto &v : h) { s = s * 1664525u + 1013904223u; v = s; }
  CK(hipMemcpy(in, h.data(), 4096, hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void *)k_chain<F, MODE, CHAINS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((k_chain<F, MODE, CHAINS>), dim3(blocks), dim3(threads), lds, 0, in, out, iters);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  hipLaunchKernelGGL((k_chain<F, MODE, CHAINS>), dim3(blocks), dim3(threads), lds, 0, in, out, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  double prods = (double)blocks * threads * iters * CHAINS;
  printf("%-28s waves/SIMD=%d  %.1f G products/s\n", name, waves_per_simd, prods / (ms * 1e-3) / 1e9);
  CK(hipFree(in)); CK(hipFree(out));
}

int main() {
  for (int w : {1, 2, 4}) {
    run<BLS_Fp, 0, 1>("Fp381 single-acc 1 chain", w);
    run<BLS_Fp, 1, 1>("Fp381 split-acc  1 chain", w);
    run<BLS_Fp, 0, 2>("Fp381 single-acc 2 chains", w);
    run<BLS_Fp, 1, 2>("Fp381 split-acc  2 chains", w);
    run<BLS_Fr, 0, 1>("Fr255 single-acc 1 chain", w);
    run<BLS_Fr, 1, 1>("Fr255 split-acc  1 chain", w);
  }
  return 0;
}
