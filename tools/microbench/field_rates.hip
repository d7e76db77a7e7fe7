// field_rates.hip -- device microbenchmark: integer VALU rates and Montgomery
// product throughput on gfx950. Used to pick the limb representation and to set
// the VALU roofline quoted in DESIGN.md.  Build+run:
//   hipcc --offload-arch=gfx950 -O3 -I../../zikkurat-algebra_amd/csrc field_rates.hip -o /tmp/fr && /tmp/fr
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include "zk_field.hpp"

using namespace zk;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

constexpr int ITERS = 256;

// 8 independent accumulation chains of v_mad_u64_u32 per thread
__global__ void k_mad64(const uint32_t *in, uint64_t *out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = in[t & 1023], b = in[(t + 7) & 1023];
  uint64_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = k + t;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = (uint64_t)(a + k) * (b ^ i) + acc[k];
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[t] = s;
}

// 8 independent chains of 32-bit multiply-low (v_mul_lo_u32)
__global__ void k_mullo(const uint32_t *in, uint64_t *out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = in[t & 1023];
  uint32_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = k + t;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = acc[k] * (a + i) ;
  }
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[t] = s;
}

// 8 independent chains of 32-bit add (v_add_u32): the full-rate reference
__global__ void k_add32(const uint32_t *in, uint64_t *out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = in[t & 1023];
  uint32_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = k + t;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = (acc[k] ^ i) + a;
  }
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[t] = s;
}

// Montgomery product throughput: 4 independent chains per thread
template <class F>
__global__ void k_fmul(const uint64_t *in, uint64_t *out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<F> x[2], y;
  fe_load_ref(x[0], in + (size_t)((t) & 1023) * F::N64);
  fe_load_ref(x[1], in + (size_t)((t + 1) & 1023) * F::N64);
  fe_load_ref(y, in + (size_t)((t + 5) & 1023) * F::N64);
  for (int i = 0; i < ITERS / 4; i++) {
    fe_mul(x[0], x[0], y);
    fe_mul(x[1], x[1], y);
  }
  Fe<F> z;
  fe_add(z, x[0], x[1]);
  fe_store_ref(out + (size_t)t * F::N64, z);
}

// ---- prototype: unsaturated radix-2^28 Montgomery product for the 381-bit field (14 limbs)
struct P28 {
  static constexpr int N = 14;
  static constexpr uint32_t MASK = (1u << 28) - 1;
  __device__ static constexpr uint32_t p(int i) {
    constexpr uint32_t P_[14] = {0xfffaaab, 0xfffffff, 0xbfeffff, 0xb153fff, 0xffeb153, 0x241eabf, 0x0f6b0f6,
                                 0x30d2a0f, 0xf385126, 0x774b84f, 0xbacd764, 0xb7b6434, 0x69a4b1b, 0x1a0111ea};
    return P_[i];
  }
  static constexpr uint32_t MINV = 0x3fcfffd;  // placeholder constant (timing only)
};
__device__ __forceinline__ void mul28(uint32_t r[14], const uint32_t a[14], const uint32_t b[14]) {
  constexpr int N = 14;
  uint32_t m[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < N; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) { acc += (uint64_t)a[i] * b[k - i]; acc += (uint64_t)m[i] * P28::p(k - i); }
    acc += (uint64_t)a[k] * b[0];
    m[k] = ((uint32_t)acc * P28::MINV) & P28::MASK;
    acc += (uint64_t)m[k] * P28::p(0);
    acc >>= 28;
  }
#pragma unroll
  for (int k = N; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = k - N + 1; i < N; i++) { acc += (uint64_t)a[i] * b[k - i]; acc += (uint64_t)m[i] * P28::p(k - i); }
    r[k - N] = (uint32_t)acc & P28::MASK;
    acc >>= 28;
  }
  r[N - 1] = (uint32_t)acc;
  // conditional subtract
  uint32_t t[N]; int32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) { int32_t d = (int32_t)r[i] - (int32_t)P28::p(i) + br; t[i] = (uint32_t)d & P28::MASK; br = d >> 28; }
#pragma unroll
  for (int i = 0; i < N; i++) r[i] = br ? r[i] : t[i];
}
__global__ void k_mul28(const uint64_t *in, uint64_t *out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t *q = (const uint32_t *)in;
  uint32_t x0[14], x1[14], y[14];
#pragma unroll
  for (int i = 0; i < 14; i++) { x0[i] = q[(t & 511) * 14 + i] & P28::MASK; x1[i] = q[((t + 1) & 511) * 14 + i] & P28::MASK; y[i] = q[((t + 5) & 511) * 14 + i] & P28::MASK; }
  for (int i = 0; i < ITERS / 4; i++) {
    mul28(x0, x0, y);
    mul28(x1, x1, y);
  }
  uint32_t *o = (uint32_t *)out;
#pragma unroll
  for (int i = 0; i < 14; i++) o[(size_t)t * 14 + i] = x0[i] ^ x1[i];
}

template <class L>
double timeit(L launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < 5; r++) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / 5.0;
}

int main() {
  int blocks = 256 * 16, threads = 256;
  size_t nthreads = (size_t)blocks * threads;
  std::vector<uint64_t> h(1024 * 6);
  uint64_t s = 1;
  for (auto &v : h) { s = s * 6364136223846793005ull + 1442695040888963407ull; v = s >> 4; }
  void *din, *dout;
  CK(hipMalloc(&din, h.size() * 8));
  CK(hipMalloc(&dout, nthreads * 8 * 8));
  CK(hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  double ops = (double)nthreads * ITERS * 8;
  double ms;
  ms = timeit([&]{ hipLaunchKernelGGL(k_add32, dim3(blocks), dim3(threads), 0, 0, (const uint32_t*)din, (uint64_t*)dout); });
  printf("v_add_u32      : %8.2f Tops/s (%.3f ms)\n", ops / ms / 1e9, ms);
  ms = timeit([&]{ hipLaunchKernelGGL(k_mad64, dim3(blocks), dim3(threads), 0, 0, (const uint32_t*)din, (uint64_t*)dout); });
  printf("v_mad_u64_u32  : %8.2f Tops/s (%.3f ms)\n", ops / ms / 1e9, ms);
  ms = timeit([&]{ hipLaunchKernelGGL(k_mullo, dim3(blocks), dim3(threads), 0, 0, (const uint32_t*)din, (uint64_t*)dout); });
  printf("v_mul_lo_u32   : %8.2f Tops/s (%.3f ms)\n", ops / ms / 1e9, ms);
  double muls = (double)nthreads * (ITERS / 4) * 2;
  ms = timeit([&]{ hipLaunchKernelGGL(k_fmul<BLS_Fp>, dim3(blocks), dim3(threads), 0, 0, (const uint64_t*)din, (uint64_t*)dout); });
  printf("BLS Fp mont-mul: %8.2f G mul/s (%.3f ms)\n", muls / ms / 1e6, ms);
  ms = timeit([&]{ hipLaunchKernelGGL(k_fmul<BLS_Fr>, dim3(blocks), dim3(threads), 0, 0, (const uint64_t*)din, (uint64_t*)dout); });
  printf("BLS Fr mont-mul: %8.2f G mul/s (%.3f ms)\n", muls / ms / 1e6, ms);
  ms = timeit([&]{ hipLaunchKernelGGL(k_fmul<BN_Fp>, dim3(blocks), dim3(threads), 0, 0, (const uint64_t*)din, (uint64_t*)dout); });
  printf("BN  Fp mont-mul: %8.2f G mul/s (%.3f ms)\n", muls / ms / 1e6, ms);
  ms = timeit([&]{ hipLaunchKernelGGL(k_mul28, dim3(blocks), dim3(threads), 0, 0, (const uint64_t*)din, (uint64_t*)dout); });
  printf("381 radix-2^28 : %8.2f G mul/s (%.3f ms)\n", muls / ms / 1e6, ms);
  return 0;
}
