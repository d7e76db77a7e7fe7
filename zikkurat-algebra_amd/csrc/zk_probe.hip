// zk_probe.hip -- live VALU roofline probe: Montgomery product throughput of the
// device field engine (the same fe_mul the MSM / NTT kernels use), measured with HIP
// events.  bench.py divides the dominant kernel's achieved product rate by this.
#include "zk_field.hpp"
#include "zk_runtime.hpp"

namespace zk {

template <class F>
__global__ void __launch_bounds__(256) k_probe_mul(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                   int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<F> x0, x1, y;
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    x0.v[i] = in[(t * 3 + i) & 1023] & F::MASK;
    x1.v[i] = in[(t * 5 + i + 7) & 1023] & F::MASK;
    y.v[i] = in[(t * 7 + i + 3) & 1023] & F::MASK;
  }
  x0.v[F::N - 1] &= 0xffff;  // keep the values < 2p
  x1.v[F::N - 1] &= 0xffff;
  y.v[F::N - 1] &= 0xffff;
  for (int i = 0; i < iters; i++) {
    fe_mul(x0, x0, y);
    fe_mul(x1, x1, y);
  }
  Fe<F> z;
  fe_add(z, x0, x1);
  out[t] = z.v[0];
}

template <class F>
static double probe(int iters) {
  const int blocks = 256 * 16, threads = 256;
  uint32_t *in = nullptr, *out = nullptr;
  ZK_CHECK(hipMalloc(&in, 1024 * 4));
  ZK_CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
  std::vector<uint32_t> h(1024);
  uint32_t s = 12345;
  for (auto &v : h) { s = s * 1664525u + 1013904223u; v = s; }
  ZK_CHECK(hipMemcpy(in, h.data(), 4096, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  ZK_CHECK(hipEventCreate(&a));
  ZK_CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_probe_mul<F>, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
  ZK_CHECK(hipEventRecord(a, 0));
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k_probe_mul<F>, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
  ZK_CHECK(hipEventRecord(b, 0));
  ZK_CHECK(hipEventSynchronize(b));
  float ms = 0;
  ZK_CHECK(hipEventElapsedTime(&ms, a, b));
  ZK_CHECK(hipEventDestroy(a));
  ZK_CHECK(hipEventDestroy(b));
  ZK_CHECK(hipFree(in));
  ZK_CHECK(hipFree(out));
  return 3.0 * 2.0 * iters * blocks * threads / (ms * 1e-3);
}

double field_mul_rate(int field) {
  switch (field) {
    case 0: return probe<BN_Fp>(64);
    case 1: return probe<BN_Fr>(64);
    case 2: return probe<BLS_Fp>(64);
    default: return probe<BLS_Fr>(64);
  }
}

}  // namespace zk
