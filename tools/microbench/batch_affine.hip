// batch_affine.hip -- measured A/B for the bucket accumulation's formula:
// the lazy XYZZ mixed add of k_accum (xyzz_add_aff_lazy: 10 products per add) against affine
// additions with a BLOCK-COOPERATIVE Montgomery-trick inversion (one inversion per 256-lane block
// and round: each lane holds K independent pair additions).  Affine add = 3 products (lambda =
// dy / dx, lambda^2, lambda (x1 - x3)) + 3 products of the batch trick (prefix, and two in the
// backward pass) + the block's prefix / suffix product scans (16 products per lane) + 1 Fermat
// inversion of the block product by one lane.  Synthetic field elements (timing only: random
// internal-form values, no curve law needed to time the same instruction stream).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../zikkurat-algebra_amd/csrc batch_affine.hip -o /tmp/ba
//   /tmp/ba   -> one JSON line per configuration on stdout
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "zk_curve.hpp"

using namespace zk;
using F = BLS_Fp;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int TAB = 4096;  // synthetic affine points (x, y), internal form, SN words each coordinate

struct Exp6 {
  uint64_t w[6];
};

__device__ __forceinline__ void ld_aff(Aff<F> &a, const uint32_t *__restrict__ tab, uint32_t i) {
  fe_load_u(a.x, tab + (size_t)(i & (TAB - 1)) * 2 * F::SN);
  fe_load_u(a.y, tab + (size_t)(i & (TAB - 1)) * 2 * F::SN + F::SN);
}

__device__ __forceinline__ uint32_t fold(const Fe<F> &a) {
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) s ^= a.v[i];
  return s;
}

// baseline: k_accum's mixed add, K per lane (runtime trip count, like k_accum's loop)
__global__ void __launch_bounds__(256, 2) k_madd(const uint32_t *__restrict__ tab, uint32_t *__restrict__ out, int K) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Aff<F> p;
  ld_aff(p, tab, t);
  Xyzz<F> acc;
  xyzz_from_aff(acc, p);
  for (int i = 0; i < K; i++) {
    ld_aff(p, tab, t * 7 + i * 13 + 1);
    xyzz_add_aff_lazy(acc, p);
  }
  out[t] = fold(acc.X) ^ fold(acc.Y) ^ fold(acc.ZZ);
}

__device__ void fe_pow_exp(Fe<F> &r, const Fe<F> &x, const Exp6 &e) {
  Fe<F> acc, t;
  fe_one(acc);
  for (int w = 5; w >= 0; w--)
    for (int b = 63; b >= 0; b--) {
      fe_sqr(t, acc);
      acc = t;
      if ((e.w[w] >> b) & 1) {
        fe_mul(t, acc, x);
        acc = t;
      }
    }
  r = acc;
}

// block-cooperative batch-affine round: lane t adds K pairs (P_i, Q_i) in affine form
// mode 0: Fermat inversion of the block product (one lane); mode 1: the inversion replaced by a
// copy (the bound for an infinitely fast inversion)
__global__ void __launch_bounds__(256, 2) k_ba(const uint32_t *__restrict__ tab, uint32_t *__restrict__ scratch,
                                               uint32_t *__restrict__ out, int K, int mode, Exp6 pm2) {
  __shared__ uint32_t pre[256 * F::SN], suf[256 * F::SN], inv_all[F::SN];
  const int t = threadIdx.x;
  const uint32_t g = blockIdx.x * blockDim.x + t;
  uint32_t *my = scratch + (size_t)g * K * F::SN;  // this lane's prefix products
  Fe<F> one, acc, a, b;
  fe_one(one);
  acc = one;
  for (int i = 0; i < K; i++) {  // forward: prefix products of dx
    Aff<F> P, Q;
    ld_aff(P, tab, g * 7 + 2 * i + 1);
    ld_aff(Q, tab, g * 5 + 2 * i + 3);
    Fe<F> dx;
    fe_sub(dx, Q.x, P.x);
    fe_mul(a, acc, dx);
    acc = a;
    fe_store_u(my + (size_t)i * F::SN, acc);
  }
  // block-level inclusive prefix and suffix products of the lane totals (Hillis-Steele, 8 steps each)
  fe_store_u(pre + t * F::SN, acc);
  fe_store_u(suf + t * F::SN, acc);
  __syncthreads();
  Fe<F> pv = acc, sv = acc;
  for (int d = 1; d < 256; d <<= 1) {
    if (t >= d) fe_load_u(a, pre + (t - d) * F::SN);
    if (t + d < 256) fe_load_u(b, suf + (t + d) * F::SN);
    __syncthreads();
    if (t >= d) {
      Fe<F> r;
      fe_mul(r, pv, a);
      pv = r;
      fe_store_u(pre + t * F::SN, pv);
    }
    if (t + d < 256) {
      Fe<F> r;
      fe_mul(r, sv, b);
      sv = r;
      fe_store_u(suf + t * F::SN, sv);
    }
    __syncthreads();
  }
  if (t == 0) {
    Fe<F> all, inv;
    fe_load_u(all, pre + 255 * F::SN);
    if (mode == 0) fe_pow_exp(inv, all, pm2);
    else inv = all;
    fe_store_u(inv_all, inv);
  }
  __syncthreads();
  // inverse of this lane's total: inv_all * prefix(t - 1) * suffix(t + 1)
  Fe<F> il;
  fe_load_u(il, inv_all);
  if (t > 0) {
    fe_load_u(a, pre + (t - 1) * F::SN);
    fe_mul(b, il, a);
    il = b;
  }
  if (t < 255) {
    fe_load_u(a, suf + (t + 1) * F::SN);
    fe_mul(b, il, a);
    il = b;
  }
  uint32_t sum = 0;
  for (int i = K - 1; i >= 0; i--) {  // backward: inverse of each dx, then the affine addition
    Aff<F> P, Q;
    ld_aff(P, tab, g * 7 + 2 * i + 1);
    ld_aff(Q, tab, g * 5 + 2 * i + 3);
    Fe<F> dx, dy, inv, prev, lam, l2, x3, y3, s;
    fe_sub(dx, Q.x, P.x);
    fe_sub(dy, Q.y, P.y);
    if (i > 0) fe_load_u(prev, my + (size_t)(i - 1) * F::SN);
    else prev = one;
    fe_mul(inv, il, prev);  // 1 / dx_i
    fe_mul(a, il, dx);      // inverse of the prefix up to i - 1
    il = a;
    fe_mul(lam, dy, inv);
    fe_sqr(l2, lam);
    fe_sub(s, l2, P.x);
    fe_sub(x3, s, Q.x);
    fe_sub(s, P.x, x3);
    fe_mul(a, lam, s);
    fe_sub(y3, a, P.y);
    sum ^= fold(x3) ^ fold(y3);
  }
  out[g] = sum;
}

// latency of one Fermat inversion on one lane
__global__ void k_inv1(const uint32_t *__restrict__ tab, uint32_t *__restrict__ out, Exp6 pm2) {
  Aff<F> P;
  ld_aff(P, tab, 5);
  Fe<F> inv;
  fe_pow_exp(inv, P.x, pm2);
  out[0] = fold(inv);
}

int main() {
  // BLS12-381 p - 2 (little-endian u64)
  const Exp6 pm2 = {{0xb9feffffffffaaa9ull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull, 0x64774b84f38512bfull,
                     0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull}};
  std::vector<uint32_t> h((size_t)TAB * 2 * F::SN, 0);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (auto &w : h) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    w = (uint32_t)s & F::MASK;
  }
  for (int i = 0; i < TAB * 2; i++) {  // values < 2^364 < p: top limb zero, padding words zero
    h[(size_t)i * F::SN + F::N - 1] = 0;
    for (int j = F::N; j < F::SN; j++) h[(size_t)i * F::SN + j] = 0;
  }
  uint32_t *dtab, *dout, *dscr;
  const int lanes = 1 << 18;  // 1024 blocks: 2 waves per SIMD on every SIMD when the kernels fit 2
  CK(hipMalloc(&dtab, h.size() * 4));
  CK(hipMemcpy(dtab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&dout, (size_t)lanes * 4));
  CK(hipMalloc(&dscr, (size_t)lanes * 64 * F::SN * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    return best;
  };
  {
    const float ms = timed([&] { hipLaunchKernelGGL(k_inv1, dim3(1), dim3(1), 0, 0, dtab, dout, pm2); });
    printf("{\"kernel\": \"fermat_inversion_one_lane\", \"us\": %.1f}\n", ms * 1e3);
  }
  for (int K : {8, 16, 32, 64}) {
    const float m = timed([&] { hipLaunchKernelGGL(k_madd, dim3(lanes / 256), dim3(256), 0, 0, dtab, dout, K); });
    const float b0 = timed([&] { hipLaunchKernelGGL(k_ba, dim3(lanes / 256), dim3(256), 0, 0, dtab, dscr, dout, K, 0, pm2); });
    const float b1 = timed([&] { hipLaunchKernelGGL(k_ba, dim3(lanes / 256), dim3(256), 0, 0, dtab, dscr, dout, K, 1, pm2); });
    const double adds = (double)lanes * K;
    printf("{\"K\": %d, \"lanes\": %d, \"xyzz_madd_ns_per_add\": %.4f, \"batch_affine_fermat_ns_per_add\": %.4f, "
           "\"batch_affine_free_inversion_ns_per_add\": %.4f, \"madd_ms\": %.3f, \"ba_fermat_ms\": %.3f, "
           "\"ba_free_ms\": %.3f}\n",
           K, lanes, m * 1e6 / adds, b0 * 1e6 / adds, b1 * 1e6 / adds, m, b0, b1);
  }
  return 0;
}
