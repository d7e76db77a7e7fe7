// Host Montgomery arithmetic of zk_host.hpp on the GPU box's CPU: the latency of one 381-bit /
// 254-bit product, square and Jacobian doubling (the critical path of finish_host, 255 chained
// doublings per MSM), minimum over 200 repetitions, in TSC ticks and ns.
//   clang++ -O3 -std=c++17 -I<dir of zk_host.hpp> host_chain.cpp -o host_chain
#include "zk_host.hpp"
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <x86intrin.h>
using namespace zkh;
template <class F>
static void run(const char *name, double ns_per_tick) {
  Jac<F> a;
  set_one(a.X); set_one(a.Y); set_one(a.Z);
  add(a.Y, a.Y, a.Y);
  add(a.X, a.X, a.Y);
  Fe<F> x = a.X, y = a.Y;
  double bm = 1e30, bs = 1e30, bd = 1e30;
  for (int rep = 0; rep < 200; rep++) {
    const uint64_t t0 = __rdtsc();
    for (int i = 0; i < 1000; i++) mul(x, x, y);
    const uint64_t t1 = __rdtsc();
    for (int i = 0; i < 1000; i++) sqr(y, y);
    const uint64_t t2 = __rdtsc();
    for (int i = 0; i < 256; i++) jac_dbl(a, a);
    const uint64_t t3 = __rdtsc();
    bm = std::min(bm, (t1 - t0) / 1000.0);
    bs = std::min(bs, (t2 - t1) / 1000.0);
    bd = std::min(bd, (t3 - t2) / 256.0);
  }
  printf("{\"field\": \"%s\", \"mul_ns\": %.1f, \"sqr_ns\": %.1f, \"jac_dbl_ns\": %.1f, \"chain_255_dbl_us\": %.1f, \"check\": \"%016llx\"}\n",
         name, bm * ns_per_tick, bs * ns_per_tick, bd * ns_per_tick, 255 * bd * ns_per_tick / 1e3,
         (unsigned long long)(x.v[0] ^ y.v[0] ^ a.X.v[0]));
}
int main() {
  const auto c0 = std::chrono::steady_clock::now();
  const uint64_t k0 = __rdtsc();
  while (std::chrono::steady_clock::now() - c0 < std::chrono::milliseconds(100)) {}
  const double ns_per_tick =
      std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - c0).count() / (double)(__rdtsc() - k0);
  run<BLS_Fp>("bls12_381_fp", ns_per_tick);
  run<BN_Fp>("bn128_fp", ns_per_tick);
}
