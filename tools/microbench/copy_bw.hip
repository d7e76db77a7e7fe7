// copy_bw.hip -- host<->device copy paths for caller (pageable) buffers, 512 MiB each:
// pageable hipMemcpy, pinned hipMemcpy, host memcpy with 1..16 threads, and
// hipHostRegister (cost of the registration + DMA from the registered buffer).
//   hipcc --offload-arch=gfx950 -O3 copy_bw.hip -o copy_bw -lpthread && ./copy_bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void par_copy(void *d, const void *s, size_t n, int nt) {
  std::vector<std::thread> th;
  const size_t per = (n + nt - 1) / nt;
  for (int t = 0; t < nt; t++)
    th.emplace_back([=] {
      const size_t o = (size_t)t * per;
      if (o < n) memcpy((char *)d + o, (const char *)s + o, o + per <= n ? per : n - o);
    });
  for (auto &x : th) x.join();
}

int main() {
  const size_t N = (size_t)512 << 20;
  char *h = (char *)malloc(N), *h2 = (char *)malloc(N);
  memset(h, 1, N);
  memset(h2, 2, N);
  void *d, *p;
  CK(hipMalloc(&d, N));
  CK(hipHostMalloc(&p, N, hipHostMallocDefault));
  memset(p, 3, N);
  auto gbps = [&](double t) { return N / t / 1e9; };
  double t;
  printf("{");
  for (int rep = 0; rep < 2; rep++) {  // second round is the steady state
    t = now(); CK(hipMemcpy(d, h, N, hipMemcpyHostToDevice)); double a = gbps(now() - t);
    t = now(); CK(hipMemcpy(h2, d, N, hipMemcpyDeviceToHost)); double b = gbps(now() - t);
    t = now(); CK(hipMemcpy(d, p, N, hipMemcpyHostToDevice)); double c = gbps(now() - t);
    t = now(); CK(hipMemcpy(p, d, N, hipMemcpyDeviceToHost)); double e = gbps(now() - t);
    if (rep) printf("\"pageable_h2d_GBps\": %.1f, \"pageable_d2h_GBps\": %.1f, \"pinned_h2d_GBps\": %.1f, \"pinned_d2h_GBps\": %.1f", a, b, c, e);
  }
  for (int nt : {1, 4, 8, 16, 32}) {
    par_copy(h2, h, N, nt);
    t = now(); par_copy(h2, h, N, nt); printf(", \"memcpy_%dthreads_GBps\": %.1f", nt, gbps(now() - t));
  }
  // registration of an existing pageable buffer, then DMA straight from / to it
  t = now(); CK(hipHostRegister(h, N, hipHostRegisterDefault)); double reg = now() - t;
  t = now(); CK(hipMemcpy(d, h, N, hipMemcpyHostToDevice)); double a = gbps(now() - t);
  t = now(); CK(hipMemcpy(h, d, N, hipMemcpyDeviceToHost)); double b = gbps(now() - t);
  t = now(); CK(hipHostUnregister(h)); double unreg = now() - t;
  printf(", \"host_register_ms\": %.2f, \"registered_h2d_GBps\": %.1f, \"registered_d2h_GBps\": %.1f, \"host_unregister_ms\": %.2f}\n",
         reg * 1e3, a, b, unreg * 1e3);
  return 0;
}
