// Streaming-copy ceiling on MI355X for the Fr vector ops' access shape (verdict r05 item 6):
// 2^24 elements x 32 B (512 MiB) in, the same out.  Variants: hipMemcpyAsync D2D; a grid-stride
// uint4 copy at several grid sizes; the same with nontemporal loads / stores; 32-B elements per lane.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/stream_bw tools/microbench/stream_bw.hip && /tmp/stream_bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NT>
__global__ void k_copy16(const v4u *__restrict__ a, v4u *__restrict__ b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    v4u v;
    if (NT & 1) v = __builtin_nontemporal_load(a + i); else v = a[i];
    if (NT & 2) __builtin_nontemporal_store(v, b + i); else b[i] = v;
  }
}
// one 32-B element per lane (two v4u at stride 32 B), like fe_load_ref / fe_store_ref
template <int NT>
__global__ void k_copy32(const v4u *__restrict__ a, v4u *__restrict__ b, size_t n_el) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_el; i += (size_t)gridDim.x * blockDim.x) {
    v4u v0, v1;
    if (NT & 1) { v0 = __builtin_nontemporal_load(a + 2 * i); v1 = __builtin_nontemporal_load(a + 2 * i + 1); }
    else { v0 = a[2 * i]; v1 = a[2 * i + 1]; }
    if (NT & 2) { __builtin_nontemporal_store(v0, b + 2 * i); __builtin_nontemporal_store(v1, b + 2 * i + 1); }
    else { b[2 * i] = v0; b[2 * i + 1] = v1; }
  }
}
// two loads in flight per lane: elements i and i + stride
__global__ void k_add2(const v4u *__restrict__ a, const v4u *__restrict__ c, v4u *__restrict__ b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    v4u x = a[i], y = c[i];
    b[i] = x + y;
  }
}

int main() {
  const size_t n_el = (size_t)1 << 24, bytes = n_el * 32, n16 = bytes / 16;
  v4u *a, *b, *c;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&c, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(c, 2, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, double moved, auto fn) {
    for (int w = 0; w < 3; w++) fn();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) fn();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-44s %8.4f ms  %6.3f TB/s\n", name, ms, moved / (ms * 1e-3) / 1e12);
    return 0;
  };
  timeit("hipMemcpyAsync D2D", 2.0 * bytes, [&] { (void)hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); });
  for (unsigned g : {1024u, 2048u, 4096u, 8192u, 16384u, 65536u}) {
    char nm[96];
    snprintf(nm, sizeof nm, "copy16 grid %u x 256", g);
    timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy16<0>, dim3(g), dim3(256), 0, 0, a, b, n16); });
    snprintf(nm, sizeof nm, "copy16 nt-store grid %u", g);
    timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy16<2>, dim3(g), dim3(256), 0, 0, a, b, n16); });
    snprintf(nm, sizeof nm, "copy16 nt-load+store grid %u", g);
    timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy16<3>, dim3(g), dim3(256), 0, 0, a, b, n16); });
    snprintf(nm, sizeof nm, "copy32 (32-B element per lane) grid %u", g);
    timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy32<0>, dim3(g), dim3(256), 0, 0, a, b, n_el); });
    snprintf(nm, sizeof nm, "copy32 nt-store grid %u", g);
    timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy32<2>, dim3(g), dim3(256), 0, 0, a, b, n_el); });
    snprintf(nm, sizeof nm, "add16 (2 in, 1 out) grid %u", g);
    timeit(nm, 3.0 * bytes, [&] { hipLaunchKernelGGL(k_add2, dim3(g), dim3(256), 0, 0, a, c, b, n16); });
  }
  return 0;
}
