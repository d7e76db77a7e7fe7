// gather_calib.hip -- calibrates rocprofv3 FETCH_SIZE for k_accum's access pattern: every
// lane gathers whole 128-B rows (8 x 16-B loads) at random row indices of a table larger
// than the 256 MiB Infinity Cache, so every row read is one fabric request of known size.
//   hipcc --offload-arch=gfx950 -O3 gather_calib.hip -o gather_calib
//   rocprofv3 --pmc FETCH_SIZE -- ./gather_calib    (bytes read by k_gather / k_gather_lds: READS*128)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %d line %d\n", (int)e_, __LINE__); exit(1);} } while (0)

constexpr size_t TABLE_ROWS = (size_t)1 << 23;   // 8M rows x 128 B = 1 GiB > MALL
constexpr size_t READS = (size_t)1 << 24;        // 16M row reads = 2 GiB
constexpr int PER_LANE = 64;

__global__ void k_gather(const uint4 *__restrict__ table, const uint32_t *__restrict__ idx, uint32_t *out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int k = 0; k < PER_LANE; k++) {
    const uint32_t r = idx[t * PER_LANE + k];
    const uint4 *row = table + (size_t)r * 8;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint4 v = row[q];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  out[t] = acc;
}

// the same gathers through global_load_lds (16 B per lane per instruction into a
// lane-linear LDS image), as k_accum issues them since round 2
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
__global__ void k_gather_lds(const uint4 *__restrict__ table, const uint32_t *__restrict__ idx, uint32_t *out) {
  __shared__ uint4 st[4][8][64];
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (int k = 0; k < PER_LANE; k++) {
    const uint32_t r = idx[t * PER_LANE + k];
    const uint4 *row = table + (size_t)r * 8;
#pragma unroll
    for (int q = 0; q < 8; q++)
      __builtin_amdgcn_global_load_lds((glb_void_t *)(row + q), (lds_void_t *)&st[wave][q][0], 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint4 v = st[wave][q][lane];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  out[t] = acc;
}

int main() {
  uint4 *table;
  uint32_t *idx, *out;
  CK(hipMalloc(&table, TABLE_ROWS * 128));
  CK(hipMalloc(&idx, READS * 4));
  CK(hipMalloc(&out, READS / PER_LANE * 4));
  CK(hipMemset(table, 1, TABLE_ROWS * 128));
  uint32_t *h = (uint32_t *)malloc(READS * 4);
  uint64_t s = 88172645463325252ull;
  for (size_t i = 0; i < READS; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = (uint32_t)(s % TABLE_ROWS);
  }
  CK(hipMemcpy(idx, h, READS * 4, hipMemcpyHostToDevice));
  const unsigned blocks = (unsigned)(READS / PER_LANE / 256);
  for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k_gather, dim3(blocks), dim3(256), 0, 0, table, idx, out);
  for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k_gather_lds, dim3(blocks), dim3(256), 0, 0, table, idx, out);
  CK(hipDeviceSynchronize());
  printf("k_gather: %zu row reads x 128 B = %zu bytes of rows + %zu bytes of indices per launch\n", READS,
         READS * 128, READS * 4);
  return 0;
}
