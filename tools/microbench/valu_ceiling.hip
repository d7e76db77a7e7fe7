// valu_ceiling.hip -- hardware issue ceilings of the integer VALU instructions the MSM and
// NTT kernels are made of, measured independently of the library (no zk_* code here).
//
// Every kernel is a loop of inline-asm instructions (the count per iteration is exact:
// nothing for the compiler to merge or hoist) over C independent chains per lane, at high
// occupancy (<= 48 VGPRs -> 8 waves per SIMD when the grid is large enough), so neither
// dependency latency nor issue gaps of a lone wave limit the rate.  The core clock is
// measured inside the kernel (s_memtime, core clocks, against s_memrealtime, 100 MHz),
// so rates are also reported per clock and per CU.
//
//   hipcc --offload-arch=gfx950 -O3 valu_ceiling.hip -o /tmp/valu_ceiling && /tmp/valu_ceiling
//
// Output: one JSON object (instruction -> lane-ops/s, lane-ops per clock per CU, the
// clock), consumed by bench.py (profiles/*valu_ceiling*.json) as the VALU roofline peak.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int REP = 8;  // unrolled repeats of the C-chain group per loop iteration

// per-lane clock samples: [0] s_memtime start, [1] end, [2] realtime start, [3] end
__device__ __forceinline__ void stamp(uint64_t *clk, int slot) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[slot] = __builtin_amdgcn_s_memtime();
    clk[slot + 2] = __builtin_amdgcn_s_memrealtime();
  }
}

enum Op { MAD64 = 0, ADD32, MULLO, MULHI, AND32, LSHR64, ADDCO, NOPS };
static const char *op_name[NOPS] = {"v_mad_u64_u32", "v_add_u32",   "v_mul_lo_u32", "v_mul_hi_u32",
                                    "v_and_b32",     "v_lshrrev_b64", "v_add_co_u32+v_addc_co_u32"};
// lane-ops counted per asm statement
static const int op_count[NOPS] = {1, 1, 1, 1, 1, 1, 2};

template <int OP, int C>
__global__ void __launch_bounds__(256) k_ceiling(uint64_t *out, uint64_t *clk, uint32_t a, uint32_t b, int iters) {
  constexpr int CC = C < 8 ? 8 : C;  // chains are issued in groups of 8
  uint64_t acc[CC];
  uint32_t w[CC];
#pragma unroll
  for (int k = 0; k < CC; k++) {
    acc[k] = threadIdx.x + k;
    w[k] = threadIdx.x * 3 + k;
  }
  uint32_t va = a + threadIdx.x, vb = b ^ threadIdx.x;
  stamp(clk, 0);
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < REP; r++) {
      // one asm statement per group of 8 chains: the compiler's hazard padding (s_nop)
      // goes between statements only
#pragma unroll
      for (int k = 0; k < C; k += 8) {
        if constexpr (OP == MAD64 && C == 1) {  // one dependent chain (latency probe)
          uint64_t cc;
          asm volatile(
              "v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_mad_u64_u32 %0, vcc, %1, %2, %0\n\t"
              "v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_mad_u64_u32 %0, vcc, %1, %2, %0\n\t"
              "v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_mad_u64_u32 %0, vcc, %1, %2, %0\n\t"
              "v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_mad_u64_u32 %0, vcc, %1, %2, %0"
              : "+v"(acc[0])
              : "v"(va), "v"(vb)
              : "vcc");
          (void)cc;
        } else if constexpr (OP == MAD64) {
          asm volatile(
              "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_mad_u64_u32 %1, vcc, %8, %9, %1\n\t"
              "v_mad_u64_u32 %2, vcc, %8, %9, %2\n\tv_mad_u64_u32 %3, vcc, %8, %9, %3\n\t"
              "v_mad_u64_u32 %4, vcc, %8, %9, %4\n\tv_mad_u64_u32 %5, vcc, %8, %9, %5\n\t"
              "v_mad_u64_u32 %6, vcc, %8, %9, %6\n\tv_mad_u64_u32 %7, vcc, %8, %9, %7"
              : "+v"(acc[k]), "+v"(acc[k + 1]), "+v"(acc[k + 2]), "+v"(acc[k + 3]), "+v"(acc[k + 4]),
                "+v"(acc[k + 5]), "+v"(acc[k + 6]), "+v"(acc[k + 7])
              : "v"(va), "v"(vb)
              : "vcc");
        } else if constexpr (OP == LSHR64) {
          asm volatile(
              "v_lshrrev_b64 %0, 3, %0\n\tv_lshrrev_b64 %1, 3, %1\n\tv_lshrrev_b64 %2, 3, %2\n\t"
              "v_lshrrev_b64 %3, 3, %3\n\tv_lshrrev_b64 %4, 3, %4\n\tv_lshrrev_b64 %5, 3, %5\n\t"
              "v_lshrrev_b64 %6, 3, %6\n\tv_lshrrev_b64 %7, 3, %7"
              : "+v"(acc[k]), "+v"(acc[k + 1]), "+v"(acc[k + 2]), "+v"(acc[k + 3]), "+v"(acc[k + 4]),
                "+v"(acc[k + 5]), "+v"(acc[k + 6]), "+v"(acc[k + 7]));
        } else if constexpr (OP == ADDCO) {
          uint32_t lo[8], hi[8];
#pragma unroll
          for (int j = 0; j < 8; j++) { lo[j] = (uint32_t)acc[k + j]; hi[j] = (uint32_t)(acc[k + j] >> 32); }
#define ZK_ADDCO(L, H) "v_add_co_u32 %" #L ", vcc, %" #L ", %16\n\tv_addc_co_u32 %" #H ", vcc, %" #H ", %17, vcc\n\t"
          asm volatile(ZK_ADDCO(0, 1) ZK_ADDCO(2, 3) ZK_ADDCO(4, 5) ZK_ADDCO(6, 7) ZK_ADDCO(8, 9)
                           ZK_ADDCO(10, 11) ZK_ADDCO(12, 13) ZK_ADDCO(14, 15)
                       : "+v"(lo[0]), "+v"(hi[0]), "+v"(lo[1]), "+v"(hi[1]), "+v"(lo[2]), "+v"(hi[2]),
                         "+v"(lo[3]), "+v"(hi[3]), "+v"(lo[4]), "+v"(hi[4]), "+v"(lo[5]), "+v"(hi[5]),
                         "+v"(lo[6]), "+v"(hi[6]), "+v"(lo[7]), "+v"(hi[7])
                       : "v"(va), "v"(vb)
                       : "vcc");
#undef ZK_ADDCO
#pragma unroll
          for (int j = 0; j < 8; j++) acc[k + j] = ((uint64_t)hi[j] << 32) | lo[j];
        } else {
#define ZK_OP8(INS)                                                                                     \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS \
               " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"          \
               : "+v"(w[k]), "+v"(w[k + 1]), "+v"(w[k + 2]), "+v"(w[k + 3]), "+v"(w[k + 4]), "+v"(w[k + 5]), \
                 "+v"(w[k + 6]), "+v"(w[k + 7])                                                        \
               : "v"(va))
          if constexpr (OP == ADD32) ZK_OP8("v_add_u32");
          else if constexpr (OP == MULLO) ZK_OP8("v_mul_lo_u32");
          else if constexpr (OP == MULHI) ZK_OP8("v_mul_hi_u32");
          else if constexpr (OP == AND32) ZK_OP8("v_and_b32");
#undef ZK_OP8
        }
      }
    }
  }
  stamp(clk, 1);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CC; k++) s ^= acc[k] ^ w[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

struct Res {
  double ops_s, ms, mhz;
};

template <int OP, int C>
static Res run(int blocks, int iters, uint64_t *dout, uint64_t *dclk) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&] {
    hipLaunchKernelGGL((k_ceiling<OP, C>), dim3(blocks), dim3(256), 0, 0, dout, dclk, 0x12345u, 0x9abcdu, iters);
  };
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; r++) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  uint64_t clk[4];
  CK(hipMemcpy(clk, dclk, sizeof(clk), hipMemcpyDeviceToHost));
  const double core = (double)(clk[1] - clk[0]), real = (double)(clk[3] - clk[2]);
  Res r;
  r.ms = ms;
  r.ops_s = (double)blocks * 256 * iters * REP * (C < 8 ? 8 : C) * op_count[OP] / (ms * 1e-3);
  r.mhz = real > 0 ? core / real * 100.0 : 0;
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return r;
}

int main(int argc, char **argv) {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8 * 4;  // 32 waves per CU x 4 rounds
  const int iters = 512;
  uint64_t *dout, *dclk;
  CK(hipMalloc(&dout, (size_t)blocks * 256 * 8));
  CK(hipMalloc(&dclk, 64));
  Res r[NOPS];
  r[MAD64] = run<MAD64, 8>(blocks, iters, dout, dclk);
  r[ADD32] = run<ADD32, 16>(blocks, iters, dout, dclk);
  r[MULLO] = run<MULLO, 16>(blocks, iters, dout, dclk);
  r[MULHI] = run<MULHI, 16>(blocks, iters, dout, dclk);
  r[AND32] = run<AND32, 16>(blocks, iters, dout, dclk);
  r[LSHR64] = run<LSHR64, 8>(blocks, iters, dout, dclk);
  r[ADDCO] = run<ADDCO, 8>(blocks, iters, dout, dclk);
  // dependency latency probe: one chain per lane, one wave per SIMD
  Res lat = run<MAD64, 1>(cus * 1, iters, dout, dclk);
  printf("{\"device\": \"%s\", \"cus\": %d, \"waves_per_simd\": 8,", prop.gcnArchName, cus);
  printf(" \"rates\": {");
  for (int o = 0; o < NOPS; o++) {
    const double per_clk_cu = r[o].ops_s / (r[o].mhz * 1e6) / cus;
    printf("%s\"%s\": {\"lane_ops_per_s\": %.4e, \"lane_ops_per_clk_per_cu\": %.2f, \"clock_mhz\": %.0f, \"ms\": %.3f}",
           o ? ", " : "", op_name[o], r[o].ops_s, per_clk_cu, r[o].mhz, r[o].ms);
  }
  const double lat_clk = (lat.mhz * 1e6) * (lat.ms * 1e-3) / ((double)iters * REP * 8);
  printf("}, \"v_mad_u64_u32_dependent_chain_clk_per_op_1wave\": %.2f}\n", lat_clk);
  return 0;
}
