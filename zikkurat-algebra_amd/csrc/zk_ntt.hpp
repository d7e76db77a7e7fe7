// zk_ntt.hpp -- C++ interface of the device NTT (used by the C ABI layer)
#pragma once
#include <stddef.h>
#include <stdint.h>
namespace zk {
// curve: 0 = bn128, 1 = bls12_381.  gen_mont: generator of the order-2^m subgroup
// (Montgomery Fr, HOST pointer).  src/dst: 2^m x 4 u64 Montgomery Fr; host pointers
// when host_io, device pointers otherwise.  inverse: interpolation incl. the 1/N factor.
void ntt(int curve, int m, const uint64_t *gen_mont, const uint64_t *src, uint64_t *dst, bool host_io,
         bool inverse);
// test hook: pass split, 12 (two passes for every 2^17..2^24), 8 (<= 2^8-point passes only) or
// 0 (default: two passes at 2^20 only)
void ntt_set_max_radix(int r);
// test hook: entries above which a pass computes its inter-pass twiddles on the fly instead of
// reading a cached table (default 2^25; 0 restores it)
void ntt_set_table_max(size_t entries);
struct Device;
// frees every cached twiddle table of this context (caller holds dev.mu)
void ntt_release(Device &dev);
}  // namespace zk
