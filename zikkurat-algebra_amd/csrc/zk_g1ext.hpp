// zk_g1ext.hpp -- C++ interface of the G1 batch conversions and the group FFT (zk_g1ext.hip)
#pragma once
#include <stdint.h>
#include <atomic>

namespace zk {

// affine (x || y, all-0xFF = infinity) -> projective (x : y : 1), infinity -> (0 : 1 : 0);
// jac: Jacobian (x : y : 1), infinity -> (1 : 1 : 0)
void g1_batch_from_affine(int curve, int n, const uint64_t *src, uint64_t *tgt, bool host_io, bool jac = false);
// projective -> affine (X/Z, Y/Z), Z = 0 -> all-0xFF; jac: Jacobian -> (X/Z^2, Y/Z^3)
void g1_batch_to_affine(int curve, int n, const uint64_t *src, uint64_t *tgt, bool host_io, bool jac = false);
// group FFT of 2^m projective (jac: Jacobian) points with Fr generator `gen` (host, Montgomery);
// outputs normalised (x : y : 1), infinity (0 : 1 : 0), in both coordinate systems
void g1_fft(int curve, int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt, bool host_io, bool inverse,
            bool jac = false);
// GLV-stage plan of a 2^m group FFT: bits per Stockham radix-2^b stage (returns the stage count;
// 0 = the fused radix-2 stages), and the GLV products per group of a radix-2^b stage
int g1_fft_plan(int curve, int m, int *bits, int cap);
int g1_fft_radix_products(int b);
// 1 when the most recent group FFT ran the GLV stages (test / bench probe)
inline std::atomic<int> &g1_fft_last_glv() {
  static std::atomic<int> v{0};
  return v;
}

}  // namespace zk
