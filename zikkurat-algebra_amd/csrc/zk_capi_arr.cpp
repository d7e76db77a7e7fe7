// zk_capi_arr.cpp -- extern "C" boundary of the Fr vector operations.
//
// One entry per symbol of the reference's generated headers, same signature:
//   lib/cbits/curves/array/mont/bls12_381_arr_mont.h:3-48   (bn128_arr_mont.h same lines)
//   lib/cbits/curves/poly/mont/bls12_381_poly_mont.h:22-23  (div/quot_by_vanishing)
// bound by Haskell's ZK.Algebra.Curves.<C>.Array (Array.hs:108-352) and Poly.hs.  All
// of them run on the GPU (zk_arr.hip); buffers are host memory, staged per call.
#include <string.h>
#include "../../include/zkalgebra_gpu.h"
#include "zk_arr.hpp"
#include "zk_host.hpp"
#include "zk_runtime.hpp"

using namespace zk;
#include "zk_g1ext.hpp"

// catch points of the recoverable error mode (zk_runtime.hpp guard): every entry point below
// calls the library through these, so no zk::Error crosses the C ABI
namespace {
void arr_op_g(int curve, int op, int n, const uint64_t *a, const uint64_t *b, const uint64_t *c, const uint64_t *kA,
              const uint64_t *kB, uint64_t *tgt, bool host_io) {
  guard([&] { zk::arr_op(curve, op, n, a, b, c, kA, kB, tgt, host_io); });
}
int arr_pred_g(int curve, int pred, int n, const uint64_t *a, const uint64_t *b, bool host_io) {
  return guard_ret(0, [&] { return zk::arr_pred(curve, pred, n, a, b, host_io); });
}
void arr_dot_g(int curve, int n, const uint64_t *a, const uint64_t *b, uint64_t *tgt, bool host_io) {
  guard([&] { zk::arr_dot(curve, n, a, b, tgt, host_io); });
}
void arr_powers_g(int curve, int n, const uint64_t *kA, const uint64_t *kB, uint64_t *tgt, bool host_io) {
  guard([&] { zk::arr_powers(curve, n, kA, kB, tgt, host_io); });
}
int poly_div_g(int curve, int n1, const uint64_t *src, int expo_n, const uint64_t *eta, int nquot, uint64_t *quot,
               int nrem, uint64_t *rem, bool host_io) {
  return guard_ret(0, [&] { return zk::poly_div_by_vanishing(curve, n1, src, expo_n, eta, nquot, quot, nrem, rem, host_io); });
}
void from_affine_g(int curve, int n, const uint64_t *src, uint64_t *tgt, bool host_io, bool jac = false) {
  guard([&] { zk::g1_batch_from_affine(curve, n, src, tgt, host_io, jac); });
}
void to_affine_g(int curve, int n, const uint64_t *src, uint64_t *tgt, bool host_io, bool jac = false) {
  guard([&] { zk::g1_batch_to_affine(curve, n, src, tgt, host_io, jac); });
}
void fft_g(int curve, int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt, bool host_io, bool inverse,
           bool jac = false) {
  guard([&] { zk::g1_fft(curve, m, gen, src, tgt, host_io, inverse, jac); });
}
}  // namespace

ZKG_API int zkg_g1_fft_last_glv(void) { return zk::g1_fft_last_glv().load(); }
ZKG_API int zkg_g1_fft_plan(int curve, int m, int *bits, int cap) { return zk::g1_fft_plan(curve, m, bits, cap); }
ZKG_API int zkg_g1_fft_radix_products(int b) { return zk::g1_fft_radix_products(b); }

namespace {
const uint64_t kZero[4] = {0, 0, 0, 0};
template <class Fh>
const uint64_t *mont_one() { return Fh::ONE; }
}  // namespace

extern "C" {

#define ZKG_ARR_ENTRIES(PFX, CID, FH)                                                                               \
  ZKG_API uint8_t PFX##_arr_mont_is_valid(int n, const uint64_t *s) { return (uint8_t)arr_pred_g(CID, PRED_IS_VALID, n, s, nullptr, true); } \
  ZKG_API uint8_t PFX##_arr_mont_is_zero(int n, const uint64_t *s) { return (uint8_t)arr_pred_g(CID, PRED_IS_ZERO, n, s, nullptr, true); }   \
  ZKG_API uint8_t PFX##_arr_mont_is_one(int n, const uint64_t *s) { return (uint8_t)arr_pred_g(CID, PRED_IS_ONE, n, s, nullptr, true); }     \
  ZKG_API uint8_t PFX##_arr_mont_is_equal(int n, const uint64_t *a, const uint64_t *b) {                            \
    return (uint8_t)arr_pred_g(CID, PRED_IS_EQUAL, n, a, b, true);                                                    \
  }                                                                                                                 \
  ZKG_API void PFX##_arr_mont_set_zero(int n, uint64_t *t) { arr_op_g(CID, ARR_SET_CONST, n, 0, 0, 0, kZero, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_set_one(int n, uint64_t *t) {                                                        \
    arr_op_g(CID, ARR_SET_CONST, n, 0, 0, 0, mont_one<FH>(), 0, t, true);                                            \
  }                                                                                                                 \
  ZKG_API void PFX##_arr_mont_set_const(int n, const uint64_t *s, uint64_t *t) { arr_op_g(CID, ARR_SET_CONST, n, 0, 0, 0, s, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_copy(int n, const uint64_t *s, uint64_t *t) { arr_op_g(CID, ARR_COPY, n, s, 0, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_from_std(int n, const uint64_t *s, uint64_t *t) { arr_op_g(CID, ARR_FROM_STD, n, s, 0, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_to_std(int n, const uint64_t *s, uint64_t *t) { arr_op_g(CID, ARR_TO_STD, n, s, 0, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_append(int n1, int n2, const uint64_t *s1, const uint64_t *s2, uint64_t *t) {         \
    arr_op_g(CID, ARR_COPY, n1, s1, 0, 0, 0, 0, t, true);                                                             \
    arr_op_g(CID, ARR_COPY, n2, s2, 0, 0, 0, 0, t + 4 * (size_t)(n1 > 0 ? n1 : 0), true);                             \
  }                                                                                                                 \
  ZKG_API void PFX##_arr_mont_neg(int n, const uint64_t *s, uint64_t *t) { arr_op_g(CID, ARR_NEG, n, s, 0, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_add(int n, const uint64_t *a, const uint64_t *b, uint64_t *t) { arr_op_g(CID, ARR_ADD, n, a, b, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_sub(int n, const uint64_t *a, const uint64_t *b, uint64_t *t) { arr_op_g(CID, ARR_SUB, n, a, b, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_sqr(int n, const uint64_t *s, uint64_t *t) { arr_op_g(CID, ARR_SQR, n, s, 0, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_mul(int n, const uint64_t *a, const uint64_t *b, uint64_t *t) { arr_op_g(CID, ARR_MUL, n, a, b, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_inv(int n, const uint64_t *s, uint64_t *t) { arr_op_g(CID, ARR_INV, n, s, 0, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_div(int n, const uint64_t *a, const uint64_t *b, uint64_t *t) { arr_op_g(CID, ARR_DIV, n, a, b, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_neg_inplace(int n, uint64_t *t) { arr_op_g(CID, ARR_NEG, n, t, 0, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_add_inplace(int n, uint64_t *t, const uint64_t *b) { arr_op_g(CID, ARR_ADD, n, t, b, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_sub_inplace(int n, uint64_t *t, const uint64_t *b) { arr_op_g(CID, ARR_SUB, n, t, b, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_sqr_inplace(int n, uint64_t *t) { arr_op_g(CID, ARR_SQR, n, t, 0, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_mul_inplace(int n, uint64_t *t, const uint64_t *b) { arr_op_g(CID, ARR_MUL, n, t, b, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_inv_inplace(int n, uint64_t *t) { arr_op_g(CID, ARR_INV, n, t, 0, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_div_inplace(int n, uint64_t *t, const uint64_t *b) { arr_op_g(CID, ARR_DIV, n, t, b, 0, 0, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_sub_inplace_reverse(int n, uint64_t *t, const uint64_t *s1) {                         \
    arr_op_g(CID, ARR_SUB_REV, n, t, s1, 0, 0, 0, t, true);                                                           \
  }                                                                                                                 \
  ZKG_API void PFX##_arr_mont_mul_add(int n, const uint64_t *a, const uint64_t *b, const uint64_t *c, uint64_t *t) { \
    arr_op_g(CID, ARR_MUL_ADD, n, a, b, c, 0, 0, t, true);                                                            \
  }                                                                                                                 \
  ZKG_API void PFX##_arr_mont_mul_sub(int n, const uint64_t *a, const uint64_t *b, const uint64_t *c, uint64_t *t) { \
    arr_op_g(CID, ARR_MUL_SUB, n, a, b, c, 0, 0, t, true);                                                            \
  }                                                                                                                 \
  ZKG_API void PFX##_arr_mont_dot_prod(int n, const uint64_t *a, const uint64_t *b, uint64_t *t) { arr_dot_g(CID, n, a, b, t, true); } \
  ZKG_API void PFX##_arr_mont_powers(int n, const uint64_t *kA, const uint64_t *kB, uint64_t *t) { arr_powers_g(CID, n, kA, kB, t, true); } \
  ZKG_API void PFX##_arr_mont_scale(int n, const uint64_t *k, const uint64_t *s, uint64_t *t) { arr_op_g(CID, ARR_SCALE, n, s, 0, 0, k, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_scale_inplace(int n, const uint64_t *k, uint64_t *t) { arr_op_g(CID, ARR_SCALE, n, t, 0, 0, k, 0, t, true); } \
  ZKG_API void PFX##_arr_mont_Ax_plus_y(int n, const uint64_t *kA, const uint64_t *x, const uint64_t *y, uint64_t *t) { \
    arr_op_g(CID, ARR_AXPY, n, x, y, 0, kA, 0, t, true);                                                              \
  }                                                                                                                 \
  ZKG_API void PFX##_arr_mont_Ax_plus_y_inplace(int n, const uint64_t *kA, uint64_t *t, const uint64_t *y) {        \
    arr_op_g(CID, ARR_AXPY, n, t, y, 0, kA, 0, t, true);                                                              \
  }                                                                                                                 \
  ZKG_API void PFX##_arr_mont_Ax_plus_By(int n, const uint64_t *kA, const uint64_t *kB, const uint64_t *x,          \
                                         const uint64_t *y, uint64_t *t) {                                          \
    arr_op_g(CID, ARR_AXPBY, n, x, y, 0, kA, kB, t, true);                                                            \
  }                                                                                                                 \
  ZKG_API void PFX##_arr_mont_Ax_plus_By_inplace(int n, const uint64_t *kA, const uint64_t *kB, uint64_t *t,        \
                                                 const uint64_t *y) {                                               \
    arr_op_g(CID, ARR_AXPBY, n, t, y, 0, kA, kB, t, true);                                                            \
  }                                                                                                                 \
  ZKG_API void PFX##_poly_mont_div_by_vanishing(int n1, const uint64_t *s, int expo_n, const uint64_t *eta,         \
                                                int nquot, uint64_t *quot, int nrem, uint64_t *rem) {               \
    poly_div_g(CID, n1, s, expo_n, eta, nquot, quot, rem ? nrem : 0, rem, true);                        \
  }                                                                                                                 \
  ZKG_API uint8_t PFX##_poly_mont_quot_by_vanishing(int n1, const uint64_t *s, int expo_n, const uint64_t *eta,     \
                                                    int nquot, uint64_t *quot) {                                    \
    return (uint8_t)poly_div_g(CID, n1, s, expo_n, eta, nquot, quot, 0, nullptr, true);                 \
  }

ZKG_ARR_ENTRIES(bn128, ZKG_BN128, zkh::BN_Fr)
ZKG_ARR_ENTRIES(bls12_381, ZKG_BLS12_381, zkh::BLS_Fr)

// device-resident forms (pointers already in HBM; coefficients / scalar results on the host)
ZKG_API void zkg_arr_op_device(int curve, int op, int n, const uint64_t *d_a, const uint64_t *d_b,
                               const uint64_t *d_c, const uint64_t *kA, const uint64_t *kB, uint64_t *d_tgt) {
  arr_op_g(curve, op, n, d_a, d_b, d_c, kA, kB, d_tgt, false);
}
ZKG_API void zkg_arr_dot_device(int curve, int n, const uint64_t *d_a, const uint64_t *d_b, uint64_t *tgt) {
  arr_dot_g(curve, n, d_a, d_b, tgt, false);
}
ZKG_API void zkg_arr_powers_device(int curve, int n, const uint64_t *kA, const uint64_t *kB, uint64_t *d_tgt) {
  arr_powers_g(curve, n, kA, kB, d_tgt, false);
}
ZKG_API int zkg_poly_div_by_vanishing_device(int curve, int n1, const uint64_t *d_src, int expo_n,
                                             const uint64_t *eta, int nquot, uint64_t *d_quot, int nrem,
                                             uint64_t *d_rem) {
  return poly_div_g(curve, n1, d_src, expo_n, eta, nquot, d_quot, d_rem ? nrem : 0, d_rem, false);
}

}  // extern "C"

// ---------------------------------------------------------------------------- G1
#include "zk_g1ext.hpp"

extern "C" {

#define ZKG_G1EXT_ENTRIES(PFX, CID)                                                                         \
  ZKG_API void PFX##_G1_proj_batch_from_affine(int N, const uint64_t *src, uint64_t *tgt) {                 \
    from_affine_g(CID, N, src, tgt, true);                                                           \
  }                                                                                                         \
  ZKG_API void PFX##_G1_proj_batch_to_affine(int N, const uint64_t *src, uint64_t *tgt) {                   \
    to_affine_g(CID, N, src, tgt, true);                                                             \
  }                                                                                                         \
  ZKG_API void PFX##_G1_proj_fft_forward(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {  \
    fft_g(CID, m, gen, src, tgt, true, false);                                                             \
  }                                                                                                         \
  ZKG_API void PFX##_G1_proj_fft_inverse(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {  \
    fft_g(CID, m, gen, src, tgt, true, true);                                                              \
  }                                                                                                         \
  /* Jacobian twins (bls12_381_G1_jac.c:139-158, 727-838; G1/Jac.hs:264-265, 374-389) */                   \
  ZKG_API void PFX##_G1_jac_batch_from_affine(int N, const uint64_t *src, uint64_t *tgt) {                  \
    from_affine_g(CID, N, src, tgt, true, true);                                                           \
  }                                                                                                         \
  ZKG_API void PFX##_G1_jac_batch_to_affine(int N, const uint64_t *src, uint64_t *tgt) {                    \
    to_affine_g(CID, N, src, tgt, true, true);                                                             \
  }                                                                                                         \
  ZKG_API void PFX##_G1_jac_fft_forward(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {   \
    fft_g(CID, m, gen, src, tgt, true, false, true);                                                       \
  }                                                                                                         \
  ZKG_API void PFX##_G1_jac_fft_inverse(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {   \
    fft_g(CID, m, gen, src, tgt, true, true, true);                                                        \
  }

ZKG_G1EXT_ENTRIES(bn128, ZKG_BN128)
ZKG_G1EXT_ENTRIES(bls12_381, ZKG_BLS12_381)

ZKG_API void zkg_g1_fft_device(int curve, int inverse, int m, const uint64_t *gen, const uint64_t *d_src,
                               uint64_t *d_tgt) {
  fft_g(curve, m, gen, d_src, d_tgt, false, inverse != 0);
}
ZKG_API void zkg_g1_batch_to_affine_device(int curve, int n, const uint64_t *d_src, uint64_t *d_tgt) {
  to_affine_g(curve, n, d_src, d_tgt, false);
}
ZKG_API void zkg_g1_jac_fft_device(int curve, int inverse, int m, const uint64_t *gen, const uint64_t *d_src,
                                   uint64_t *d_tgt) {
  fft_g(curve, m, gen, d_src, d_tgt, false, inverse != 0, true);
}
ZKG_API void zkg_g1_jac_batch_to_affine_device(int curve, int n, const uint64_t *d_src, uint64_t *d_tgt) {
  to_affine_g(curve, n, d_src, d_tgt, false, true);
}

}  // extern "C"
