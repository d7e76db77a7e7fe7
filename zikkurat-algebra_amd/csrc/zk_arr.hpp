// zk_arr.hpp -- C++ interface of the device Fr vector operations (zk_arr.hip).
//
// Replaces the reference's generated per-curve vector code around the NTT:
//   <C>_arr_mont_*                      lib/cbits/curves/array/mont/bls12_381_arr_mont.h:3-48
//   <C>_poly_mont_div_by_vanishing      lib/cbits/curves/poly/mont/bls12_381_poly_mont.c:317-397
//   <C>_poly_mont_quot_by_vanishing     bls12_381_poly_mont.c:402-413
// All operands are Fr in the reference's Montgomery form (4 x u64, canonical).
#pragma once
#include <stdint.h>

namespace zk {

enum ArrOp : int {
  ARR_NEG = 0,      // tgt = -a
  ARR_ADD,          // tgt = a + b
  ARR_SUB,          // tgt = a - b
  ARR_SUB_REV,      // tgt = b - a            (sub_inplace_reverse: tgt = src1 - tgt)
  ARR_SQR,          // tgt = a^2
  ARR_MUL,          // tgt = a * b
  ARR_MUL_ADD,      // tgt = a * b + c
  ARR_MUL_SUB,      // tgt = a * b - c
  ARR_SCALE,        // tgt = kA * a
  ARR_AXPY,         // tgt = kA * a + b
  ARR_AXPBY,        // tgt = kA * a + kB * b
  ARR_FROM_STD,     // tgt = a * R  (standard -> Montgomery)
  ARR_TO_STD,       // tgt = a / R  (Montgomery -> standard)
  ARR_COPY,         // tgt = a
  ARR_SET_CONST,    // tgt = kA
  ARR_INV,          // tgt = 1/a  (batch inversion; any zero input -> every output 0)
  ARR_DIV,          // tgt = a / b (a * batch_inv(b), same zero rule on b)
  ARR_NUM_OPS
};

enum ArrPred : int { PRED_IS_VALID = 0, PRED_IS_ZERO, PRED_IS_ONE, PRED_IS_EQUAL };

// device or host pointers (host_io): a, b, c are n-element Fr arrays (unused ones may be
// null); kA, kB are single HOST elements.  tgt may alias a or b (the in-place forms).
void arr_op(int curve, int op, int n, const uint64_t *a, const uint64_t *b, const uint64_t *c, const uint64_t *kA,
            const uint64_t *kB, uint64_t *tgt, bool host_io);
int arr_pred(int curve, int pred, int n, const uint64_t *a, const uint64_t *b, bool host_io);
void arr_dot(int curve, int n, const uint64_t *a, const uint64_t *b, uint64_t *tgt_host, bool host_io);
void arr_powers(int curve, int n, const uint64_t *kA, const uint64_t *kB, uint64_t *tgt, bool host_io);
// returns 1 if the remainder is zero (quot_by_vanishing); rem may be null
int poly_div_by_vanishing(int curve, int n1, const uint64_t *src, int expo_n, const uint64_t *eta, int nquot,
                          uint64_t *quot, int nrem, uint64_t *rem, bool host_io);

}  // namespace zk
