// zk_quad.hpp -- quad-cooperative XYZZ point operations for latency-bound phases (the MSM's
// Y-sum fold, the level-0 stitch and the job sums): the 4 lanes of an aligned
// quad hold the operands REPLICATED and split one point operation's products by dependency
// level, exchanging results with DPP quad broadcasts, so an operation costs its dependency
// depth in product latencies instead of its product count.
#pragma once
#include "zk_curve.hpp"

namespace zk {

// Quad-cooperative XYZZ addition (add-2008-s) for latency-bound phases: the 4 lanes of an
// aligned quad hold acc and b REPLICATED and split the 14 products by dependency level
//   L1: U1 = X1 ZZ2, U2 = X2 ZZ1, S1 = Y1 ZZZ2, S2 = Y2 ZZZ1 | ZZ1 ZZ2, ZZZ1 ZZZ2   (2 deep)
//   L2: PP = P^2, RR = R^2                                                             (1)
//   L3: PPP = P PP, Q = U1 PP, ZZ3 = (ZZ1 ZZ2) PP                                      (1)
//   L4: R (Q - X3), S1 PPP, ZZZ3 = (ZZZ1 ZZZ2) PPP                                     (1)
// with quad broadcasts in between: 5 product latencies instead of 14.  Every lane executes
// the same instruction stream (operands picked by selects, not branches); the result is
// replicated again.  Special cases are decided on replicated values, so quads never split.
template <class F>
__device__ __forceinline__ void fe_sel4(Fe<F> &r, const Fe<F> &v0, const Fe<F> &v1, const Fe<F> &v2,
                                        const Fe<F> &v3, int q) {
  // explicit masks: a ternary chain here is lowered to an indexed private array (scratch)
  const uint32_t k0 = 0u - (uint32_t)(q == 0), k1 = 0u - (uint32_t)(q == 1);
  const uint32_t k2 = 0u - (uint32_t)(q == 2), k3 = 0u - (uint32_t)(q == 3);
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = (v0.v[i] & k0) | (v1.v[i] & k1) | (v2.v[i] & k2) | (v3.v[i] & k3);
}
// quad broadcast from lane SRC of the quad: DPP quad_perm [SRC,SRC,SRC,SRC] (one VALU move
// per word, no LDS round trip)
template <int SRC, class F>
__device__ __forceinline__ void fe_bcast(Fe<F> &r, const Fe<F> &v) {
#pragma unroll
  for (int i = 0; i < F::N; i++)
    r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.v[i], SRC * 0x55, 0xf, 0xf, false);
}
template <class F>
__device__ __forceinline__ void xyzz_add_quad(Xyzz<F> &acc, const Xyzz<F> &b, uint32_t *__restrict__ park) {
  if (xyzz_is_inf(b)) return;
  if (xyzz_is_inf(acc)) { acc = b; return; }
  const int q = (int)(threadIdx.x & 3);
  if (park) xyzz_store(park, acc);  // only the rare doubling branch reads it back (nullptr: from acc)
  Fe<F> x, y, m1, m2;
  fe_sel4(x, acc.X, b.X, acc.Y, b.Y, q);
  fe_sel4(y, b.ZZ, acc.ZZ, b.ZZZ, acc.ZZZ, q);
  fe_mul(m1, x, y);  // q: U1, U2, S1, S2 (kept in the producing lane)
  fe_sel4(x, acc.ZZ, acc.ZZZ, acc.ZZ, acc.ZZZ, q);
  fe_sel4(y, b.ZZ, b.ZZZ, b.ZZ, b.ZZZ, q);
  fe_mul(m2, x, y);  // q0: ZZ1 ZZ2, q1: ZZZ1 ZZZ2
  Fe<F> P, R;
  {
    Fe<F> u, v;
    fe_bcast<0>(u, m1);
    fe_bcast<1>(v, m1);
    fe_sub(P, v, u);  // U2 - U1
    fe_bcast<2>(u, m1);
    fe_bcast<3>(v, m1);
    fe_sub(R, v, u);  // S2 - S1
  }
  Fe<F> PP, RR;
  fe_sel4(x, P, R, P, R, q);
  fe_sqr(y, x);  // q0: PP, q1: RR
  fe_bcast<0>(PP, y);
  fe_bcast<1>(RR, y);
  if (fe_is_zero(PP)) {  // P == 0 (replicated: the whole quad agrees)
    if (fe_is_zero(RR)) {
      Xyzz<F> a0, d;
      if (park) xyzz_load(a0, park);
      else a0 = acc;  // acc is still unmodified here
      xyzz_dbl(d, a0);
      acc = d;
    } else {
      xyzz_set_inf(acc);
    }
    return;
  }
  Fe<F> PPP, Q, ZZ3;
  {
    Fe<F> u1, zza;
    fe_bcast<0>(u1, m1);
    fe_bcast<0>(zza, m2);
    fe_sel4(x, P, u1, zza, P, q);
    fe_mul(y, x, PP);  // q0: PPP, q1: Q, q2: ZZ3
    fe_bcast<0>(PPP, y);
    fe_bcast<1>(Q, y);
    fe_bcast<2>(ZZ3, y);
  }
  Fe<F> X3, t;
  fe_sub(t, RR, PPP);
  fe_sub(t, t, Q);
  fe_sub(X3, t, Q);  // X3 = RR - PPP - 2Q
  fe_sub(t, Q, X3);
  {
    Fe<F> s1, zzza;
    fe_bcast<2>(s1, m1);
    fe_bcast<1>(zzza, m2);
    fe_sel4(x, R, s1, zzza, R, q);
    fe_sel4(y, t, PPP, PPP, t, q);
  }
  fe_mul(m1, x, y);  // q0: R (Q - X3), q1: S1 PPP, q2: ZZZ3
  Fe<F> a0, a1;
  fe_bcast<0>(a0, m1);
  fe_bcast<1>(a1, m1);
  fe_sub(acc.Y, a0, a1);
  fe_bcast<2>(acc.ZZZ, m1);
  acc.X = X3;
  acc.ZZ = ZZ3;
}

// lane q of the quad stores coordinate q of a replicated point
template <class F>
__device__ __forceinline__ void xyzz_store_quad(uint32_t *__restrict__ p, const Xyzz<F> &a, int q) {
  Fe<F> c;
  fe_sel4(c, a.X, a.Y, a.ZZ, a.ZZZ, q);
  fe_store_u(p + q * F::SN, c);
}

}  // namespace zk
