// zk_arr.hip -- Fr vector operations and division by a vanishing polynomial on gfx950.
//
// Replaces the reference's generated vector code that sits between NTTs in a prover
// (SURVEY.md 8f row 4):
//   <C>_arr_mont_{neg,add,sub,sqr,mul,inv,div}[_inplace], _sub_inplace_reverse,
//   _mul_add, _mul_sub, _scale[_inplace], _Ax_plus_y[_inplace], _Ax_plus_By[_inplace],
//   _from_std, _to_std, _copy, _set_*, _append, _dot_prod, _powers, _is_*
//        lib/cbits/curves/array/mont/bls12_381_arr_mont.c (bn128_arr_mont.c same layout)
//   <C>_Fr_mont_batch_inv                         bls12_381_Fr_mont.c:258-285
//   <C>_poly_mont_div_by_vanishing / _quot_by_vanishing / _degree
//        lib/cbits/curves/poly/mont/bls12_381_poly_mont.c:26-32, 317-413
//
// Every result is the canonical Montgomery representative, so any exact schedule is
// bit-identical to the reference's sequential loops; the reference's corner cases are
// kept: batch inversion maps EVERY output to 0 when any input is 0 (its prefix-product
// trick degenerates that way, Fr_mont.c:266-281), inv(0) = 0.
//
// Representation: values are loaded in the reference form x*R (R = 2^256) into the
// device's unsaturated limbs (zk_field.hpp).  A product of two reference-form values
// gives x y R^2 / R'; one more product by KIN = R'^2/R (fe_to_int) returns x y R.  A
// coefficient used for a whole array is converted once (kA -> kA*R'), after which a
// single product per element yields reference form directly.
//
// Roofline: element-wise ops move 32 B per operand and per result (HBM-bound at
// 2^24 elements: a product costs ~170 mads, the VALU sustains ~1.5e11 Fr products/s,
// i.e. ~2 products per 64 B of traffic at 8 TB/s).  Batch inversion is a chunked
// Montgomery trick: CHK consecutive elements per lane, one Fermat inversion per chunk.
#include <hipcub/hipcub.hpp>
#include "zk_field.hpp"
#include "zk_host.hpp"
#include "zk_runtime.hpp"
#include "zk_arr.hpp"

namespace zk {

struct U256 {
  uint64_t w[4];
};

struct ArrArgs {
  int op, n;
  const uint64_t *a, *b, *c;
  uint64_t *tgt;
  U256 kA, kB;   // coefficients (reference form)
  U256 cstd;     // R * R' mod p: from_std constant (x -> x R in one product)
};

template <class F>
__device__ __forceinline__ void ld(Fe<F> &x, const uint64_t *p, size_t i) { fe_load_ref(x, p + i * 4); }
template <class F>
__device__ __forceinline__ void st(uint64_t *p, size_t i, const Fe<F> &x) { fe_store_ref(p + i * 4, x); }
template <class F>
__device__ __forceinline__ void ld_const(Fe<F> &x, const U256 &k) {
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    w[2 * j] = (uint32_t)k.w[j];
    w[2 * j + 1] = (uint32_t)(k.w[j] >> 32);
  }
  fe_unpack(x, w);
}
// reference-form product: (xR)(yR) -> xyR
template <class F>
__device__ __forceinline__ void mul_ref(Fe<F> &r, const Fe<F> &a, const Fe<F> &b) {
  Fe<F> t;
  fe_mul(t, a, b);
  fe_to_int(r, t);
}

template <class F>
__global__ void __launch_bounds__(256) k_arr_map(ArrArgs g) {
  Fe<F> kA, kB, cs;
  if (g.op == ARR_SCALE || g.op == ARR_AXPY || g.op == ARR_AXPBY || g.op == ARR_SET_CONST) {
    Fe<F> t;
    ld_const(t, g.kA);
    if (g.op == ARR_SET_CONST) kA = t; else fe_to_int(kA, t);
  }
  if (g.op == ARR_AXPBY) {
    Fe<F> t;
    ld_const(t, g.kB);
    fe_to_int(kB, t);
  }
  if (g.op == ARR_FROM_STD) ld_const(cs, g.cstd);
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)g.n; i += stride) {
    Fe<F> x, y, z, r;
    switch (g.op) {
      case ARR_NEG: ld(x, g.a, i); fe_neg(r, x); break;
      case ARR_ADD: ld(x, g.a, i); ld(y, g.b, i); fe_add(r, x, y); break;
      case ARR_SUB: ld(x, g.a, i); ld(y, g.b, i); fe_sub(r, x, y); break;
      case ARR_SUB_REV: ld(x, g.a, i); ld(y, g.b, i); fe_sub(r, y, x); break;
      case ARR_SQR: ld(x, g.a, i); fe_sqr(z, x); fe_to_int(r, z); break;
      case ARR_MUL: ld(x, g.a, i); ld(y, g.b, i); mul_ref(r, x, y); break;
      case ARR_MUL_ADD: ld(x, g.a, i); ld(y, g.b, i); mul_ref(z, x, y); ld(y, g.c, i); fe_add(r, z, y); break;
      case ARR_MUL_SUB: ld(x, g.a, i); ld(y, g.b, i); mul_ref(z, x, y); ld(y, g.c, i); fe_sub(r, z, y); break;
      case ARR_SCALE: ld(x, g.a, i); fe_mul(r, kA, x); break;
      case ARR_AXPY: ld(x, g.a, i); fe_mul(z, kA, x); ld(y, g.b, i); fe_add(r, z, y); break;
      case ARR_AXPBY: ld(x, g.a, i); fe_mul(z, kA, x); ld(y, g.b, i); fe_mul(x, kB, y); fe_add(r, z, x); break;
      case ARR_FROM_STD: ld(x, g.a, i); fe_mul(r, x, cs); break;
      case ARR_TO_STD: ld(x, g.a, i); fe_ref_to_std(r, x); break;
      case ARR_COPY: ld(r, g.a, i); break;
      default: r = kA; break;  // ARR_SET_CONST
    }
    st(g.tgt, i, r);
  }
}

// Round 6: the element-wise ops as one kernel PER OP (the switch above compiles every op's registers
// into every launch) with the HBM accesses of a wavefront staged through LDS: a wave's 64 elements
// (2 KiB per array) move as two 1-KiB runs of 16 B per lane -- every load and store instruction one
// contiguous kilobyte -- and each lane takes its 32-B element from the wave's LDS image.  Each wave
// owns its LDS slices and only reads what its own lanes wrote (no workgroup barrier: the wave's
// ds_write / ds_read order is kept by the LDS queue of that wave).  STAGED = 0 keeps per-lane 32-B
// accesses (A/B: ZK_ARR_STAGE=0).
// NT: nontemporal (streaming) HBM loads and stores -- every byte is touched once (measured on the
// 512 MiB copy shape, tools/microbench/stream_bw.hip: 5.76 -> 6.22 TB/s with 1024 workgroups,
// profiles/r06c_stream_bw.txt)
typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint4 *p) {
  if (NT) {
    const v4u_t v = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st16(uint4 *p, const uint4 &v) {
  if (NT) {
    v4u_t w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<v4u_t *>(p));
  } else {
    *p = v;
  }
}
template <class F, bool NT>
__device__ __forceinline__ void ld_staged(Fe<F> &x, const uint64_t *__restrict__ p, size_t e0, size_t n,
                                          uint4 *__restrict__ sl, int lane) {
  const uint4 *src = reinterpret_cast<const uint4 *>(p + e0 * 4);
  const size_t nc = (n - e0 < 64 ? n - e0 : 64) * 2;  // 16-B chunks of this wave's elements
  const uint4 z = make_uint4(0, 0, 0, 0);
  const uint4 c0 = (size_t)lane < nc ? ld16<NT>(src + lane) : z;
  const uint4 c1 = (size_t)lane + 64 < nc ? ld16<NT>(src + lane + 64) : z;
  sl[lane] = c0;
  sl[lane + 64] = c1;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint4 a = sl[2 * lane], b = sl[2 * lane + 1];
  uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  fe_unpack(x, w);
}
template <class F, bool NT>
__device__ __forceinline__ void st_staged(uint64_t *__restrict__ p, size_t e0, size_t n, const Fe<F> &x,
                                          uint4 *__restrict__ sl, int lane) {
  Fe<F> c = x;
  fe_canon(c);
  uint32_t w[8];
  fe_pack(w, c);
  sl[2 * lane] = make_uint4(w[0], w[1], w[2], w[3]);
  sl[2 * lane + 1] = make_uint4(w[4], w[5], w[6], w[7]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint4 *dst = reinterpret_cast<uint4 *>(p + e0 * 4);
  const size_t nc = (n - e0 < 64 ? n - e0 : 64) * 2;
  if ((size_t)lane < nc) st16<NT>(dst + lane, sl[lane]);
  if ((size_t)lane + 64 < nc) st16<NT>(dst + lane + 64, sl[lane + 64]);
}

// the global half of ld_staged: a wave's two 1-KiB runs of one array into registers (issued early,
// so the loads of the next elements fly while the current ones are computed: PF below)
struct Runs {
  uint4 c0, c1;
};
template <bool NT>
__device__ __forceinline__ void fetch_runs(Runs &r, const uint64_t *__restrict__ p, size_t e0, size_t n, int lane) {
  const uint4 *src = reinterpret_cast<const uint4 *>(p + e0 * 4);
  const size_t nc = (n - e0 < 64 ? n - e0 : 64) * 2;
  const uint4 z = make_uint4(0, 0, 0, 0);
  r.c0 = (size_t)lane < nc ? ld16<NT>(src + lane) : z;
  r.c1 = (size_t)lane + 64 < nc ? ld16<NT>(src + lane + 64) : z;
}
template <class F>
__device__ __forceinline__ void place_runs(Fe<F> &x, const Runs &r, uint4 *__restrict__ sl, int lane) {
  sl[lane] = r.c0;
  sl[lane + 64] = r.c1;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint4 a = sl[2 * lane], b = sl[2 * lane + 1];
  uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  fe_unpack(x, w);
}

// PF: software-pipelined -- the next grid-stride step's runs are fetched into registers before the
// current step is computed (8 VGPRs per array)
template <class F, int OP, bool STAGED, bool NT, bool PF = false>
__global__ void __launch_bounds__(256) k_arr_op(ArrArgs g) {
  Fe<F> kA, kB, cs;
  if (OP == ARR_SCALE || OP == ARR_AXPY || OP == ARR_AXPBY || OP == ARR_SET_CONST) {
    Fe<F> t;
    ld_const(t, g.kA);
    if (OP == ARR_SET_CONST) kA = t; else fe_to_int(kA, t);
  }
  if (OP == ARR_AXPBY) {
    Fe<F> t;
    ld_const(t, g.kB);
    fe_to_int(kB, t);
  }
  if (OP == ARR_FROM_STD) ld_const(cs, g.cstd);
  constexpr bool NA = OP != ARR_SET_CONST;
  constexpr bool NB = OP == ARR_ADD || OP == ARR_SUB || OP == ARR_SUB_REV || OP == ARR_MUL || OP == ARR_MUL_ADD ||
                      OP == ARR_MUL_SUB || OP == ARR_AXPY || OP == ARR_AXPBY;
  constexpr bool NC = OP == ARR_MUL_ADD || OP == ARR_MUL_SUB;
  // [wave][a, b, c][chunk]; the result reuses slice 0 (read before: a wave's DS ops run in order)
  constexpr int NS = (NA ? 1 : 0) + (NB ? 1 : 0) + (NC ? 1 : 0) > 0 ? (NA ? 1 : 0) + (NB ? 1 : 0) + (NC ? 1 : 0) : 1;
  __shared__ uint4 lds[4][STAGED ? NS : 1][128];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t n = (size_t)g.n;
  auto compute = [&](Fe<F> &r, const Fe<F> &x, const Fe<F> &y, const Fe<F> &z) {
    switch (OP) {
      case ARR_NEG: fe_neg(r, x); break;
      case ARR_ADD: fe_add(r, x, y); break;
      case ARR_SUB: fe_sub(r, x, y); break;
      case ARR_SUB_REV: fe_sub(r, y, x); break;
      case ARR_SQR: { Fe<F> t; fe_sqr(t, x); fe_to_int(r, t); } break;
      case ARR_MUL: mul_ref(r, x, y); break;
      case ARR_MUL_ADD: { Fe<F> t; mul_ref(t, x, y); fe_add(r, t, z); } break;
      case ARR_MUL_SUB: { Fe<F> t; mul_ref(t, x, y); fe_sub(r, t, z); } break;
      case ARR_SCALE: fe_mul(r, kA, x); break;
      case ARR_AXPY: { Fe<F> t; fe_mul(t, kA, x); fe_add(r, t, y); } break;
      case ARR_AXPBY: { Fe<F> t, u; fe_mul(t, kA, x); fe_mul(u, kB, y); fe_add(r, t, u); } break;
      case ARR_FROM_STD: fe_mul(r, x, cs); break;
      case ARR_TO_STD: fe_ref_to_std(r, x); break;
      case ARR_COPY: r = x; break;
      default: r = kA; break;  // ARR_SET_CONST
    }
  };
  if constexpr (STAGED && PF) {
    const size_t step = (size_t)gridDim.x * 256;
    size_t e0 = (size_t)blockIdx.x * 256 + (size_t)wave * 64;
    Runs ra, rb, rc;
    if (e0 < n) {
      if (NA) fetch_runs<NT>(ra, g.a, e0, n, lane);
      if (NB) fetch_runs<NT>(rb, g.b, e0, n, lane);
      if (NC) fetch_runs<NT>(rc, g.c, e0, n, lane);
    }
    while (e0 < n) {  // wave-uniform
      Fe<F> x, y, z, r;
      if (NA) place_runs(x, ra, lds[wave][0], lane);
      if (NB) place_runs(y, rb, lds[wave][NA ? 1 : 0], lane);
      if (NC) place_runs(z, rc, lds[wave][NS - 1], lane);
      const size_t e1 = e0 + step;
      if (e1 < n) {
        if (NA) fetch_runs<NT>(ra, g.a, e1, n, lane);
        if (NB) fetch_runs<NT>(rb, g.b, e1, n, lane);
        if (NC) fetch_runs<NT>(rc, g.c, e1, n, lane);
      }
      compute(r, x, y, z);
      st_staged<F, NT>(g.tgt, e0, n, r, lds[wave][0], lane);
      e0 = e1;
    }
    return;
  }
  for (size_t e0b = (size_t)blockIdx.x * 256; e0b < n; e0b += (size_t)gridDim.x * 256) {
    const size_t e0 = e0b + (size_t)wave * 64;
    const size_t i = e0 + lane;
    if (STAGED && e0 >= n) continue;  // the whole wave is past the end (wave-uniform)
    if (!STAGED && i >= n) continue;
    Fe<F> x, y, z, r;
    auto LD = [&](Fe<F> &v, const uint64_t *p, int k) {
      if (STAGED) ld_staged<F, NT>(v, p, e0, n, lds[wave][STAGED ? k : 0], lane);
      else ld(v, p, i);
    };
    if (NA) LD(x, g.a, 0);
    if (NB) LD(y, g.b, NA ? 1 : 0);
    if (NC) LD(z, g.c, NS - 1);
    compute(r, x, y, z);
    if (STAGED) st_staged<F, NT>(g.tgt, e0, n, r, lds[wave][0], lane);
    else if (i < n) st(g.tgt, i, r);
  }
}

// ---------------------------------------------------------------------------- inversion

// x^e (internal form), e = 256-bit exponent (sliding window, zk_field.hpp fe_pow_sw; the
// exponent is the same for every lane: no divergence)
template <class F>
__device__ __forceinline__ void fe_pow_int(Fe<F> &r, const Fe<F> &x, const U256 &e) {
  fe_pow_sw(r, x, e.w, 4);
}

// Chunked Montgomery trick: lane t owns elements [t*CHK, (t+1)*CHK).  Pass 1 stores the
// running prefix products (internal form, packed) in `scratch`; one Fermat inversion of
// the chunk product; the backward pass emits 1/x_i (ARR_INV) or a_i / x_i (ARR_DIV, with
// x = b).  Any zero x raises *zflag (the final kernel then zeroes everything).
// Round 6: lane t's chunk is the strided set {t, t + T, t + 2T, ...} (T = lanes) instead of the
// CHK consecutive elements from t CHK: a wavefront's loads and stores then touch 64 consecutive
// elements (2 KiB) per instruction, where the consecutive chunks put 64 lanes 4 KiB apart (one
// cache line per lane per access).  The product trick works on any partition.  STRIDED = false
// keeps the round-5 chunks (ZK_INV_STRIDE=0, A/B).
template <class F, bool SG = true, bool STRIDED = true>
__global__ void __launch_bounds__(256) k_inv_chunks(int op, int n, int CHK, const uint64_t *__restrict__ a,
                                                    const uint64_t *__restrict__ x, uint64_t *__restrict__ scratch,
                                                    uint64_t *tgt, U256 pm2, uint32_t *zflag, int lanes) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t T = STRIDED ? (size_t)lanes : 1;
  const size_t i0 = STRIDED ? t : t * CHK;
  if ((STRIDED && t >= T) || i0 >= (size_t)n) return;
  // the chunk: i0, i0 + T, ..., cnt elements
  const size_t left = ((size_t)n - i0 + T - 1) / T;
  const size_t cnt = left < (size_t)CHK ? left : (size_t)CHK;
  Fe<F> P;
  fe_one(P);
  bool zero = false;
  for (size_t k = 0; k < cnt; k++) {
    const size_t i = i0 + k * T;
    Fe<F> v, vi, q;
    ld(v, x, i);
    zero |= fe_is_zero(v);
    fe_to_int(vi, v);
    fe_mul(q, P, vi);
    P = q;
    st(scratch, i, P);
  }
  if (zero) atomicOr(zflag, 1u);
  Fe<F> inv;
  if (SG) fe_inv_sg(inv, P);  // (prod)^-1, internal form: divsteps (zk_inv.hpp), Fermat with ZK_INV_SG=0
  else fe_pow_int(inv, P, pm2);
  for (size_t k = cnt; k-- > 0;) {
    const size_t i = i0 + k * T;
    Fe<F> prev, out, v, vi, q;
    if (k > 0) ld(prev, scratch, i - T); else fe_one(prev);
    fe_mul(out, inv, prev);  // 1/x_i (internal)
    ld(v, x, i);
    fe_to_int(vi, v);
    fe_mul(q, inv, vi);
    inv = q;
    if (op == ARR_DIV) {
      Fe<F> ai, r;
      ld(ai, a, i);
      fe_mul(r, out, ai);  // (1/x) R' * a R / R' = (a/x) R
      st(tgt, i, r);
    } else {
      Fe<F> r;
      fe_to_ref(r, out);
      st(tgt, i, r);
    }
  }
}

// The strided chunks with TWO interleaved chains per lane (round 6, ZK_INV_ILP=0 restores the one-
// chain kernel): elements k = 0, 2, 4, ... and k = 1, 3, 5, ... of a lane's chunk keep separate running
// products, so every step issues two independent products where the one-chain kernel waits for the
// previous product's last column; the two totals share ONE inversion (P0 P1)^-1, split as
// P0^-1 = (P0 P1)^-1 P1 and P1^-1 = (P0 P1)^-1 P0 (two products per lane).  A lane with an odd count
// pads chain 1 with a 1 (its product runs, its load and store do not).  Scratch holds each element's
// running product within its own chain.
template <class F>
__device__ __forceinline__ void fe_sel(Fe<F> &r, bool c, const Fe<F> &a, const Fe<F> &b) {
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = c ? a.v[i] : b.v[i];
}
// Straight-line steps: every load and store of a step is unconditional (a lane past its count
// re-reads / re-writes its element k0 with the same value), so no branch splits the step and the
// compiler's wait counts let the step's loads fly together (a conditional load or store makes it
// wait for everything outstanding where the paths merge).
template <class F>
__global__ void __launch_bounds__(256) k_inv_chunks2(int op, int n, int CHK, const uint64_t *__restrict__ a,
                                                     const uint64_t *__restrict__ x, uint64_t *__restrict__ scratch,
                                                     uint64_t *tgt, uint32_t *zflag, int lanes) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t T = (size_t)lanes;
  if (t >= T || t >= (size_t)n) return;
  const size_t left = ((size_t)n - t + T - 1) / T;
  const size_t cnt = left < (size_t)CHK ? left : (size_t)CHK;
  const size_t pairs = (cnt + 1) / 2;
  const bool div = op == ARR_DIV;
  Fe<F> P0, P1, one;
  fe_one(one);
  P0 = one;
  P1 = one;
  bool zero = false;
  for (size_t j = 0; j < pairs; j++) {
    const size_t k0 = 2 * j, i0 = t + k0 * T;
    const bool has1 = k0 + 1 < cnt;
    const size_t i1 = has1 ? i0 + T : i0;
    Fe<F> v0, v1, w0, w1, u1, q0, q1;
    ld(v0, x, i0);
    ld(v1, x, i1);
    zero |= fe_is_zero(v0);
    zero |= fe_is_zero(v1);
    fe_to_int(w0, v0);
    fe_to_int(u1, v1);
    fe_sel(w1, has1, u1, one);
    fe_mul(q0, P0, w0);
    fe_mul(q1, P1, w1);
    P0 = q0;
    P1 = q1;
    Fe<F> s1;
    fe_sel(s1, has1, P1, P0);
    st(scratch, i0, P0);
    st(scratch, i1, s1);
  }
  if (zero) atomicOr(zflag, 1u);
  Fe<F> P, inv, inv0, inv1;
  fe_mul(P, P0, P1);
  fe_inv_sg(inv, P);
  fe_mul(inv0, inv, P1);
  fe_mul(inv1, inv, P0);
  for (size_t j = pairs; j-- > 0;) {
    const size_t k0 = 2 * j, i0 = t + k0 * T;
    const bool has1 = k0 + 1 < cnt;
    const size_t i1 = has1 ? i0 + T : i0;
    // the chains' previous elements k0 - 2 and k0 - 1 (any valid index when j = 0: unused)
    const size_t ip0 = j > 0 ? i0 - 2 * T : i0, ip1 = j > 0 ? i0 - T : i0;
    Fe<F> p0, p1, o0, o1, v0, v1, w0, w1, u1, q0, q1, a0, a1, r0, r1, e0, e1;
    ld(e0, scratch, ip0);
    ld(e1, scratch, ip1);
    ld(v0, x, i0);
    ld(v1, x, i1);
    ld(a0, a, div ? i0 : 0);  // a is the dividend (ARR_DIV) or unused: then element 0 of x's buffer
    ld(a1, a, div ? i1 : 0);
    fe_sel(p0, j > 0, e0, one);
    fe_sel(p1, j > 0, e1, one);
    fe_to_int(w0, v0);
    fe_to_int(u1, v1);
    fe_sel(w1, has1, u1, one);
    fe_mul(o0, inv0, p0);  // 1/x_(k0) (internal)
    fe_mul(o1, inv1, p1);  // 1/x_(k0 + 1)
    fe_mul(q0, inv0, w0);
    fe_mul(q1, inv1, w1);
    inv0 = q0;
    inv1 = q1;
    if (div) {
      fe_mul(r0, o0, a0);  // (1/x) R' * a R / R' = (a/x) R
      fe_mul(r1, o1, a1);
    } else {
      fe_to_ref(r0, o0);
      fe_to_ref(r1, o1);
    }
    Fe<F> s1;
    fe_sel(s1, has1, r1, r0);
    st(tgt, i0, r0);
    st(tgt, i1, s1);
  }
}

__global__ void k_zero_if_flag(int n, uint64_t *__restrict__ tgt, const uint32_t *__restrict__ zflag) {
  if (*zflag == 0) return;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)n * 4; i += stride) tgt[i] = 0;
}

// ---------------------------------------------------------------------------- predicates

__global__ void k_pred(int pred, int n, const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, U256 prime,
                       U256 one, uint32_t *__restrict__ fail) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  bool bad = false;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)n; i += stride) {
    const uint64_t *x = a + i * 4;
    switch (pred) {
      case PRED_IS_VALID: {  // x < p, Fr_mont.c:288-298
        bool lt = false, decided = false;
        for (int j = 3; j >= 0 && !decided; j--) {
          if (x[j] != prime.w[j]) { lt = x[j] < prime.w[j]; decided = true; }
        }
        bad |= !lt;
        break;
      }
      case PRED_IS_ZERO: bad |= (x[0] | x[1] | x[2] | x[3]) != 0; break;
      case PRED_IS_ONE:
        bad |= (x[0] != one.w[0]) | (x[1] != one.w[1]) | (x[2] != one.w[2]) | (x[3] != one.w[3]);
        break;
      default: {
        const uint64_t *y = b + i * 4;
        bad |= (x[0] != y[0]) | (x[1] != y[1]) | (x[2] != y[2]) | (x[3] != y[3]);
      }
    }
  }
  if (bad) atomicOr(fail, 1u);
}

// ---------------------------------------------------------------------------- dot product

constexpr int DOT_THREADS = 256;
template <class F>
__global__ void __launch_bounds__(DOT_THREADS) k_dot(int n, const uint64_t *__restrict__ a,
                                                     const uint64_t *__restrict__ b, uint64_t *__restrict__ part) {
  __shared__ uint32_t lds[DOT_THREADS * F::N];
  Fe<F> acc;
  fe_zero(acc);
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)n; i += stride) {
    Fe<F> x, y, z, s;
    ld(x, a, i);
    ld(y, b, i);
    fe_mul(z, x, y);  // x y R^2 / R' (converted once, after the sum)
    fe_add(s, acc, z);
    acc = s;
  }
  for (int q = 0; q < F::N; q++) lds[threadIdx.x * F::N + q] = acc.v[q];
  __syncthreads();
  for (int s = DOT_THREADS / 2; s >= 1; s >>= 1) {
    if ((int)threadIdx.x < s) {
      Fe<F> o, r;
      for (int q = 0; q < F::N; q++) o.v[q] = lds[(threadIdx.x + s) * F::N + q];
      fe_add(r, acc, o);
      acc = r;
      for (int q = 0; q < F::N; q++) lds[threadIdx.x * F::N + q] = acc.v[q];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) st(part, blockIdx.x, acc);  // canonical, still in the R^2/R' form
}
// the block partials' sum: one 256-thread block, each thread adding every 256th partial, then the
// same LDS tree as k_dot (round 5 summed the 1024 partials on ONE thread: 0.34 ms of a 0.55 ms
// 2^24 dot product, profiles/r06c_prof)
template <class F>
__global__ void __launch_bounds__(DOT_THREADS) k_dot_final(int nparts, const uint64_t *__restrict__ part,
                                                           uint64_t *__restrict__ out) {
  __shared__ uint32_t lds[DOT_THREADS * F::N];
  Fe<F> acc;
  fe_zero(acc);
  for (int i = threadIdx.x; i < nparts; i += DOT_THREADS) {
    Fe<F> x, s;
    ld(x, part, i);
    fe_add(s, acc, x);
    acc = s;
  }
  for (int q = 0; q < F::N; q++) lds[threadIdx.x * F::N + q] = acc.v[q];
  __syncthreads();
  for (int s = DOT_THREADS / 2; s >= 1; s >>= 1) {
    if ((int)threadIdx.x < s) {
      Fe<F> o, r;
      for (int q = 0; q < F::N; q++) o.v[q] = lds[(threadIdx.x + s) * F::N + q];
      fe_add(r, acc, o);
      acc = r;
      for (int q = 0; q < F::N; q++) lds[threadIdx.x * F::N + q] = acc.v[q];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    Fe<F> r;
    fe_to_int(r, acc);  // x y R^2/R' * R'/R = x y R (the product by 32 on the 9 x 29-bit fields)
    st(out, 0, r);
  }
}

// ---------------------------------------------------------------------------- powers

// tlo[i] = B^i (internal, i < 2^h);  thi[j] = A * B^(j 2^h) (reference form)
template <class F>
__global__ void k_pow_tables(int h, int nlo, int nhi, U256 kA, U256 kB, uint64_t *__restrict__ tlo,
                             uint64_t *__restrict__ thi) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<F> Bref, B;
  ld_const(Bref, kB);
  fe_to_int(B, Bref);
  if (i < nlo) {
    Fe<F> acc, base = B, t;
    fe_one(acc);
    for (int e = i; e; e >>= 1) {
      if (e & 1) { fe_mul(t, acc, base); acc = t; }
      fe_sqr(t, base);
      base = t;
    }
    st(tlo, i, acc);
  }
  if (i < nhi) {
    Fe<F> base = B, t, acc;
    for (int s = 0; s < h; s++) { fe_sqr(t, base); base = t; }  // B^(2^h)
    ld_const(acc, kA);  // reference form A R
    for (int e = i; e; e >>= 1) {
      if (e & 1) { fe_mul(t, acc, base); acc = t; }
      fe_sqr(t, base);
      base = t;
    }
    st(thi, i, acc);
  }
}
template <class F>
__global__ void __launch_bounds__(256) k_powers(int n, int h, const uint64_t *__restrict__ tlo,
                                                const uint64_t *__restrict__ thi, uint64_t *__restrict__ tgt) {
  // round 6: the output leaves through the wave's LDS image as 1-KiB nontemporal runs (k_arr_op);
  // the two tables are small and L2-resident
  __shared__ uint4 lds[4][128];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t N = (size_t)n;
  for (size_t e0b = (size_t)blockIdx.x * 256; e0b < N; e0b += (size_t)gridDim.x * 256) {
    const size_t e0 = e0b + (size_t)wave * 64, i = e0 + lane;
    if (e0 >= N) continue;  // wave-uniform
    Fe<F> lo, hi, r;
    const size_t ii = i < N ? i : N - 1;
    ld(lo, tlo, ii & ((1u << h) - 1));
    ld(hi, thi, ii >> h);
    fe_mul(r, hi, lo);  // A B^(j 2^h) R * B^l R' / R'
    st_staged<F, true>(tgt, e0, N, r, lds[wave], lane);
  }
}

// ---------------------------------------------------------------------------- vanishing

// degree of a[0, n) (-1: zero polynomial), scanned from the top by a grid of DEG_GRID blocks:
// round k has block b take the (k DEG_GRID + b)-th chunk of DEG_CHUNK coefficients counted from
// the end, and every block stops once a nonzero coefficient was found at or above its next chunk
// -- the usual polynomial, nonzero near its top, costs one round (DEG_GRID x 32 KiB) instead of
// the whole array.  (A grid of one block per chunk scans everything: all of its blocks are
// resident before the top one finishes -- 0.198 ms at 2^23.6 coefficients, profiles/r06r_*.)
constexpr int DEG_CHUNK = 1024, DEG_GRID = 256;
__global__ void __launch_bounds__(256) k_degree(int n, const uint64_t *__restrict__ a, int *__restrict__ deg) {
  const long long nchunk = ((long long)n + DEG_CHUNK - 1) / DEG_CHUNK;
  const uint4 *x = reinterpret_cast<const uint4 *>(a);
  __shared__ int stop;
  for (long long c = nchunk - 1 - (long long)blockIdx.x; c >= 0; c -= gridDim.x) {
    const long long lo = c * DEG_CHUNK;
    if (threadIdx.x == 0) stop = __hip_atomic_load(deg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= lo;
    __syncthreads();
    if (stop) return;  // one value for the whole block
    const long long hi = min((long long)n, lo + DEG_CHUNK);
    int best = -1;
    uint4 u[DEG_CHUNK / 256][2];
#pragma unroll
    for (int k = 0; k < DEG_CHUNK / 256; k++) {  // every load of the chunk in flight at once
      const long long i = lo + (long long)threadIdx.x + 256 * k;
      u[k][0] = i < hi ? x[2 * i] : make_uint4(0, 0, 0, 0);
      u[k][1] = i < hi ? x[2 * i + 1] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < DEG_CHUNK / 256; k++)
      if (u[k][0].x | u[k][0].y | u[k][0].z | u[k][0].w | u[k][1].x | u[k][1].y | u[k][1].z | u[k][1].w)
        best = (int)(lo + (long long)threadIdx.x + 256 * k);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o, 64));  // one atomic per wavefront
    if ((threadIdx.x & 63) == 0 && best >= 0) atomicMax(deg, best);
    __syncthreads();  // every thread has read `stop` before thread 0 rewrites it
  }
}
// quotient by x^n - eta (deg_p >= n): q_j = a_{j+n} + eta q_{j+n}, one lane per residue
// class j mod n walking its chain from the top (poly_mont.c:360-372 / 337-347)
template <class F>
__global__ void __launch_bounds__(256) k_vanish_quot(int deg, int n, const uint64_t *__restrict__ a, U256 eta,
                                                     uint64_t *__restrict__ quot) {
  const int rho = blockIdx.x * blockDim.x + threadIdx.x;
  const int top = deg - n;  // largest quotient index
  if (rho >= n || rho > top) return;
  Fe<F> e, er;
  ld_const(er, eta);
  fe_to_int(e, er);
  Fe<F> q;
  fe_zero(q);
  const int jmax = rho + ((top - rho) / n) * n;
  for (int j = jmax; j >= rho; j -= n) {
    Fe<F> ai, t;
    ld(ai, a, (size_t)j + n);
    fe_mul(t, e, q);  // eta * q_{j+n} (0 at the top of the chain)
    fe_add(q, ai, t);
    st(quot, (size_t)j, q);
  }
}
// The same chains fused with the remainder, on the LDS-staged nontemporal 1-KiB runs of the Fr
// ops: wavefront w owns residues [e0, e0 + 64) and walks their chains top-down in lockstep -- at
// step s its lanes read a[e0 + s n + n ..] and write quot[e0 + s n ..], each a contiguous run
// (lanes whose chain has not started read past the degree, i.e. zeros, and keep q = 0, so no
// masking); after step 0 each lane holds q_rho and writes rem_rho = a_rho + eta q_rho (q_rho = 0
// for rho > deg - n, where the remainder is a_rho itself).  Every quotient index <= deg - n and
// every remainder index < n is written; the host clears only the buffers' tails.
// STAGED = false (the default, see div_vanishing_t): the same fused chains with per-lane 32-B accesses
template <class F, bool STAGED = true>
__global__ void __launch_bounds__(256) k_vanish_fused(int deg, int n, const uint64_t *__restrict__ a, U256 eta,
                                                      uint64_t *__restrict__ quot, uint64_t *__restrict__ rem) {
  __shared__ uint4 lds[4][128];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t e0 = (size_t)blockIdx.x * 256 + (size_t)wave * 64;
  if (e0 >= (size_t)n) return;  // wave-uniform
  const size_t top = (size_t)(deg - n), N = (size_t)n;
  const size_t rlim = (size_t)min((size_t)n, e0 + 64);  // residues of this wave: [e0, rlim)
  Fe<F> e, er, q;
  ld_const(er, eta);
  fe_to_int(e, er);
  fe_zero(q);
  if constexpr (!STAGED) {
    const size_t rho = e0 + lane;
    if (rho >= N) return;
    if (rho <= top) {
      for (size_t j = rho + ((top - rho) / N) * N;; j -= N) {
        Fe<F> ai, t;
        ld(ai, a, j + N);
        fe_mul(t, e, q);
        fe_add(q, ai, t);
        st(quot, j, q);
        if (j < N) break;
      }
    }
    Fe<F> ar, t, r;
    ld(ar, a, rho);
    fe_mul(t, e, q);
    fe_add(r, ar, t);
    st(rem, rho, r);
    return;
  }
  // every load is independent of the products: the remainder's runs are fetched first and each
  // step's runs one step ahead (registers), so a wavefront keeps loads in flight through its chain
  Runs rr, rn;
  fetch_runs<true>(rr, a, e0, rlim, lane);
  if (e0 <= top) {
    const size_t lim = (size_t)deg + 1;
    size_t s = (top - e0) / N;  // chain length of residue e0 (the longest) - 1
    fetch_runs<true>(rn, a, e0 + s * N + N, lim, lane);
    for (;;) {
      const size_t j0 = e0 + s * N;
      Fe<F> ai, t;
      place_runs(ai, rn, lds[wave], lane);
      if (s > 0) fetch_runs<true>(rn, a, j0, lim, lane);  // step s - 1 reads a[j0 - N + N ..]
      fe_mul(t, e, q);
      fe_add(q, ai, t);
      st_staged<F, true>(quot, j0, min(top + 1, rlim + s * N), q, lds[wave], lane);
      if (s == 0) break;
      s--;
    }
  }
  Fe<F> ar, t, r;
  place_runs(ar, rr, lds[wave], lane);
  fe_mul(t, e, q);
  fe_add(r, ar, t);
  st_staged<F, true>(rem, e0, rlim, r, lds[wave], lane);
}
template <class F>
__global__ void __launch_bounds__(256) k_vanish_rem(int deg, int n, const uint64_t *__restrict__ a,
                                                    const uint64_t *__restrict__ quot, U256 eta,
                                                    uint64_t *__restrict__ rem) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  Fe<F> aj, r;
  ld(aj, a, j);
  if (j <= deg - n) {
    Fe<F> e, er, q, t;
    ld_const(er, eta);
    fe_to_int(e, er);
    ld(q, quot, j);
    fe_mul(t, e, q);
    fe_add(r, aj, t);
  } else {
    r = aj;
  }
  st(rem, j, r);
}

// ---------------------------------------------------------------------------- host side

struct CfgBN { using Fd = BN_Fr; using Fh = zkh::BN_Fr; };
struct CfgBLS { using Fd = BLS_Fr; using Fh = zkh::BLS_Fr; };

template <class Fh>
static U256 to_u256(const zkh::Fe<Fh> &x) {
  U256 u;
  for (int j = 0; j < 4; j++) u.w[j] = x.v[j];
  return u;
}
static U256 load_u256(const uint64_t *p) {
  U256 u = {{0, 0, 0, 0}};
  if (p) for (int j = 0; j < 4; j++) u.w[j] = p[j];
  return u;
}

// R * R' mod p as a plain integer: R' = 2^(RB N) = R * 2^(RB N - 256), so R R' = R^2 2^d
template <class Cfg>
static U256 from_std_const() {
  using Fh = typename Cfg::Fh;
  using Fd = typename Cfg::Fd;
  zkh::Fe<Fh> x;
  memcpy(x.v, Fh::R2, sizeof x.v);
  for (int d = 0; d < Fd::RB * Fd::N - 64 * Fh::N; d++) zkh::add(x, x, x);
  return to_u256(x);
}
template <class Cfg>
static U256 p_minus_2() {
  using Fh = typename Cfg::Fh;
  U256 e;
  for (int j = 0; j < 4; j++) e.w[j] = Fh::P[j];
  uint64_t br = 2;
  for (int j = 0; j < 4 && br; j++) {
    const uint64_t o = e.w[j];
    e.w[j] = o - br;
    br = o < br ? 1 : 0;
  }
  return e;
}

static unsigned grid_for(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;  // grid-stride loops beyond ~16 waves per SIMD
  return (unsigned)(b ? b : 1);
}

// staging of host operands: every array is copied into the call's arena
struct Stage {
  Device &dev;
  bool host;
  explicit Stage(Device &d, bool h) : dev(d), host(h) {}
  const uint64_t *in(const uint64_t *p, size_t n) {
    if (!host || !p) return p;
    uint64_t *d = dev.arena.take<uint64_t>(n * 4);
    if (n) ZK_CHECK(hipMemcpyAsync(d, p, n * 32, hipMemcpyHostToDevice, dev.stream));
    return d;
  }
  uint64_t *out(uint64_t *p, size_t n) { return host ? dev.arena.take<uint64_t>(n * 4) : p; }
  void back(uint64_t *host_p, const uint64_t *dev_p, size_t n) {  // waits (pinned pieces for large outputs)
    if (host && n) copy_to_host(dev, dev.stream, host_p, dev_p, n * 32);
  }
};

// ZK_ARR_STAGE (A/B hook; default: 4 for the streaming ops, 2 for the ops with a product per
// element): 2 staged + nontemporal, 4 the same software-pipelined (every array's runs fetched before
// the first is placed; with a grid-stride loop the next step's runs fly during the products), 1
// staged, 0 per-lane 32-B accesses; ZK_ARR_MAP=1: the round-5 single switch kernel k_arr_map.
// Grid: the streaming shapes are fastest with one workgroup per 256 elements (no grid-stride loop:
// add / sub 5.8-6.0 TB/s at 2^24, copy 5.8) or 1024 workgroups, and worst at the 4096 the round-5
// kernel used (tools/microbench/stream_bw.hip, profiles/r06c_stream_bw.txt); the ops with a product
// per element overlap it with the streams best at 4096-8192 workgroups (scale 4.4 -> 4.8 TB/s, mul
// 4.8 -> 5.0-5.2, Ax_plus_y 5.0 -> 5.35 at 8192; profiles/r06e_arr_ab.txt, r06f_arr_grid.txt,
// r06i_arr_pf_grid.txt).  Stage 4 on the streaming ops: mul_add 5.6 -> 6.0 TB/s, add / sub / copy
// 5.7-5.9 -> 5.8-6.1 (r06h_arr_pf_ab.txt, r06i); on the product ops it measured level or slower.
// ZK_ARR_GRID overrides the cap for every op (A/B hook, read once).
static unsigned stream_grid(size_t n, bool products = false) {
  static const size_t cap_env = [] {
    const char *e = getenv("ZK_ARR_GRID");
    const long v = e ? atol(e) : 0;
    return v > 0 ? (size_t)v : (size_t)0;
  }();
  const size_t cap = cap_env ? cap_env : (products ? (size_t)8192 : (size_t)1 << 30);
  size_t b = (n + 255) / 256;
  if (b > cap) b = cap;
  return (unsigned)(b ? b : 1);
}
static bool arr_op_has_product(int op) {
  return op == ARR_SQR || op == ARR_MUL || op == ARR_SCALE || op == ARR_AXPY || op == ARR_AXPBY ||
         op == ARR_FROM_STD || op == ARR_TO_STD;
}
template <class F>
static void launch_arr_op(int op, const ArrArgs &g, dim3 grid, hipStream_t st) {
  static const int stage_env = [] {
    const char *e = getenv("ZK_ARR_STAGE");
    return e ? atoi(e) : -1;
  }();
  const int stage = stage_env >= 0 ? stage_env : (arr_op_has_product(op) ? 2 : 4);
  static const bool legacy = [] {
    const char *e = getenv("ZK_ARR_MAP");
    return e && e[0] == '1';
  }();
  if (legacy) {
    hipLaunchKernelGGL(k_arr_map<F>, grid, dim3(256), 0, st, g);
    ZK_CHECK(hipGetLastError());
    return;
  }
#define ZK_ARR_CASE(OPC)                                                                   \
  case OPC:                                                                                \
    if (stage == 4) hipLaunchKernelGGL((k_arr_op<F, OPC, true, true, true>), grid, dim3(256), 0, st, g);  \
    else if (stage == 2) hipLaunchKernelGGL((k_arr_op<F, OPC, true, true>), grid, dim3(256), 0, st, g);   \
    else if (stage == 1) hipLaunchKernelGGL((k_arr_op<F, OPC, true, false>), grid, dim3(256), 0, st, g);  \
    else hipLaunchKernelGGL((k_arr_op<F, OPC, false, false>), grid, dim3(256), 0, st, g);                 \
    break;
  switch (op) {
    ZK_ARR_CASE(ARR_NEG)
    ZK_ARR_CASE(ARR_ADD)
    ZK_ARR_CASE(ARR_SUB)
    ZK_ARR_CASE(ARR_SUB_REV)
    ZK_ARR_CASE(ARR_SQR)
    ZK_ARR_CASE(ARR_MUL)
    ZK_ARR_CASE(ARR_MUL_ADD)
    ZK_ARR_CASE(ARR_MUL_SUB)
    ZK_ARR_CASE(ARR_SCALE)
    ZK_ARR_CASE(ARR_AXPY)
    ZK_ARR_CASE(ARR_AXPBY)
    ZK_ARR_CASE(ARR_FROM_STD)
    ZK_ARR_CASE(ARR_TO_STD)
    ZK_ARR_CASE(ARR_COPY)
    ZK_ARR_CASE(ARR_SET_CONST)
    default: ZK_REQUIRE(false, "arr op: unknown op code");
  }
#undef ZK_ARR_CASE
  ZK_CHECK(hipGetLastError());
}

template <class Cfg>
static void arr_op_t(Device &dev, int op, int n, const uint64_t *a, const uint64_t *b, const uint64_t *c,
                     const uint64_t *kA, const uint64_t *kB, uint64_t *tgt, bool host_io) {
  using F = typename Cfg::Fd;
  hipStream_t st = dev.stream;
  const size_t N = (size_t)(n > 0 ? n : 0);
  dev.arena.reserve(N * 32 * 5 + (1 << 20));
  dev.arena.reset();
  Stage sg(dev, host_io);
  const bool needb = op == ARR_ADD || op == ARR_SUB || op == ARR_SUB_REV || op == ARR_MUL || op == ARR_MUL_ADD ||
                     op == ARR_MUL_SUB || op == ARR_AXPY || op == ARR_AXPBY || op == ARR_DIV;
  const bool needa = op != ARR_SET_CONST;
  const uint64_t *da = needa ? sg.in(a, N) : nullptr;
  const uint64_t *db = needb ? sg.in(b, N) : nullptr;
  const uint64_t *dc = (op == ARR_MUL_ADD || op == ARR_MUL_SUB) ? sg.in(c, N) : nullptr;
  uint64_t *dt = sg.out(tgt, N);
  if (N) {
    if (op == ARR_INV || op == ARR_DIV) {
      // elements per Fermat inversion: a lane's chain is ~6 products per element plus one
      // inversion (323 products with the sliding window), the work N (6 + 323 / CHK); the lanes
      // N / CHK are sized to ZK_INV_LANES (default 131072: two wavefronts per SIMD at 164 VGPRs),
      // CHK within [8, 128] (2^24: 128 -> 8.5 products per element instead of 16 at CHK 32; inv
      // 2.64 -> 1.94 ms, div 2.35 -> 1.86 ms through the host wrapper, profiles/r05u_*)
      static const size_t inv_lanes = [] {
        const char *e = getenv("ZK_INV_LANES");
        const long v = e ? atol(e) : 0;
        return v > 0 ? (size_t)v : (size_t)131072;
      }();
      const size_t cq = N / inv_lanes;
      const int CHK = cq < 8 ? 8 : (cq > 128 ? 128 : (int)cq);
      uint64_t *scratch = dev.arena.take<uint64_t>(N * 4);
      uint32_t *flag = dev.arena.take<uint32_t>(1);
      ZK_CHECK(hipMemsetAsync(flag, 0, 4, st));
      const size_t lanes = (N + CHK - 1) / CHK;
      static const bool sg = [] {
        const char *e = getenv("ZK_INV_SG");
        return !(e && e[0] == '0');
      }();
      static const bool strided = [] {
        const char *e = getenv("ZK_INV_STRIDE");
        return !(e && e[0] == '0');
      }();
      const dim3 ig(div_up(lanes, 256)), ib(256);
      const uint64_t *xs = op == ARR_DIV ? db : da;
      const U256 pm2 = p_minus_2<Cfg>();
      static const bool ilp2 = [] {
        const char *e = getenv("ZK_INV_ILP");
        return !(e && e[0] == '0');
      }();
      if (sg && strided && ilp2)
        hipLaunchKernelGGL(k_inv_chunks2<F>, ig, ib, 0, st, op, n, CHK, op == ARR_DIV ? da : xs, xs, scratch, dt, flag, (int)lanes);
      else if (sg && strided)
        hipLaunchKernelGGL((k_inv_chunks<F, true, true>), ig, ib, 0, st, op, n, CHK, da, xs, scratch, dt, pm2, flag, (int)lanes);
      else if (sg)
        hipLaunchKernelGGL((k_inv_chunks<F, true, false>), ig, ib, 0, st, op, n, CHK, da, xs, scratch, dt, pm2, flag, (int)lanes);
      else
        hipLaunchKernelGGL((k_inv_chunks<F, false, false>), ig, ib, 0, st, op, n, CHK, da, xs, scratch, dt, pm2, flag, (int)lanes);
      ZK_CHECK(hipGetLastError());
      hipLaunchKernelGGL(k_zero_if_flag, dim3(grid_for(N * 4)), dim3(256), 0, st, n, dt, flag);
      ZK_CHECK(hipGetLastError());
    } else {
      ArrArgs g;
      g.op = op;
      g.n = n;
      g.a = da;
      g.b = db;
      g.c = dc;
      g.tgt = dt;
      g.kA = load_u256(kA);
      g.kB = load_u256(kB);
      g.cstd = from_std_const<Cfg>();
      launch_arr_op<F>(op, g, dim3(stream_grid(N, arr_op_has_product(op))), st);
    }
  }
  sg.back(tgt, dt, N);
  ZK_CHECK(hipStreamSynchronize(st));
}

template <class Cfg>
static int arr_pred_t(Device &dev, int pred, int n, const uint64_t *a, const uint64_t *b, bool host_io) {
  using Fh = typename Cfg::Fh;
  hipStream_t st = dev.stream;
  const size_t N = (size_t)(n > 0 ? n : 0);
  dev.arena.reserve(N * 32 * 2 + (1 << 20));
  dev.arena.reset();
  Stage sg(dev, host_io);
  const uint64_t *da = sg.in(a, N);
  const uint64_t *db = pred == PRED_IS_EQUAL ? sg.in(b, N) : nullptr;
  uint32_t *fail = dev.arena.take<uint32_t>(1);
  ZK_CHECK(hipMemsetAsync(fail, 0, 4, st));
  U256 prime, one;
  for (int j = 0; j < 4; j++) { prime.w[j] = Fh::P[j]; one.w[j] = Fh::ONE[j]; }
  if (N) {
    hipLaunchKernelGGL(k_pred, dim3(grid_for(N)), dim3(256), 0, st, pred, n, da, db, prime, one, fail);
    ZK_CHECK(hipGetLastError());
  }
  uint32_t *h = reinterpret_cast<uint32_t *>(dev.host_staging(4));
  ZK_CHECK(hipMemcpyAsync(h, fail, 4, hipMemcpyDeviceToHost, st));
  ZK_CHECK(hipStreamSynchronize(st));
  return *h ? 0 : 1;
}

template <class Cfg>
static void arr_dot_t(Device &dev, int n, const uint64_t *a, const uint64_t *b, uint64_t *tgt_host, bool host_io) {
  using F = typename Cfg::Fd;
  hipStream_t st = dev.stream;
  const size_t N = (size_t)(n > 0 ? n : 0);
  dev.arena.reserve(N * 32 * 2 + (1 << 20));
  dev.arena.reset();
  Stage sg(dev, host_io);
  const uint64_t *da = sg.in(a, N), *db = sg.in(b, N);
  unsigned blocks = grid_for(N);
  if (blocks > 1024) blocks = 1024;
  uint64_t *part = dev.arena.take<uint64_t>((size_t)blocks * 4);
  uint64_t *out = dev.arena.take<uint64_t>(4);
  hipLaunchKernelGGL(k_dot<F>, dim3(blocks), dim3(DOT_THREADS), 0, st, n, da, db, part);
  ZK_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_dot_final<F>, dim3(1), dim3(DOT_THREADS), 0, st, (int)blocks, part, out);
  ZK_CHECK(hipGetLastError());
  uint64_t *h = reinterpret_cast<uint64_t *>(dev.host_staging(32));
  ZK_CHECK(hipMemcpyAsync(h, out, 32, hipMemcpyDeviceToHost, st));
  ZK_CHECK(hipStreamSynchronize(st));
  memcpy(tgt_host, h, 32);
}

template <class Cfg>
static void arr_powers_t(Device &dev, int n, const uint64_t *kA, const uint64_t *kB, uint64_t *tgt, bool host_io) {
  using F = typename Cfg::Fd;
  hipStream_t st = dev.stream;
  if (n <= 0) return;  // powers: n == 0 writes nothing (arr_mont.c)
  const size_t N = (size_t)n;
  int lg = 0;
  while (((size_t)1 << lg) < N) lg++;
  const int h = (lg + 1) / 2;
  const int nlo = 1 << h, nhi = (int)((N + nlo - 1) >> h);
  dev.arena.reserve(N * 32 + ((size_t)nlo + nhi) * 32 + (1 << 20));
  dev.arena.reset();
  Stage sg(dev, host_io);
  uint64_t *dt = sg.out(tgt, N);
  uint64_t *tlo = dev.arena.take<uint64_t>((size_t)nlo * 4);
  uint64_t *thi = dev.arena.take<uint64_t>((size_t)nhi * 4);
  const int nt = nlo > nhi ? nlo : nhi;
  hipLaunchKernelGGL(k_pow_tables<F>, dim3(div_up(nt, 256)), dim3(256), 0, st, h, nlo, nhi, load_u256(kA),
                     load_u256(kB), tlo, thi);
  ZK_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_powers<F>, dim3(stream_grid(N, true)), dim3(256), 0, st, n, h, tlo, thi, dt);
  ZK_CHECK(hipGetLastError());
  sg.back(tgt, dt, N);
  ZK_CHECK(hipStreamSynchronize(st));
}

template <class Cfg>
static int div_vanishing_t(Device &dev, int n1, const uint64_t *src, int n, const uint64_t *eta, int nquot,
                           uint64_t *quot, int nrem, uint64_t *rem, bool host_io) {
  hipStream_t st = dev.stream;
  ZK_REQUIRE(n >= 1, "poly_div_by_vanishing: expo_n must be >= 1");  // poly_mont.c:330
  ZK_REQUIRE(quot != nullptr, "poly_div_by_vanishing: quot cannot be NULL");  // poly_mont.c:327
  const size_t N1 = (size_t)(n1 > 0 ? n1 : 0);
  const bool want_rem = rem != nullptr;
  const size_t NR = want_rem ? (size_t)nrem : (size_t)n;  // quot_by_vanishing: internal rem of n
  dev.arena.reserve((N1 + (size_t)nquot + NR) * 32 + (1 << 20));
  dev.arena.reset();
  Stage sg(dev, host_io);
  const uint64_t *da = sg.in(src, N1);
  uint64_t *dq = sg.out(quot, (size_t)nquot);
  uint64_t *dr = want_rem ? sg.out(rem, NR) : dev.arena.take<uint64_t>(NR * 4);
  int *ddeg = dev.arena.take<int>(1);
  ZK_CHECK(hipMemsetAsync(ddeg, 0xff, 4, st));  // -1
  if (N1) {
    hipLaunchKernelGGL(k_degree, dim3((unsigned)std::min<size_t>(DEG_GRID, (N1 + DEG_CHUNK - 1) / DEG_CHUNK)), dim3(256), 0,
                       st, n1, da, ddeg);
    ZK_CHECK(hipGetLastError());
  }
  int *hdeg = reinterpret_cast<int *>(dev.host_staging(4));
  ZK_CHECK(hipMemcpyAsync(hdeg, ddeg, 4, hipMemcpyDeviceToHost, st));
  ZK_CHECK(hipStreamSynchronize(st));
  const int deg = *hdeg;
  ZK_REQUIRE(nquot >= deg - n + 1, "poly_div_by_vanishing: quotient buffer too small");  // poly_mont.c:328
  ZK_REQUIRE(!want_rem || nrem >= n, "poly_div_by_vanishing: remainder buffer too small");  // :329
  const U256 e = load_u256(eta);
  static const bool legacy = [] {  // ZK_VANISH_LEGACY=1: the round-5 kernels (A/B hook, read once)
    const char *v = getenv("ZK_VANISH_LEGACY");
    return v && v[0] == '1';
  }();
  // the fused kernel writes quot[0, deg - n] and rem[0, n): only the tails are cleared
  const size_t qw = (deg >= n && !legacy) ? (size_t)(deg - n + 1) : 0, rw = (deg >= n && !legacy) ? (size_t)n : 0;
  if ((size_t)nquot > qw) ZK_CHECK(hipMemsetAsync(dq + qw * 4, 0, ((size_t)nquot - qw) * 32, st));
  if (NR > rw) ZK_CHECK(hipMemsetAsync(dr + rw * 4, 0, (NR - rw) * 32, st));
  if (deg < n) {  // quotient 0, remainder = p (poly_mont.c:332-341)
    if (deg >= 0) {
      ZK_REQUIRE(NR >= (size_t)deg + 1, "poly_div_by_vanishing: remainder buffer too small");
      ZK_CHECK(hipMemcpyAsync(dr, da, (size_t)(deg + 1) * 32, hipMemcpyDeviceToDevice, st));
    }
  } else {
    using F = typename Cfg::Fd;
    if (legacy) {
      hipLaunchKernelGGL(k_vanish_quot<F>, dim3(div_up(n, 256)), dim3(256), 0, st, deg, n, da, e, dq);
      ZK_CHECK(hipGetLastError());
      hipLaunchKernelGGL(k_vanish_rem<F>, dim3(div_up(n, 256)), dim3(256), 0, st, deg, n, da, dq, e, dr);
    } else {
      // per-lane 32-B accesses by default: 0.186 vs 0.197 ms for the LDS-staged runs at deg 3 x 2^22
      // (profiles/r06r_vanish_prof.txt); ZK_VANISH_STAGED=1 selects those (A/B hook, read once)
      static const bool staged = [] {
        const char *v = getenv("ZK_VANISH_STAGED");
        return v && v[0] == '1';
      }();
      if (staged) hipLaunchKernelGGL((k_vanish_fused<F, true>), dim3(div_up(n, 256)), dim3(256), 0, st, deg, n, da, e, dq, dr);
      else hipLaunchKernelGGL((k_vanish_fused<F, false>), dim3(div_up(n, 256)), dim3(256), 0, st, deg, n, da, e, dq, dr);
    }
    ZK_CHECK(hipGetLastError());
  }
  sg.back(quot, dq, (size_t)nquot);
  if (want_rem) {
    sg.back(rem, dr, NR);
    ZK_CHECK(hipStreamSynchronize(st));
    return -1;
  }
  // quot_by_vanishing: is the remainder (n coefficients) zero?
  uint32_t *fail = dev.arena.take<uint32_t>(1);
  ZK_CHECK(hipMemsetAsync(fail, 0, 4, st));
  U256 z = {{0, 0, 0, 0}};
  hipLaunchKernelGGL(k_pred, dim3(grid_for(NR)), dim3(256), 0, st, (int)PRED_IS_ZERO, (int)NR, dr, nullptr, z, z,
                     fail);
  ZK_CHECK(hipGetLastError());
  uint32_t *h = reinterpret_cast<uint32_t *>(dev.host_staging(4));
  ZK_CHECK(hipMemcpyAsync(h, fail, 4, hipMemcpyDeviceToHost, st));
  ZK_CHECK(hipStreamSynchronize(st));
  return *h ? 0 : 1;
}

// ---------------------------------------------------------------------------- public

void arr_op(int curve, int op, int n, const uint64_t *a, const uint64_t *b, const uint64_t *c, const uint64_t *kA,
            const uint64_t *kB, uint64_t *tgt, bool host_io) {
  ZK_REQUIRE(op >= 0 && op < ARR_NUM_OPS, "arr_op: unknown operation");
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  if (curve == 0) arr_op_t<CfgBN>(dev, op, n, a, b, c, kA, kB, tgt, host_io);
  else arr_op_t<CfgBLS>(dev, op, n, a, b, c, kA, kB, tgt, host_io);
}
int arr_pred(int curve, int pred, int n, const uint64_t *a, const uint64_t *b, bool host_io) {
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  return curve == 0 ? arr_pred_t<CfgBN>(dev, pred, n, a, b, host_io) : arr_pred_t<CfgBLS>(dev, pred, n, a, b, host_io);
}
void arr_dot(int curve, int n, const uint64_t *a, const uint64_t *b, uint64_t *tgt_host, bool host_io) {
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  if (curve == 0) arr_dot_t<CfgBN>(dev, n, a, b, tgt_host, host_io);
  else arr_dot_t<CfgBLS>(dev, n, a, b, tgt_host, host_io);
}
void arr_powers(int curve, int n, const uint64_t *kA, const uint64_t *kB, uint64_t *tgt, bool host_io) {
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  if (curve == 0) arr_powers_t<CfgBN>(dev, n, kA, kB, tgt, host_io);
  else arr_powers_t<CfgBLS>(dev, n, kA, kB, tgt, host_io);
}
int poly_div_by_vanishing(int curve, int n1, const uint64_t *src, int expo_n, const uint64_t *eta, int nquot,
                          uint64_t *quot, int nrem, uint64_t *rem, bool host_io) {
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  return curve == 0 ? div_vanishing_t<CfgBN>(dev, n1, src, expo_n, eta, nquot, quot, nrem, rem, host_io)
                    : div_vanishing_t<CfgBLS>(dev, n1, src, expo_n, eta, nquot, quot, nrem, rem, host_io);
}

}  // namespace zk
