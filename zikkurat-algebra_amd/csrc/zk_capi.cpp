// zk_capi.cpp -- the extern "C" boundary (include/zkalgebra_gpu.h).
//
// Part 1 mirrors the reference's generated C entry points one for one:
//   <C>_G1_proj_MSM_{mont,std}_coeff_{proj,affine}_out  bls12_381_G1_proj.c:597-670
//   <C>_G1_proj_MSM_std_coeff_proj_out_variable          bls12_381_G1_proj.c:507
//   <C>_G1_jac_MSM_{mont,std}_coeff_{jac,affine}_out    bls12_381_G1_jac.c:555-718
//   <C>_poly_mont_ntt_{forward,inverse}                  bls12_381_poly_mont.c:457,516
// Every one of them runs on the GPU; there is no CPU fallback path.
#include <hip/hip_runtime.h>
#include <string.h>
#include "../../include/zkalgebra_gpu.h"
#include "zk_gen.hpp"
#include "zk_host.hpp"
#include "zk_msm.hpp"
#include "zk_ntt.hpp"
#include "zk_runtime.hpp"

using namespace zk;

namespace {

enum Out { PROJ, AFFINE, JAC };

template <class C>
void msm_entry(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int nl, bool mont,
               int window, Out out) {
  using HF = typename HostOf<C>::Fp;
  constexpr int NP = C::NP64;
  uint64_t proj[3 * NP];
  bool ok = false;
  guard([&] {
    msm_g1<C>(npoints, expos, nl, grps, /*host_inputs=*/true, mont, window, proj);
    ok = true;
  });
  if (!ok) return;  // recoverable error mode: the message is in zkg_last_error
  zkh::Proj<HF> p;
  memcpy(p.X.v, proj, NP * 8);
  memcpy(p.Y.v, proj + NP, NP * 8);
  memcpy(p.Z.v, proj + 2 * NP, NP * 8);
  if (out == AFFINE) {
    zkh::Aff<HF> a;
    zkh::proj_to_aff(a, p);
    memcpy(tgt, a.x.v, NP * 8);
    memcpy(tgt + NP, a.y.v, NP * 8);
    return;
  }
  zkh::Proj<HF> q;
  zkh::proj_normalize(q, p);
  if (out == JAC && zkh::proj_is_inf(q)) zkh::set_one(q.X);  // Jacobian infinity (1:1:0), G1_jac.c:183-187
  memcpy(tgt, q.X.v, NP * 8);
  memcpy(tgt + NP, q.Y.v, NP * 8);
  memcpy(tgt + 2 * NP, q.Z.v, NP * 8);
}

template <class HF, class C>
void host_b3(zkh::Fe<HF> &b3) { HostOf<C>::b3(b3); }

}  // namespace

extern "C" {

#define ZKG_MSM_ENTRIES(PFX, CURVE)                                                                             \
  ZKG_API void PFX##_G1_proj_MSM_mont_coeff_proj_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t,  \
                                                     int nl) {                                                  \
    msm_entry<CURVE>(n, e, g, t, nl, true, 0, PROJ);                                                           \
  }                                                                                                             \
  ZKG_API void PFX##_G1_proj_MSM_std_coeff_proj_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t,   \
                                                    int nl) {                                                   \
    msm_entry<CURVE>(n, e, g, t, nl, false, 0, PROJ);                                                          \
  }                                                                                                             \
  ZKG_API void PFX##_G1_proj_MSM_mont_coeff_affine_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t, \
                                                       int nl) {                                                \
    msm_entry<CURVE>(n, e, g, t, nl, true, 0, AFFINE);                                                         \
  }                                                                                                             \
  ZKG_API void PFX##_G1_proj_MSM_std_coeff_affine_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t,  \
                                                      int nl) {                                                 \
    msm_entry<CURVE>(n, e, g, t, nl, false, 0, AFFINE);                                                        \
  }                                                                                                             \
  ZKG_API void PFX##_G1_proj_MSM_std_coeff_proj_out_variable(int n, const uint64_t *e, const uint64_t *g,       \
                                                             uint64_t *t, int nl, int window) {                 \
    int c = window < 4 ? 4 : (window > 24 ? 24 : window);                                                       \
    msm_entry<CURVE>(n, e, g, t, nl, false, c, PROJ);                                                          \
  }                                                                                                             \
  ZKG_API void PFX##_G1_jac_MSM_std_coeff_jac_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t,     \
                                                  int nl) {                                                     \
    msm_entry<CURVE>(n, e, g, t, nl, false, 0, JAC);                                                           \
  }                                                                                                             \
  ZKG_API void PFX##_G1_jac_MSM_mont_coeff_jac_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t,    \
                                                   int nl) {                                                    \
    msm_entry<CURVE>(n, e, g, t, nl, true, 0, JAC);                                                            \
  }                                                                                                             \
  ZKG_API void PFX##_G1_jac_MSM_std_coeff_affine_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t,  \
                                                     int nl) {                                                  \
    msm_entry<CURVE>(n, e, g, t, nl, false, 0, AFFINE);                                                        \
  }                                                                                                             \
  ZKG_API void PFX##_G1_jac_MSM_mont_coeff_affine_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t, \
                                                      int nl) {                                                 \
    msm_entry<CURVE>(n, e, g, t, nl, true, 0, AFFINE);                                                         \
  }

ZKG_MSM_ENTRIES(bn128, BN254)
ZKG_MSM_ENTRIES(bls12_381, BLS381)

// G2 MSM: <C>_G2_proj_MSM_* (bls12_381_G2_proj.h:43-46)
#define ZKG_G2_MSM_ENTRIES(PFX, CURVE)                                                                          \
  ZKG_API void PFX##_G2_proj_MSM_mont_coeff_proj_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t,  \
                                                     int nl) {                                                  \
    msm_entry<CURVE>(n, e, g, t, nl, true, 0, PROJ);                                                           \
  }                                                                                                             \
  ZKG_API void PFX##_G2_proj_MSM_std_coeff_proj_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t,   \
                                                    int nl) {                                                   \
    msm_entry<CURVE>(n, e, g, t, nl, false, 0, PROJ);                                                          \
  }                                                                                                             \
  ZKG_API void PFX##_G2_proj_MSM_mont_coeff_affine_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t, \
                                                       int nl) {                                                \
    msm_entry<CURVE>(n, e, g, t, nl, true, 0, AFFINE);                                                         \
  }                                                                                                             \
  ZKG_API void PFX##_G2_proj_MSM_std_coeff_affine_out(int n, const uint64_t *e, const uint64_t *g, uint64_t *t,  \
                                                      int nl) {                                                 \
    msm_entry<CURVE>(n, e, g, t, nl, false, 0, AFFINE);                                                        \
  }

ZKG_G2_MSM_ENTRIES(bn128, BN254_G2)
ZKG_G2_MSM_ENTRIES(bls12_381, BLS381_G2)

ZKG_API void bn128_poly_mont_ntt_forward(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {
  guard([&] { zk::ntt(ZKG_BN128, m, gen, src, tgt, true, false); });
}
ZKG_API void bn128_poly_mont_ntt_inverse(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {
  guard([&] { zk::ntt(ZKG_BN128, m, gen, src, tgt, true, true); });
}
ZKG_API void bls12_381_poly_mont_ntt_forward(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {
  guard([&] { zk::ntt(ZKG_BLS12_381, m, gen, src, tgt, true, false); });
}
ZKG_API void bls12_381_poly_mont_ntt_inverse(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt) {
  guard([&] { zk::ntt(ZKG_BLS12_381, m, gen, src, tgt, true, true); });
}

// ---------------------------------------------------------------------------- Part 2

ZKG_API const char *zkg_version(void) { return "zkalgebra_gpu 0.1 (gfx950)"; }

ZKG_API int zkg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
ZKG_API void zkg_set_error_mode(int mode) { zk::set_error_mode(mode); }
ZKG_API int zkg_last_error(char *msg, size_t cap) { return zk::take_last_error(msg, cap); }

ZKG_API void zkg_set_device(int device) {
  guard([&] { ZK_CHECK(hipSetDevice(device)); });
}
ZKG_API void *zkg_device_malloc(size_t bytes) {
  return guard_ret<void *>(nullptr, [&] {
    void *p = nullptr;
    ZK_CHECK(hipMalloc(&p, bytes ? bytes : 1));
    return p;
  });
}
ZKG_API void zkg_device_free(void *ptr) {
  guard([&] {
    if (ptr) ZK_CHECK(hipFree(ptr));
  });
}
ZKG_API void zkg_memcpy_htod(void *dst, const void *src, size_t bytes) {
  guard([&] { ZK_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)); });
}
ZKG_API void zkg_memcpy_dtoh(void *dst, const void *src, size_t bytes) {
  guard([&] { ZK_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost)); });
}
ZKG_API void zkg_device_synchronize(void) {
  guard([&] { ZK_CHECK(hipDeviceSynchronize()); });
}

ZKG_API void zkg_g1_msm_device(int curve, int npoints, const uint64_t *d_expos, int expo_nlimbs, int expos_mont,
                               const uint64_t *d_grps, uint64_t *tgt_proj, int window_size) {
  guard([&] {
  int c = window_size <= 0 ? 0 : (window_size < 4 ? 4 : (window_size > 24 ? 24 : window_size));
  if (curve == ZKG_BN128) {
    uint64_t p[12];
    msm_g1<BN254>(npoints, d_expos, expo_nlimbs, d_grps, false, expos_mont != 0, c, p);
    zkg_g1_proj_normalize(curve, p, tgt_proj);
  } else {
    uint64_t p[18];
    msm_g1<BLS381>(npoints, d_expos, expo_nlimbs, d_grps, false, expos_mont != 0, c, p);
    zkg_g1_proj_normalize(curve, p, tgt_proj);
  }
  });
}

ZKG_API void zkg_g2_msm_device(int curve, int npoints, const uint64_t *d_expos, int expo_nlimbs, int expos_mont,
                               const uint64_t *d_grps, uint64_t *tgt_proj, int window_size) {
  guard([&] {
  int c = window_size <= 0 ? 0 : (window_size < 4 ? 4 : (window_size > 24 ? 24 : window_size));
  if (curve == ZKG_BN128) {
    uint64_t p[24];
    msm_g1<BN254_G2>(npoints, d_expos, expo_nlimbs, d_grps, false, expos_mont != 0, c, p);
    zkh::Proj<HostOf<BN254_G2>::Fp> q, r;
    memcpy(&q, p, sizeof q);
    zkh::proj_normalize(r, q);
    memcpy(tgt_proj, &r, sizeof r);
  } else {
    uint64_t p[36];
    msm_g1<BLS381_G2>(npoints, d_expos, expo_nlimbs, d_grps, false, expos_mont != 0, c, p);
    zkh::Proj<HostOf<BLS381_G2>::Fp> q, r;
    memcpy(&q, p, sizeof q);
    zkh::proj_normalize(r, q);
    memcpy(tgt_proj, &r, sizeof r);
  }
  });
}

ZKG_API void zkg_ntt_device(int curve, int inverse, int m, const uint64_t *gen, const uint64_t *d_src,
                            uint64_t *d_tgt) {
  guard([&] { zk::ntt(curve, m, gen, d_src, d_tgt, false, inverse != 0); });
}

}  // extern "C"

template <class C>
static void proj_op(int op, const uint64_t *a, const uint64_t *b, uint64_t *out) {
  using HF = typename HostOf<C>::Fp;
  constexpr int NP = C::NP64;
  zkh::Proj<HF> p, q, r;
  memcpy(p.X.v, a, NP * 8);
  memcpy(p.Y.v, a + NP, NP * 8);
  memcpy(p.Z.v, a + 2 * NP, NP * 8);
  if (op == 0) {
    memcpy(q.X.v, b, NP * 8);
    memcpy(q.Y.v, b + NP, NP * 8);
    memcpy(q.Z.v, b + 2 * NP, NP * 8);
    zkh::Fe<HF> b3;
    HostOf<C>::b3(b3);
    zkh::proj_add(r, p, q, b3);
  } else if (op == 1) {
    zkh::proj_normalize(r, p);
  } else {
    zkh::Aff<HF> af;
    zkh::proj_to_aff(af, p);
    memcpy(out, af.x.v, NP * 8);
    memcpy(out + NP, af.y.v, NP * 8);
    return;
  }
  memcpy(out, r.X.v, NP * 8);
  memcpy(out + NP, r.Y.v, NP * 8);
  memcpy(out + 2 * NP, r.Z.v, NP * 8);
}

extern "C" {

ZKG_API void zkg_g1_proj_add(int curve, const uint64_t *a, const uint64_t *b, uint64_t *out) {
  if (curve == ZKG_BN128) proj_op<BN254>(0, a, b, out); else proj_op<BLS381>(0, a, b, out);
}
ZKG_API void zkg_g1_proj_normalize(int curve, const uint64_t *a, uint64_t *out) {
  if (curve == ZKG_BN128) proj_op<BN254>(1, a, nullptr, out); else proj_op<BLS381>(1, a, nullptr, out);
}
ZKG_API void zkg_g1_proj_to_affine(int curve, const uint64_t *a, uint64_t *out) {
  if (curve == ZKG_BN128) proj_op<BN254>(2, a, nullptr, out); else proj_op<BLS381>(2, a, nullptr, out);
}

ZKG_API void zkg_gen_fr(int curve, uint64_t seed, int64_t start, int64_t count, uint64_t *out) {
  if (curve == ZKG_BN128) zkg::gen_field<zkh::BN_Fr>(seed, start, count, out);
  else zkg::gen_field<zkh::BLS_Fr>(seed, start, count, out);
}

ZKG_API void zkg_gen_g1_points(int curve, uint64_t seed, int64_t start, int64_t count, uint64_t *out) {
  if (curve == ZKG_BN128) {
    const uint64_t gx[] = ZK_BN128_GX_FP64, gy[] = ZK_BN128_GY_FP64, b3[] = ZK_BN128_B3_FP64;
    zkg::gen_points<zkh::BN_Fp, zkh::BN_Fr>(seed, start, count, out, gx, gy, b3);
  } else {
    const uint64_t gx[] = ZK_BLS12_381_GX_FP64, gy[] = ZK_BLS12_381_GY_FP64, b3[] = ZK_BLS12_381_B3_FP64;
    zkg::gen_points<zkh::BLS_Fp, zkh::BLS_Fr>(seed, start, count, out, gx, gy, b3);
  }
}

ZKG_API void zkg_fft_generator(int curve, int m, uint64_t *out) {
  if (curve == ZKG_BN128) {
    zkh::Fe<zkh::BN_Fr> g;
    const uint64_t v[] = ZK_BN128_FFT_GEN_FR64;
    memcpy(g.v, v, sizeof g.v);
    for (int i = m; i < ZK_BN128_FFT_LOG; i++) zkh::sqr(g, g);
    memcpy(out, g.v, sizeof g.v);
  } else {
    zkh::Fe<zkh::BLS_Fr> g;
    const uint64_t v[] = ZK_BLS12_381_FFT_GEN_FR64;
    memcpy(g.v, v, sizeof g.v);
    for (int i = m; i < ZK_BLS12_381_FFT_LOG; i++) zkh::sqr(g, g);
    memcpy(out, g.v, sizeof g.v);
  }
}

ZKG_API int zkg_msm_default_window(int npoints) { return zk::msm_default_window(npoints); }
ZKG_API int zkg_msm_window(int curve, int npoints, int expo_nlimbs, int expos_mont) {
  const int bits = expos_mont ? (curve == ZKG_BN128 ? 254 : 255) : 64 * (expo_nlimbs < 4 ? expo_nlimbs : 4);
  return zk::msm_default_window_bits(npoints, bits);
}

ZKG_API void zkg_msm_profile(int on) { zk::msm_set_profile(on); }
ZKG_API void zkg_msm_set_group_limit(size_t entries) { zk::msm_set_group_limit(entries); }
ZKG_API void zkg_msm_set_ysum_mode(int mode) { zk::msm_set_ysum_mode(mode); }
ZKG_API void zkg_msm_set_ahead_min(int lg) { zk::msm_set_ahead_min(lg); }
ZKG_API void zkg_ntt_set_max_radix(int r) { zk::ntt_set_max_radix(r); }

ZKG_API void zkg_ntt_set_table_max(size_t entries) { zk::ntt_set_table_max(entries); }
ZKG_API void zkg_arena_set_limit(size_t bytes) { zk::arena_set_limit(bytes); }
ZKG_API int zkg_msm_last_groups(void) { return zk::msm_last_groups_read(); }
ZKG_API size_t zkg_msm_workspace_bytes(int curve, int npoints, int expo_nlimbs, int expos_mont, int host_inputs,
                                       int window_size, int groups) {
  return guard_ret<size_t>(0, [&] {
    if (curve == ZKG_BN128)
      return zk::msm_workspace_bytes<BN254>(npoints, expo_nlimbs, expos_mont != 0, host_inputs != 0, window_size,
                                            groups);
    return zk::msm_workspace_bytes<BLS381>(npoints, expo_nlimbs, expos_mont != 0, host_inputs != 0, window_size,
                                           groups);
  });
}

ZKG_API int zkg_set_devices(const int *ids, int n) { return zk::set_device_set(ids, n); }
ZKG_API int zkg_get_devices(int *ids, int cap) {
  const std::vector<int> v = zk::device_set();
  for (int i = 0; i < (int)v.size() && i < cap; i++) ids[i] = v[i];
  return (int)v.size();
}

ZKG_API void zkg_release(void) {
  guard([&] {
  int prev = 0;
  ZK_CHECK(hipGetDevice(&prev));
  DeviceGuard restore(prev);
  for (Device *d : all_devices()) {
    std::lock_guard<std::mutex> lock(d->mu);
    ZK_CHECK(hipSetDevice(d->id));
    ZK_CHECK(hipStreamSynchronize(d->stream));
    zk::ntt_release(*d);
    d->release_memory();
  }
  });
}

ZKG_API void zkg_timer_enable(int on) { timer_set_enabled(on != 0); }
ZKG_API void zkg_timer_reset(void) { timer_reset_all(); }
ZKG_API void zkg_timer_read(double *total_ms, long *launches) { timer_read_all(total_ms, launches); }

}  // extern "C"
