// zk_msm.hpp -- C++ interface of the device MSM (used by the C ABI layer)
#pragma once
#include <stddef.h>
#include <stdint.h>
#include "zk_curve.hpp"
#include "zk_host.hpp"

namespace zk {

template <class C> struct HostOf;
template <> struct HostOf<BN254> {
  using Fp = zkh::BN_Fp;
  using Fr = zkh::BN_Fr;
  static void b3(zkh::Fe<Fp> &r) { const uint64_t v[] = ZK_BN128_B3_FP64; memcpy(r.v, v, sizeof r.v); }
};
template <> struct HostOf<BLS381> {
  using Fp = zkh::BLS_Fp;
  using Fr = zkh::BLS_Fr;
  static void b3(zkh::Fe<Fp> &r) { const uint64_t v[] = ZK_BLS12_381_B3_FP64; memcpy(r.v, v, sizeof r.v); }
};

template <> struct HostOf<BN254_G2> {
  using Fp = zkh::HF2<zkh::BN_Fp>;
  using Fr = zkh::BN_Fr;
};
template <> struct HostOf<BLS381_G2> {
  using Fp = zkh::HF2<zkh::BLS_Fp>;
  using Fr = zkh::BLS_Fr;
};

int msm_default_window(int n);
int msm_default_window_bits(int n, int bits);  // G1: the window for `bits`-bit scalars (curve-aware)
void msm_set_profile(int on);  // per-phase event timing of every MSM call, printed to stderr
void msm_set_group_limit(size_t entries);  // test hook: max sorted entries per pipeline pass (0: default)
void msm_set_ysum_mode(int mode);          // test hook: G1 Y-sum kernel (-1 auto, 0 k_ysum2, 1 k_ysum3)
void msm_set_ahead_min(int lg);           // test hook: sort-ahead from 2^lg device-resident pairs (0 off, < 0 default)
int msm_last_groups_read();  // window groups of the most recent msm_run (degrade-path tests)

// scalars: n x nl u64 (Montgomery Fr if mont, else plain integers of 64 nl bits, any nl >= 1)
// points : n x 2*NP64 u64 affine Montgomery (all-0xFF = infinity)
// out    : 3*NP64 u64 projective, reference Montgomery form, NOT normalised
// host_inputs: pointers are host memory (staged by the call) vs device-resident
// device bytes of one pass's working set, windows split into `groups` passes
template <class C>
size_t msm_workspace_bytes(int n, int nl, bool mont, bool host_inputs, int window, int groups);
template <class C>
void msm_g1(int n, const uint64_t *scalars, int nl, const uint64_t *points, bool host_inputs, bool mont,
            int window, uint64_t *out_proj);

}  // namespace zk
