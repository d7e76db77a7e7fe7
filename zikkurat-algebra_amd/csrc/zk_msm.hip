// zk_msm.hip -- G1 instantiations of the Pippenger MSM (template bodies: zk_msm_impl.hpp)
#include "zk_msm_impl.hpp"

namespace zk {

int msm_default_window(int n) {
  // GPU window, from window x chunk sweeps on MI355X (profiles/r01_v5_window_sweep_*.txt,
  // profiles/r03l_small_window_chunk_sweep.txt): 2^10 -> 9, 2^11..2^12 -> 10, 2^13..2^16 -> 13,
  // 2^17..2^24 -> 16, 2^25..2^26 -> 20.  (The reference uses round(log2 n - 3.5), G1_proj.c:600;
  // the result does not depend on the choice.)  The accumulation's cost falls with c (fewer
  // windows) while the bucket reduction's rises with it (W * 2^(c-1) buckets); at the small sizes
  // the odd c = 13 also gives Y-sum / job-sum shapes that fill whole blocks (2^14: 0.77 -> 0.62 ms,
  // 2^15: 0.94 -> 0.70, 2^17: 1.36 -> 0.97 ms against the round-2 table c = lg n - 3).
  if (n <= 1) return 4;
  const int lg = ilog2((unsigned)n);
  int c;
  if (lg <= 10) c = lg - 1;
  else if (lg <= 12) c = 10;
  else if (lg <= 16) c = 13;
  else if (lg <= 24) c = 16;
  else c = 20;
  if (c < 4) c = 4;
  if (c > 20) c = 20;
  return c;
}

// The G1 window for `bits`-bit scalars: the table above (swept on BLS12-381's 255-bit Fr), except
// where a wider window leaves a full top window and measured faster (profiles/r04z_*, r04za_*):
// BN128 (254 bits = 14 x 17 + 16) takes c = 17 from 2^20 to 2^24 (2^20 2.05 -> 1.97 ms, 2^23
// 14.0 -> 13.0, 2^24 27.7 -> 26.7), BLS12-381 (255 = 12 x 20 + 15) c = 20 at 2^24 (45.7 -> 41.8 ms)
// and, since the two-wave Y sums (k_ysum3), at 2^23 (24.0 -> 23.7 ms; profiles/r05c_*).
// Windows whose top window holds only the carry (BLS12-381 c = 17 / 19 / 21) put ~n/2 entries in one
// bucket and lose badly (2^26 c = 21: 302 vs 150 ms).
int msm_default_window_bits(int n, int bits) {
  const int c = msm_default_window(n);
  if (n <= 1) return c;
  const int lg = ilog2((unsigned)n);
  if (bits == 254 && lg >= 20 && lg <= 24) return 17;
  if (bits == 255 && (lg == 23 || lg == 24)) return 20;
  return c;
}

void msm_set_ysum_mode(int mode) { ysum_mode().store(mode < 0 ? -1 : (mode ? 1 : 0)); }
void msm_set_ahead_min(int lg) { msm_ahead_min().store(lg < 0 ? -1 : lg); }
void msm_set_profile(int on) { msm_profile_flag().store(on); }
int msm_last_groups_read() { return msm_last_groups().load(); }
void msm_set_group_limit(size_t entries) {
  msm_group_limit().store(entries == 0 || entries > MSM_MAX_GROUP_ENTRIES ? MSM_MAX_GROUP_ENTRIES : entries);
}

template size_t msm_workspace_bytes<BN254>(int, int, bool, bool, int, int);
template size_t msm_workspace_bytes<BLS381>(int, int, bool, bool, int, int);
template void msm_g1<BN254>(int, const uint64_t *, int, const uint64_t *, bool, bool, int, uint64_t *);
template void msm_g1<BLS381>(int, const uint64_t *, int, const uint64_t *, bool, bool, int, uint64_t *);

}  // namespace zk
