// zk_msm.hip -- G1 instantiations of the Pippenger MSM (template bodies: zk_msm_impl.hpp)
#include "zk_msm_impl.hpp"

namespace zk {

int msm_default_window(int n) {
  // GPU window: more buckets are cheap on a wide device, fewer windows save
  // accumulation work.  (The reference uses round(log2 n - 3.5), G1_proj.c:600; the
  // result does not depend on the choice.)
  if (n <= 1) return 4;
  int lg = ilog2((unsigned)n);
  int c = lg - 4;
  if (c < 4) c = 4;
  if (c > 20) c = 20;
  return c;
}


template void msm_g1<BN254>(int, const uint64_t *, int, const uint64_t *, bool, bool, int, uint64_t *);
template void msm_g1<BLS381>(int, const uint64_t *, int, const uint64_t *, bool, bool, int, uint64_t *);

}  // namespace zk
