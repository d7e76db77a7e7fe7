// zk_msm_g2_bn.hip -- BN128 G2 instantiation of the Pippenger MSM: the same
// pipeline over Fp2 (zk_field2.hpp); template bodies in zk_msm_impl.hpp.  Replaces
// bn128_G2_proj_MSM_{std,mont}_coeff_{proj,affine}_out (bn128_G2_proj.c, the layout of
// bls12_381_G2_proj.c:498-660).  One curve per unit so the two (long) compiles run in parallel.
#include "zk_msm_impl.hpp"

namespace zk {

template void msm_g1<BN254_G2>(int, const uint64_t *, int, const uint64_t *, bool, bool, int, uint64_t *);

}  // namespace zk
