// zk_msm_g2.hip -- G2 instantiations of the Pippenger MSM: the same
// pipeline over Fp2 (zk_field2.hpp); template bodies in zk_msm_impl.hpp.  Replaces
// <C>_G2_proj_MSM_{std,mont}_coeff_{proj,affine}_out (bls12_381_G2_proj.c:498-660).
#include "zk_msm_impl.hpp"

namespace zk {

template void msm_g1<BN254_G2>(int, const uint64_t *, int, const uint64_t *, bool, bool, int, uint64_t *);
template void msm_g1<BLS381_G2>(int, const uint64_t *, int, const uint64_t *, bool, bool, int, uint64_t *);

}  // namespace zk
