/*
 * zkalgebra_gpu.h -- C ABI of the MI355X (gfx950) MSM / NTT library.
 *
 * Part 1 exports EXACTLY the symbols and signatures of the reference's generated C
 * that its Haskell FFI modules bind with `foreign import ccall unsafe` (drop-in
 * boundary).  Part 2 adds device-resident and helper entry points that
 * the reference does not have (benchmarking, multi-GPU sharding, input generation).
 *
 * Layouts (identical to the reference, Class/Flat.hs:81-83):
 *   u64 little-endian limbs; Fr = 4 limbs; Fp = 4 (bn128) or 6 (bls12_381) limbs;
 *   affine G1 = x || y (Montgomery Fp), infinity = all bytes 0xFF;
 *   projective G1 = X || Y || Z (x = X/Z, y = Y/Z), Jacobian = X || Y || Z (x = X/Z^2).
 * All buffers are caller-owned and are not retained after the call returns.
 * Every call is synchronous and thread-safe.  There are no error codes on the
 * reference ABI: by default, on a device error the library prints a message and aborts (the
 * reference asserts, bls12_381_G1_proj.c:518,632) -- it never falls back to a CPU path.
 * zkg_set_error_mode(1) makes errors recoverable: the failing call prints the message,
 * returns early (outputs unspecified) and zkg_last_error() reports it to the calling thread.
 *
 * Projective / Jacobian outputs are returned NORMALISED (Z = 1, or the canonical
 * infinity (0:1:0) / Jacobian (1:1:0)); they are equal as points to the reference's
 * un-normalised outputs (whose exact coordinates depend on its operation order and
 * are not reproducible).  Affine outputs are bit-identical.
 */
#ifndef ZKALGEBRA_GPU_H
#define ZKALGEBRA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZKG_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------
 * Part 1: reference symbols.  <C> in {bn128, bls12_381}.
 * ---------------------------------------------------------------------------- */

/* MSM, G1, homogeneous projective.
 *   lib/cbits/curves/g1/proj/bls12_381_G1_proj.h:43-46 (bn128_G1_proj.h same lines)
 *   mont_coeff_proj_out  <- Haskell `msm`    (lib/src/ZK/Algebra/Curves/<C>/G1/Proj.hs:229,245)
 *   std_coeff_proj_out   <- Haskell `msmStd` (G1/Proj.hs:228,262)
 *   _affine_out          <- bls12_381_G1_proj.c:654-670
 *   expos: npoints x expo_nlimbs u64 (Montgomery Fr for mont_coeff, plain integers for
 *   std_coeff, used verbatim -- no reduction mod r).  expo_nlimbs: any >= 1; std scalars
 *   are 64*expo_nlimbs-bit integers (G1_proj.c:511,552); for mont the first min(nl,4) limbs
 *   of each row are the Montgomery value (the reference's result is undefined for nl != 4).
 *   grps : npoints affine points.  tgt: 3*NP (proj) or 2*NP (affine) u64. */
ZKG_API void bn128_G1_proj_MSM_mont_coeff_proj_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bn128_G1_proj_MSM_std_coeff_proj_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bn128_G1_proj_MSM_mont_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bn128_G1_proj_MSM_std_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
/* bn128_G1_proj.c:506 -- window_size is honoured as the GPU window (clamped to [4,24]) */
ZKG_API void bn128_G1_proj_MSM_std_coeff_proj_out_variable(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs, int window_size);

ZKG_API void bls12_381_G1_proj_MSM_mont_coeff_proj_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G1_proj_MSM_std_coeff_proj_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G1_proj_MSM_mont_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G1_proj_MSM_std_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
/* bls12_381_G1_proj.c:507 */
ZKG_API void bls12_381_G1_proj_MSM_std_coeff_proj_out_variable(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs, int window_size);

/* MSM, G1, Jacobian output (secondary; bls12_381_G1_jac.h:43-46, bound by G1/Jac.hs:225-226) */
ZKG_API void bn128_G1_jac_MSM_std_coeff_jac_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bn128_G1_jac_MSM_mont_coeff_jac_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bn128_G1_jac_MSM_std_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bn128_G1_jac_MSM_mont_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G1_jac_MSM_std_coeff_jac_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G1_jac_MSM_mont_coeff_jac_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G1_jac_MSM_std_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G1_jac_MSM_mont_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);

/* NTT over Fr, natural order in/out, 2^m elements, gen = Montgomery generator of the
 * order-2^m subgroup (Haskell passes fftSubgroupGen).  Out-of-place.
 *   lib/cbits/curves/poly/mont/bls12_381_poly_mont.h:27-28 (bn128_poly_mont.h same)
 *   forward <- Haskell forwardNTT (lib/src/ZK/Algebra/Curves/<C>/Poly.hs:397,409)
 *   inverse <- Haskell inverseNTT (Poly.hs:398,421) */
ZKG_API void bn128_poly_mont_ntt_forward(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt);
ZKG_API void bn128_poly_mont_ntt_inverse(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt);
ZKG_API void bls12_381_poly_mont_ntt_forward(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt);
ZKG_API void bls12_381_poly_mont_ntt_inverse(int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt);

/* MSM on G2: the twist over Fp2 = Fp[u]/(u^2+1), same conventions
 * as G1 with NP doubled (Fp2 element = c0 || c1); affine infinity = all-0xFF.
 *   bls12_381_G2_proj.h:43-46 (bn128_G2_proj.h same lines), bound by G2/Proj.hs */
ZKG_API void bn128_G2_proj_MSM_std_coeff_proj_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bn128_G2_proj_MSM_mont_coeff_proj_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bn128_G2_proj_MSM_std_coeff_affine_out (int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bn128_G2_proj_MSM_mont_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G2_proj_MSM_std_coeff_proj_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G2_proj_MSM_mont_coeff_proj_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G2_proj_MSM_std_coeff_affine_out (int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);
ZKG_API void bls12_381_G2_proj_MSM_mont_coeff_affine_out(int npoints, const uint64_t *expos, const uint64_t *grps, uint64_t *tgt, int expo_nlimbs);

/* G1 batch conversions and the group (curve) FFT.
 *   bls12_381_G1_proj.h:9-10, 48-49 (bn128_G1_proj.h same lines); Haskell batchFromAffine /
 *   batchToAffine (G1/Proj.hs:409-430), forwardFFT / inverseFFT = curveFFT / curveIFFT
 *   (G1/Proj.hs:270-294).  Projective outputs of the FFT are normalised, like the
 *   reference's (bls12_381_G1_proj.c:719, 785). */
ZKG_API void bn128_G1_proj_batch_from_affine( int N, const uint64_t *src , uint64_t *tgt );
ZKG_API void bn128_G1_proj_batch_to_affine  ( int N, const uint64_t *src , uint64_t *tgt );
ZKG_API void bn128_G1_proj_fft_forward( int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt );
ZKG_API void bn128_G1_proj_fft_inverse( int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_G1_proj_batch_from_affine( int N, const uint64_t *src , uint64_t *tgt );
ZKG_API void bls12_381_G1_proj_batch_to_affine  ( int N, const uint64_t *src , uint64_t *tgt );
ZKG_API void bls12_381_G1_proj_fft_forward( int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_G1_proj_fft_inverse( int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt );

/* Jacobian twins (round 6): bls12_381_G1_jac.h:9-10, 48-49 (bn128_G1_jac.h same lines); bound by the
 * Jacobian G1 instance -- batchFromAffine / batchToAffine (G1/Jac.hs:374-389; Curve.msm on Jac.G1 is
 * msmJac cs gs = msm cs (batchToAffine gs), Jac.hs:188, 220) and forwardFFT / inverseFFT = curveFFT /
 * curveIFFT (Jac.hs:189-190, 264-291).  Conventions: affine infinity -> (1 : 1 : 0)
 * (bls12_381_G1_jac.c:108-116, 183-187); Z = 0 -> all-0xFF (to_affine, :120-125); FFT outputs
 * normalised (x : y : 1), infinity (0 : 1 : 0) (jac normalize, :62-67, applied at :773-775, :835-837). */
ZKG_API void bn128_G1_jac_batch_from_affine( int N, const uint64_t *src , uint64_t *tgt );
ZKG_API void bn128_G1_jac_batch_to_affine  ( int N, const uint64_t *src , uint64_t *tgt );
ZKG_API void bn128_G1_jac_fft_forward( int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt );
ZKG_API void bn128_G1_jac_fft_inverse( int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_G1_jac_batch_from_affine( int N, const uint64_t *src , uint64_t *tgt );
ZKG_API void bls12_381_G1_jac_batch_to_affine  ( int N, const uint64_t *src , uint64_t *tgt );
ZKG_API void bls12_381_G1_jac_fft_forward( int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_G1_jac_fft_inverse( int m, const uint64_t *gen, const uint64_t *src, uint64_t *tgt );

/* Fr vector operations around the NTT.  <C> in {bn128, bls12_381}.
 *   lib/cbits/curves/array/mont/bls12_381_arr_mont.h:3-48 (bn128_arr_mont.h same lines),
 *   bound by Haskell ZK.Algebra.Curves.<C>.Array (Array.hs:108-352).
 *   n elements of Montgomery Fr (4 u64 each); coefficients are single elements.
 *   inv / div follow the reference's batch inversion (Fr_mont.c:258-285): if ANY
 *   (divisor) element is zero, EVERY output element is zero.  n == 0 is a no-op (the
 *   reference asserts n >= 1 in batch_inv). */
ZKG_API uint8_t bn128_arr_mont_is_valid ( int n, const uint64_t *src );
ZKG_API uint8_t bn128_arr_mont_is_zero  ( int n, const uint64_t *src );
ZKG_API uint8_t bn128_arr_mont_is_one   ( int n, const uint64_t *src );
ZKG_API uint8_t bn128_arr_mont_is_equal ( int n, const uint64_t *src1, const uint64_t *src2 );
ZKG_API void bn128_arr_mont_set_zero ( int n, uint64_t *tgt );
ZKG_API void bn128_arr_mont_set_one  ( int n, uint64_t *tgt );
ZKG_API void bn128_arr_mont_set_const( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bn128_arr_mont_copy     ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bn128_arr_mont_from_std ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bn128_arr_mont_to_std   ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bn128_arr_mont_append( int n1, int n2, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bn128_arr_mont_neg ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bn128_arr_mont_add ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bn128_arr_mont_sub ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bn128_arr_mont_sqr ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bn128_arr_mont_mul ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bn128_arr_mont_inv ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bn128_arr_mont_div ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bn128_arr_mont_neg_inplace ( int n, uint64_t *tgt );
ZKG_API void bn128_arr_mont_add_inplace ( int n, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bn128_arr_mont_sub_inplace ( int n, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bn128_arr_mont_sqr_inplace ( int n, uint64_t *tgt );
ZKG_API void bn128_arr_mont_mul_inplace ( int n, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bn128_arr_mont_inv_inplace ( int n, uint64_t *tgt );
ZKG_API void bn128_arr_mont_div_inplace ( int n, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bn128_arr_mont_sub_inplace_reverse ( int n, uint64_t *tgt, const uint64_t *src1 );
ZKG_API void bn128_arr_mont_mul_add ( int n, const uint64_t *src1, const uint64_t *src2, const uint64_t *src3, uint64_t *tgt );
ZKG_API void bn128_arr_mont_mul_sub ( int n, const uint64_t *src1, const uint64_t *src2, const uint64_t *src3, uint64_t *tgt );
ZKG_API void bn128_arr_mont_dot_prod ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bn128_arr_mont_powers ( int n, const uint64_t *coeffA, const uint64_t *coeffB, uint64_t *tgt );
ZKG_API void bn128_arr_mont_scale ( int n, const uint64_t *coeff, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bn128_arr_mont_scale_inplace ( int n, const uint64_t *coeff, uint64_t *tgt );
ZKG_API void bn128_arr_mont_Ax_plus_y ( int n, const uint64_t *coeffA, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bn128_arr_mont_Ax_plus_y_inplace ( int n, const uint64_t *coeffA, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bn128_arr_mont_Ax_plus_By ( int n, const uint64_t *coeffA, const uint64_t *coeffB, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bn128_arr_mont_Ax_plus_By_inplace ( int n, const uint64_t *coeffA, const uint64_t *coeffB, uint64_t *tgt, const uint64_t *src2 );
/* division by the vanishing polynomial x^expo_n - eta (bls12_381_poly_mont.c:317-413) */
ZKG_API void bn128_poly_mont_div_by_vanishing ( int n1, const uint64_t *src1, int expo_n, const uint64_t *eta, int nquot, uint64_t *quot, int nrem, uint64_t *rem );
ZKG_API uint8_t bn128_poly_mont_quot_by_vanishing( int n1, const uint64_t *src1, int expo_n, const uint64_t *eta, int nquot, uint64_t *quot );

ZKG_API uint8_t bls12_381_arr_mont_is_valid ( int n, const uint64_t *src );
ZKG_API uint8_t bls12_381_arr_mont_is_zero  ( int n, const uint64_t *src );
ZKG_API uint8_t bls12_381_arr_mont_is_one   ( int n, const uint64_t *src );
ZKG_API uint8_t bls12_381_arr_mont_is_equal ( int n, const uint64_t *src1, const uint64_t *src2 );
ZKG_API void bls12_381_arr_mont_set_zero ( int n, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_set_one  ( int n, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_set_const( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_copy     ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_from_std ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_to_std   ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_append( int n1, int n2, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_neg ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_add ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_sub ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_sqr ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_mul ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_inv ( int n, const uint64_t *src, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_div ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_neg_inplace ( int n, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_add_inplace ( int n, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bls12_381_arr_mont_sub_inplace ( int n, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bls12_381_arr_mont_sqr_inplace ( int n, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_mul_inplace ( int n, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bls12_381_arr_mont_inv_inplace ( int n, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_div_inplace ( int n, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bls12_381_arr_mont_sub_inplace_reverse ( int n, uint64_t *tgt, const uint64_t *src1 );
ZKG_API void bls12_381_arr_mont_mul_add ( int n, const uint64_t *src1, const uint64_t *src2, const uint64_t *src3, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_mul_sub ( int n, const uint64_t *src1, const uint64_t *src2, const uint64_t *src3, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_dot_prod ( int n, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_powers ( int n, const uint64_t *coeffA, const uint64_t *coeffB, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_scale ( int n, const uint64_t *coeff, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_scale_inplace ( int n, const uint64_t *coeff, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_Ax_plus_y ( int n, const uint64_t *coeffA, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_Ax_plus_y_inplace ( int n, const uint64_t *coeffA, uint64_t *tgt, const uint64_t *src2 );
ZKG_API void bls12_381_arr_mont_Ax_plus_By ( int n, const uint64_t *coeffA, const uint64_t *coeffB, const uint64_t *src1, const uint64_t *src2, uint64_t *tgt );
ZKG_API void bls12_381_arr_mont_Ax_plus_By_inplace ( int n, const uint64_t *coeffA, const uint64_t *coeffB, uint64_t *tgt, const uint64_t *src2 );
/* division by the vanishing polynomial x^expo_n - eta (bls12_381_poly_mont.c:317-413) */
ZKG_API void bls12_381_poly_mont_div_by_vanishing ( int n1, const uint64_t *src1, int expo_n, const uint64_t *eta, int nquot, uint64_t *quot, int nrem, uint64_t *rem );
ZKG_API uint8_t bls12_381_poly_mont_quot_by_vanishing( int n1, const uint64_t *src1, int expo_n, const uint64_t *eta, int nquot, uint64_t *quot );

/* ------------------------------------------------------------------------------
 * Part 2: extensions (not in the reference).  curve: 0 = bn128, 1 = bls12_381.
 * ---------------------------------------------------------------------------- */
#define ZKG_BN128 0
#define ZKG_BLS12_381 1

ZKG_API const char *zkg_version(void);
/* error channel: mode 0 = print and abort on a device error (default, reference-like),
 * 1 = print, return from the failing call (outputs unspecified) and record the message;
 * zkg_last_error returns 1 and copies the calling thread's last message (cleared), else 0 */
ZKG_API void zkg_set_error_mode(int mode);
ZKG_API int zkg_last_error(char *msg, size_t cap);
ZKG_API int zkg_device_count(void);
ZKG_API void zkg_set_device(int device);           /* binds the calling thread */
ZKG_API void *zkg_device_malloc(size_t bytes);
ZKG_API void zkg_device_free(void *ptr);
ZKG_API void zkg_memcpy_htod(void *dst, const void *src, size_t bytes);
ZKG_API void zkg_memcpy_dtoh(void *dst, const void *src, size_t bytes);
ZKG_API void zkg_device_synchronize(void);

/* Device set of the host-buffer MSM entry points (G1 and G2, every Part-1 MSM symbol): the
 * pairs are split into n contiguous chunks, chunk k computed on device ids[k] (copying only its
 * own chunk over that device's PCIe link), the partial sums added in list order.  A device may
 * be listed more than once (one stream / arena per occurrence).  n <= 1: the calling thread's
 * device only (the default; also set by the environment variable ZKG_DEVICES = "all" or
 * "0,1,..." at first use).  A one-entry set pins the host-buffer MSMs (and NTTs) to that device.
 * The host-buffer NTT symbols (2^16 points and up) compute on the calling thread's device when the
 * set lists it, else on the first listed device, and move chunk k of the input / output over
 * listed device k's PCIe link (peer copies over xGMI).  In a one-process-per-GPU job (bench.py
 * --gpus N, or any RCCL job) leave the set empty: every rank would otherwise push its host copies
 * through every GPU's link.  Returns 0, or -1 (set unchanged) for an invalid id.  The
 * device-resident zkg_*_device calls always run on the calling thread's device. */
ZKG_API int zkg_set_devices(const int *ids, int n);
ZKG_API int zkg_get_devices(int *ids, int cap);  /* returns the set's size; copies min(size, cap) ids */

/* Frees every device buffer the library holds (per-device working-set arenas, pinned staging,
 * cached NTT twiddle tables) after waiting for the calls in flight; later calls re-allocate. */
ZKG_API void zkg_release(void);

/* Multi-GPU exchange owned by the library (RCCL over xGMI, linked from /opt/rocm): one
 * communicator per process, one process per GPU.  The reference is single-device
 * (bls12_381_G1_proj.c:630-644); these calls shard its MSM by contiguous chunk of the pairs.
 * Rendezvous is the caller's: rank 0 writes the 128-byte id with zkg_comm_unique_id, every rank
 * calls zkg_comm_init with it on the device it will use (zkg_set_device first).  Every rank must
 * make the same sequence of zkg_comm_* / *_sharded calls.  Return 0 on success, -1 on misuse
 * (no communicator, bad arguments), else the RCCL error code (a message goes to stderr). */
#define ZKG_COMM_ID_BYTES 128
ZKG_API int zkg_comm_unique_id(void *out);
ZKG_API int zkg_comm_init(int rank, int world, const void *unique_id);
ZKG_API int zkg_comm_destroy(void);
ZKG_API int zkg_comm_rank(void);   /* -1 without a communicator */
ZKG_API int zkg_comm_world(void);  /* 0 without a communicator */
/* ncclAllGather of `bytes` host bytes per rank into recv (world * bytes, rank order) */
ZKG_API int zkg_comm_allgather(const void *send, void *recv, size_t bytes);
ZKG_API int zkg_comm_barrier(void);
ZKG_API int zkg_comm_max_f64(double *x);  /* in place: the maximum over ranks */
/* every rank passes `count` projective G1 partials (3 NP u64 each, host); all ranks receive
 * the normalised sum of the world * count partials, added in (rank, index) order */
ZKG_API int zkg_g1_comm_sum_partials(int curve, const uint64_t *partials, int count, uint64_t *tgt_proj);
/* Device-resident sharded MSM: this rank's chunk (npoints_local pairs, DEVICE pointers) is
 * computed on the communicator's device as `local_shards` contiguous sub-chunks, the
 * world * local_shards partial sums are all-gathered by ncclAllGather on the library's stream and
 * added in (rank, sub-chunk) order; tgt_proj (HOST, 3 NP u64) receives the normalised total on
 * every rank.  local_shards must be the same on every rank (1 = one partial per rank). */
ZKG_API int zkg_g1_msm_device_sharded(int curve, int npoints_local, const uint64_t *d_expos, int expo_nlimbs,
                                      int expos_mont, const uint64_t *d_grps, int window_size, int local_shards,
                                      uint64_t *tgt_proj);

/* device-resident MSM: d_expos / d_grps are DEVICE pointers (already in HBM);
 * tgt_proj is a HOST buffer of 3*NP u64 receiving the normalised projective sum. */
ZKG_API void zkg_g1_msm_device(int curve, int npoints, const uint64_t *d_expos, int expo_nlimbs, int expos_mont,
                               const uint64_t *d_grps, uint64_t *tgt_proj, int window_size);
/* device-resident G2 MSM (same contract as zkg_g1_msm_device; tgt_proj = 3 Fp2 elements) */
ZKG_API void zkg_g2_msm_device(int curve, int npoints, const uint64_t *d_expos, int expo_nlimbs, int expos_mont,
                               const uint64_t *d_grps, uint64_t *tgt_proj, int window_size);
/* device-resident NTT: d_src / d_tgt DEVICE pointers; gen on the host */
ZKG_API void zkg_ntt_device(int curve, int inverse, int m, const uint64_t *gen, const uint64_t *d_src, uint64_t *d_tgt);

/* device-resident Fr vector ops: d_* are DEVICE pointers, kA/kB and dot's tgt HOST.
 * op codes: 0 neg, 1 add, 2 sub, 3 sub_rev (b - a), 4 sqr, 5 mul, 6 mul_add, 7 mul_sub,
 * 8 scale (kA a), 9 Ax_plus_y, 10 Ax_plus_By, 11 from_std, 12 to_std, 13 copy,
 * 14 set_const (kA), 15 inv, 16 div (a / b) */
ZKG_API void zkg_arr_op_device(int curve, int op, int n, const uint64_t *d_a, const uint64_t *d_b,
                               const uint64_t *d_c, const uint64_t *kA, const uint64_t *kB, uint64_t *d_tgt);
ZKG_API void zkg_arr_dot_device(int curve, int n, const uint64_t *d_a, const uint64_t *d_b, uint64_t *tgt);
ZKG_API void zkg_arr_powers_device(int curve, int n, const uint64_t *kA, const uint64_t *kB, uint64_t *d_tgt);
ZKG_API int zkg_poly_div_by_vanishing_device(int curve, int n1, const uint64_t *d_src, int expo_n,
                                             const uint64_t *eta, int nquot, uint64_t *d_quot, int nrem,
                                             uint64_t *d_rem);

/* device-resident G1 group FFT / batch_to_affine (d_* DEVICE pointers, gen on the host) */
ZKG_API void zkg_g1_fft_device(int curve, int inverse, int m, const uint64_t *gen, const uint64_t *d_src,
                               uint64_t *d_tgt);
ZKG_API void zkg_g1_batch_to_affine_device(int curve, int n, const uint64_t *d_src, uint64_t *d_tgt);
/* the same on Jacobian rows (the <C>_G1_jac_fft_* / _batch_to_affine conventions above) */
ZKG_API void zkg_g1_jac_fft_device(int curve, int inverse, int m, const uint64_t *gen, const uint64_t *d_src,
                                   uint64_t *d_tgt);
ZKG_API void zkg_g1_jac_batch_to_affine_device(int curve, int n, const uint64_t *d_src, uint64_t *d_tgt);

/* host helpers on G1 (projective, reference Montgomery form) */
ZKG_API void zkg_g1_proj_add(int curve, const uint64_t *a, const uint64_t *b, uint64_t *out);
ZKG_API void zkg_g1_proj_normalize(int curve, const uint64_t *a, uint64_t *out);
ZKG_API void zkg_g1_proj_to_affine(int curve, const uint64_t *a, uint64_t *out);

/* deterministic synthetic inputs (spec: zikkurat-algebra_amd/csrc/zk_gen.cpp) */
ZKG_API void zkg_gen_fr(int curve, uint64_t seed, int64_t start, int64_t count, uint64_t *out);
ZKG_API void zkg_gen_g1_points(int curve, uint64_t seed, int64_t start, int64_t count, uint64_t *out);
/* Montgomery generator of the order-2^m subgroup: fftDomain gen^(2^(M-m))
 * (Class/FFT.hs:60-66; BLS12_381/Fr/Mont.hs:145-151, BN128/Fr/Mont.hs:146-148) */
ZKG_API void zkg_fft_generator(int curve, int m, uint64_t *out);

/* MSM window heuristic used when window_size is not given */
ZKG_API int zkg_msm_default_window(int npoints);
/* the window a G1 MSM of `npoints` pairs runs with by default on `curve` (ZKG_BN128 /
 * ZKG_BLS12_381) for its scalar form (Montgomery Fr, or std integers of expo_nlimbs limbs):
 * zkg_msm_default_window's table, made curve-aware where a full top window measured faster */
ZKG_API int zkg_msm_window(int curve, int npoints, int expo_nlimbs, int expos_mont);

/* per-phase HIP-event profile of every MSM call, printed to stderr (diagnostics) */
ZKG_API void zkg_msm_profile(int on);
/* test hook: cap on the sorted (window, point) entries one MSM pipeline pass handles
 * (default and maximum 2^30; 0 restores it).  Larger MSMs run in window groups. */
ZKG_API void zkg_msm_set_group_limit(size_t entries);
/* test hook: the G1 MSM's Y-sum kernel -- -1: by size (k_ysum3, two waves per SIMD, when the
 * Y-sum lanes fill several rounds of the chip: c = 20 from 2^23 pairs), 0: always k_ysum2,
 * 1: always k_ysum3 (block-level shapes, c >= 12) */
ZKG_API void zkg_msm_set_ysum_mode(int mode);
/* test hook: device-resident G1/G2 MSMs of at least 2^lg pairs whose windows fit one pass run as
 * two window groups with both bucket sorts on a second stream (B's beside A's accumulation);
 * lg = 0 disables it, lg < 0 restores the default: from 2^23 pairs (or the environment's
 * ZK_MSM_AHEAD_MIN) for the curves whose accumulation leaves VGPRs for the sort (BN128 G1), off
 * otherwise */
ZKG_API void zkg_msm_set_ahead_min(int lg);
/* test hook: NTT pass split -- 12: two passes of 2^9..2^12-point DFTs (4096-element tiles) for
 * every 2^17..2^24; 8: passes of <= 2^8-point DFTs only; 0: the default (two passes at 2^20 only) */
ZKG_API void zkg_ntt_set_max_radix(int r);
/* test hook: inter-pass twiddle table entries above which an NTT pass computes its twiddles on
 * the fly (default 2^25, i.e. only transforms of 2^26 and more; 0 restores it) */
ZKG_API void zkg_ntt_set_table_max(size_t entries);
/* test hook: device bytes one working-set arena may hold (0: unlimited), to exercise the
 * out-of-memory degrade path (smaller MSM window groups) */
ZKG_API void zkg_arena_set_limit(size_t bytes);
/* window groups (pipeline passes) of the most recent single-device MSM pass */
ZKG_API int zkg_msm_last_groups(void);
/* 1 when the most recent group FFT (G1 fft / ifft) ran the GLV stages (every input point in the
 * order-r subgroup), 0 when it ran the integer-scalar stages */
ZKG_API int zkg_g1_fft_last_glv(void);
/* the GLV-stage plan of a 2^m group FFT (zk_g1ext.hip radix_plan): writes the bits of each
 * Stockham radix-2^b stage into bits[0..cap) and returns the stage count (0: the fused radix-2
 * stages, m of them); zkg_g1_fft_radix_products(b) = GLV lane-pair products per group of 2^b points */
ZKG_API int zkg_g1_fft_plan(int curve, int m, int *bits, int cap);
ZKG_API int zkg_g1_fft_radix_products(int b);
/* device bytes of one G1 MSM's working set (the arena it reserves) with its windows split into
 * `groups` passes; window_size <= 0: the default window */
ZKG_API size_t zkg_msm_workspace_bytes(int curve, int npoints, int expo_nlimbs, int expos_mont, int host_inputs,
                                       int window_size, int groups);

/* timing probe of the dominant kernel (MSM bucket accumulation / NTT pass chain),
 * measured with HIP events on each device's own stream; read sums over devices */
ZKG_API void zkg_timer_enable(int on);
ZKG_API void zkg_timer_reset(void);
ZKG_API void zkg_timer_read(double *total_ms, long *launches);

#ifdef __cplusplus
}
#endif
#endif /* ZKALGEBRA_GPU_H */
