#!/bin/bash
# Static instruction counts of the dominant kernels' hot loops (CPU, no GPU needed):
#   bash tools/isa_profile.sh TAG   -> profiles/TAG_isa_k_accum_{bls12_381,bn128}.json
# Compiles the MSM translation unit with --save-temps into a scratch dir and runs
# tools/isa_count.py on the gfx950 assembly.  bench.py prices its VALU roofline from these
# files (issue slots per bucket mixed add) and the measured issue ceiling.
set -e
TAG=${1:?tag}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cd "$T"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --save-temps -c "$ROOT/zikkurat-algebra_amd/csrc/zk_msm.hip" -o zk_msm.o
S=zk_msm-hip-amdgcn-amd-amdhsa-gfx950.s
python3 "$ROOT/tools/isa_count.py" $S 'k_accumINS_6BLS381' --json "$ROOT/profiles/${TAG}_isa_k_accum_bls12_381.json" \
  --note "one lazy XYZZ mixed add (madd) of an affine point into a bucket accumulator, BLS12-381 Fp"
python3 "$ROOT/tools/isa_count.py" $S 'k_accumINS_5BN254' --json "$ROOT/profiles/${TAG}_isa_k_accum_bn128.json" \
  --note "one XYZZ mixed add (madd) of an affine point into a bucket accumulator, BN128 Fp"
rm -rf "$T"
