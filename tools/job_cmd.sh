# r04za: BN128 c = 16 vs 17 at 2^19..2^24; BLS12-381 c = 16 vs 20 at 2^22..2^24
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for lg in 19 20 21 22 23 24; do
  timeout -k 10 200 python -u tools/sweep_window.py bn128 $lg 16 17 2>&1 | grep -v amdgpu.ids || exit 1
done
for lg in 22 23 24; do
  timeout -k 10 300 python -u tools/sweep_window.py bls12_381 $lg 16 20 2>&1 | grep -v amdgpu.ids || exit 1
done
