# r04k: window sweep for 2^17..2^19 (the Y sums cost the same 0.32 ms at c = 16 from 2^18 to 2^20)
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for lg in 17 18 19 20; do
    timeout -k 10 200 python -u tools/sweep_window.py bls12_381 $lg 13 14 15 16 2>&1 | grep -v amdgpu.ids || exit 1
  done
  for lg in 17 18 19 20; do
    timeout -k 10 200 python -u tools/sweep_window.py bn128 $lg 13 14 15 16 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
