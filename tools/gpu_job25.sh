set -o pipefail
cd $GRAFT_REPO_ROOT
for spec in 3 4; do
  for cfg in "bls12_381 12" "bls12_381 14" "bls12_381 16" "bls12_381 17" "bls12_381 18" "bls12_381 20" "bn128 20" "bls12_381 22" "bn128 23"; do
    ZK_MSM_SPEC=$spec ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py $cfg 0 2>&1 | tail -2 | sed "s/^/SPEC=$spec /" || exit 1
  done
done
