set -o pipefail
cd $GRAFT_REPO_ROOT
for sch in 4 8; do for spec in 2 3 4; do
  for cfg in "bls12_381 20" "bn128 20" "bls12_381 14" "bls12_381 17"; do
    ZK_MSM_SCH=$sch ZK_MSM_SPEC=$spec timeout -k 10 120 python tools/sweep_window.py $cfg 0 2>&1 | tail -1 | sed "s/^/SCH=$sch SPEC=$spec /" || exit 1
  done
done; done
