set -o pipefail
cd $GRAFT_REPO_ROOT
for spec in "bls12_381 12 0" "bls12_381 16 0"; do
  ZK_MSM_PROFILE=1 timeout -k 10 200 python tools/sweep_window.py $spec 2>&1 | tail -2 || { echo FAILED; exit 1; }
done
