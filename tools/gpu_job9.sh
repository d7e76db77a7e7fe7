set -o pipefail
cd $GRAFT_REPO_ROOT
for spec in "bls12_381 10 6 7 8 9 10" "bls12_381 12 8 9 10 11 12" "bls12_381 14 10 11 12 13 14" "bls12_381 16 12 13 14 15 16" "bn128 20 14 15 16 17" "bls12_381 25 16 18 19 20"; do
  timeout -k 10 200 python tools/sweep_window.py $spec 2>&1 | grep -v "^\[zk" || { echo SWEEP FAILED $spec; exit 1; }
done
