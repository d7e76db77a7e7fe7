set -o pipefail
cd $GRAFT_REPO_ROOT
for v in base w3 w4; do
  if [ $v = base ]; then unset ZK_LIB_PATH; else export ZK_LIB_PATH=$GRAFT_REPO_ROOT/variants/$v.so; fi
  echo "== $v"
  ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 16 2>&1 | tail -2 || exit 1
done
