set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g2.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
for qd in 1 0; do
  echo "QUAD=$qd"
  for qa in 8 4 2; do
    ZK_MSM_QUAD=$qd ZK_MSM_QA=$qa ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -2 | head -1 | sed "s/^/QA=$qa /" || exit 1
  done
done
ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 14 0 2>&1 | tail -2
