set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g2.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
for lg in 20 23; do
  ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 $lg 0 2>&1 | tail -2 || exit 1
  ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bn128 $lg 0 2>&1 | tail -2 || exit 1
done
