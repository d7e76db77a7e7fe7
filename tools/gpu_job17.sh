set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g2.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
for ys in 0 1 2; do
  for qy in 8 16; do
    ZK_MSM_YSUM=$ys ZK_MSM_QY=$qy ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -2 | head -1 | sed "s/^/YS=$ys QY=$qy /" || exit 1
  done
done
ZK_MSM_YSUM=1 ZK_MSM_QY=4 ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -2 | head -1 | sed "s/^/YS=1 QY=4 /" || exit 1
for ys in 0 1 2; do
  ZK_MSM_YSUM=$ys ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bn128 20 0 2>&1 | tail -2 | head -1 | sed "s/^/BN YS=$ys /" || exit 1
done
