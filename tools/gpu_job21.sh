set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g2.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 || exit 1
ZK_MSM_OFFSCAN=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py -x -q -k "skewed or random" --timeout 300 --timeout-method thread 2>&1 | tail -1 || exit 1
for off in 0 1; do
  ZK_MSM_OFFSCAN=$off ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -2 | sed "s/^/OFF=$off /" || exit 1
done
ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 14 0 2>&1 | tail -2 || exit 1
ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bn128 20 0 2>&1 | tail -2 || exit 1
timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -1 || exit 1
