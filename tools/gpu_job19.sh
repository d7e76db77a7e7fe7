set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g2.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 || exit 1
ZK_MSM_STITCH_SEG=0 timeout -k 10 200 python -u -m pytest tests/test_gpu_msm.py -x -q -k skewed --timeout 300 --timeout-method thread 2>&1 | tail -1 || exit 1
for seg in 0 1; do
  for sch in 4 8 16; do
    ZK_MSM_STITCH_SEG=$seg ZK_MSM_SCH=$sch ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -2 | head -1 | sed "s/^/SEG=$seg SCH=$sch /" || exit 1
  done
done
for seg in 0 1; do
  ZK_MSM_STITCH_SEG=$seg ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 14 0 2>&1 | tail -2 | head -1 | sed "s/^/2^14 SEG=$seg /" || exit 1
  ZK_MSM_STITCH_SEG=$seg ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bn128 20 0 2>&1 | tail -2 | head -1 | sed "s/^/BN SEG=$seg /" || exit 1
done
