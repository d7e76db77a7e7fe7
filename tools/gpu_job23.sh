set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g2.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 || exit 1
for spec in 3 5; do
  for cfg in "bls12_381 12" "bls12_381 14" "bls12_381 16" "bls12_381 17" "bls12_381 18" "bls12_381 20" "bn128 20"; do
    ZK_MSM_SPEC=$spec ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py $cfg 0 2>&1 | tail -2 | sed "s/^/SPEC=$spec /" || exit 1
  done
done
