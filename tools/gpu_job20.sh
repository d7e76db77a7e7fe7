set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g2.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 || exit 1
timeout -k 10 200 python tools/g2_ab.py gpurun_out/g2_idx.npz || exit 1
for sch in 4 8; do
  ZK_MSM_SCH=$sch ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -2 | head -1 | sed "s/^/SCH=$sch /" || exit 1
  ZK_MSM_SCH=$sch ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 14 0 2>&1 | tail -2 | head -1 | sed "s/^/2^14 SCH=$sch /" || exit 1
done
