set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1 || { echo tests FAILED; tail -30 gpurun_out/t2.log; exit 1; }
echo tests ok
for cfg in "8 8" "4 8" "8 4" "16 8" "4 4" "16 16"; do
  set -- $cfg
  echo "QY=$1 QA=$2"
  ZK_MSM_QY=$1 ZK_MSM_QA=$2 ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 16 2>&1 | tail -2 || exit 1
done
