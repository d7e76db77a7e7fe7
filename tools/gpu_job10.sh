set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g2.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t10.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/t10.log; exit 1; }
tail -1 gpurun_out/t10.log
for spec in "bls12_381 10 0" "bls12_381 12 0" "bls12_381 14 0" "bls12_381 16 0" "bls12_381 18 0" "bls12_381 20 0" "bls12_381 26 0"; do
  timeout -k 10 200 python tools/sweep_window.py $spec 2>&1 | grep -v "^\[zk" || { echo SWEEP FAILED $spec; exit 1; }
done
