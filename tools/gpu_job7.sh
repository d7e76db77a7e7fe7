set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_msm.py -x -v -k config --timeout 400 --timeout-method thread --durations=5 > gpurun_out/t9.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|slowest|s call" gpurun_out/t9.log | tail -20
exit $rc
