set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_g2.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t7.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/t7.log | tail -30
exit $rc
