set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_g1ext.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t6.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/t6.log | tail -40
exit $rc
