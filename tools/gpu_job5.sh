set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_arr.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?
tail -30 gpurun_out/t5.log
exit $rc
