set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof18 -o run -- python3 tools/sweep_window.py bls12_381 20 0 > gpurun_out/prof18.log 2>&1 || exit 1
find gpurun_out/prof18 -name "*.csv" | head
