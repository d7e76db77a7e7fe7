set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1 && echo tests=ok
timeout -k 10 300 python bench.py > gpurun_out/b1.json 2> gpurun_out/b1.err && echo bench=ok
