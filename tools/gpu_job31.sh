set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputests31.log 2>&1 && echo tests=ok &&
timeout -k 10 120 python tools/sweep_window.py bls12_381 23 0 > gpurun_out/sweep31.txt 2>&1 &&
timeout -k 10 120 python tools/sweep_window.py bn128 22 0 >> gpurun_out/sweep31.txt 2>&1 && echo sweep=ok &&
timeout -k 10 300 python bench.py > gpurun_out/bench31.json 2> gpurun_out/bench31.err && echo bench=ok
