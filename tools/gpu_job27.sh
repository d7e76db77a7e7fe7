set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_arr.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputests27.log 2>&1 && echo tests=ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --ntt-steps 10 > gpurun_out/bench27.json 2> gpurun_out/bench27.err && echo bench=ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --curve bn128 --ntt-steps 10 > gpurun_out/bench27bn.json 2> gpurun_out/bench27bn.err && echo benchbn=ok
