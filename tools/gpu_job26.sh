set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputests26.log 2>&1 && echo tests=ok &&
timeout -k 10 300 python bench.py > gpurun_out/bench26.json 2> gpurun_out/bench26.err && echo bench=ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof26 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ntt-steps 3 > gpurun_out/bench26p.json 2>gpurun_out/bench26p.err && echo prof=ok &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc26a -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --ntt-steps 2 > /dev/null 2>gpurun_out/pmc26a.err && echo pmca=ok &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc26b -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --ntt-steps 2 > /dev/null 2>gpurun_out/pmc26b.err && echo pmcb=ok &&
timeout -k 10 300 python tools/bench_ext.py > gpurun_out/bench_ext26.json 2> gpurun_out/bench_ext26.err && echo ext=ok
