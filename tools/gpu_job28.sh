set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputests28.log 2>&1 && echo tests=ok &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke28.log 2>&1 && echo smoke=ok &&
timeout -k 10 300 python bench.py > gpurun_out/bench28.json 2> gpurun_out/bench28.err && echo bench=ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof28 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ntt-steps 3 > gpurun_out/bench28p.json 2>gpurun_out/bench28p.err && echo prof=ok &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc28a -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --ntt-steps 2 > /dev/null 2>gpurun_out/pmc28a.err && echo pmca=ok &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc28b -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --ntt-steps 2 > /dev/null 2>gpurun_out/pmc28b.err && echo pmcb=ok
