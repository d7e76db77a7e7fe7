set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t8.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/t8.log; exit 1; }
tail -2 gpurun_out/t8.log
timeout -k 10 300 python bench.py > gpurun_out/b8.json 2> gpurun_out/b8.err || { echo BENCH FAILED; tail gpurun_out/b8.err; exit 1; }
timeout -k 10 400 python tools/bench_ext.py > gpurun_out/ext8.json 2> gpurun_out/ext8.err || { echo EXT FAILED; tail gpurun_out/ext8.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --ntt-steps 3 > gpurun_out/b8p.json 2> gpurun_out/b8p.err || { echo PROF FAILED; tail gpurun_out/b8p.err; exit 1; }
echo all ok
