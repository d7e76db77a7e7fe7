set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python tools/sweep_window.py bls12_381 23 16 17 18 19 20 > gpurun_out/sw23.txt 2>&1 || { echo SWEEP FAILED; tail gpurun_out/sw23.txt; exit 1; }
cat gpurun_out/sw23.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o run --output-format csv -- ./tools/microbench/gather_calib > gpurun_out/calib.log 2>&1 || { echo CALIB FAILED; tail gpurun_out/calib.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcA -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --ntt-steps 2 > /dev/null 2> gpurun_out/pmcA.err || { echo PMCA FAILED; tail gpurun_out/pmcA.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcB -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --ntt-steps 2 > /dev/null 2> gpurun_out/pmcB.err || { echo PMCB FAILED; tail gpurun_out/pmcB.err; exit 1; }
python tools/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB gpurun_out/calib > gpurun_out/pmc_summary.json && cat gpurun_out/pmc_summary.json
