# r04zc: kernel stats of BLS12-381 2^26 MSMs with the sub-bin sort
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04zc_p26 -o run --output-format csv -- python3 tools/sweep_window.py bls12_381 26 20 > gpurun_out/r04zc_p26.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multidev.py -m gpu -k "config5" 2>&1 | tail -2 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_g1ext.py -m gpu 2>&1 | tail -2 || exit 1
