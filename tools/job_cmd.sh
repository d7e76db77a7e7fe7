# r04t: GLV FFT with the pair-shared table and the sparse-z membership test
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_g1ext.py -m gpu 2>&1 | tail -3 || exit 1
timeout -k 10 300 python -u tools/fft_time.py 16 3 check 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u tools/fft_time.py 16 3 2>&1 | grep -v amdgpu.ids || exit 1
