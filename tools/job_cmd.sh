# r04u: config-5 size (BLS12-381 2^26, one GPU): per-phase profile and window sweep
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -c "
import sys; sys.path.insert(0, 'tools'); import sweep_window as s
s.run('bls12_381', 26, [0], reps=3, profile=True)
" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 500 python -u tools/sweep_window.py bls12_381 26 18 19 21 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_g1ext.py -m gpu 2>&1 | tail -3 || exit 1
timeout -k 10 300 python -u tools/fft_time.py 16 3 check 2>&1 | grep -v amdgpu.ids || exit 1
