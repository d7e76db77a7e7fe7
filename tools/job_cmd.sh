# r04y: level 1.5 restricted to c >= 19: skew 2^22 (c = 20 device path) + configs first, 2^26 profile
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_msm.py -m gpu -k "skewed_2_22 or config4 or config5" 2>&1 | tail -3 || exit 1
timeout -k 10 400 python -u -c "
import sys; sys.path.insert(0, 'tools'); import sweep_window as s
s.run('bls12_381', 26, [0], reps=3, profile=True)
s.run('bls12_381', 25, [0], reps=3, profile=True)
" 2>&1 | grep -v amdgpu.ids || exit 1
