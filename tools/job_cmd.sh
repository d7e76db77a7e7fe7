# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# r04g: shape-chosen quad stitch (sizes 2^10..2^20), quad FFT stages at 2 waves/SIMD vs one lane
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g1ext.py -x -q -m gpu --timeout 300 --timeout-method thread 2>&1 | tail -3
for rep in 1 2; do
  timeout -k 10 200 python -u tools/fft_time.py 16 2 2>&1 | grep -v amdgpu.ids || exit 1
  ZK_FFT_QUAD=0 timeout -k 10 200 python -u tools/fft_time.py 16 2 2>&1 | sed 's/^/[one-lane] /' | grep -v amdgpu.ids || exit 1
done
for lg in 10 11 12 13 14 15 16 18 20; do
  timeout -k 10 120 python -u -c "
import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import sweep_window as s; s.run('bls12_381', $lg, [0], reps=10)
s.run('bls12_381', $lg, [0], reps=2, profile=True)" 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
done
