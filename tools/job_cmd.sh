# r04n: GLV group FFT after the window-offset fix; bits-path timeline and phases
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_g1ext.py tests/test_gpu_msm_bits.py -m gpu 2>&1 | tail -15 || exit 1
timeout -k 10 300 python -u tools/fft_time.py 16 3 check 2>&1 | grep -v amdgpu.ids || exit 1
for lg in 10 12; do
  ZK_PROBE_PHASES=1 timeout -k 10 120 python -u tools/small_probe.py bls12_381 $lg 20 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r04n_tr10 -o run --output-format csv -- python3 tools/small_probe.py bls12_381 10 6 > gpurun_out/r04n_tr10.log 2>&1 || exit 1
