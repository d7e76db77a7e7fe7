#!/bin/bash
# round-6 job: G1 ext tests (Jacobian twins, m = 16 digests) + radix group-FFT A/B timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_g1ext.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06a_g1ext_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r06a_g1ext_tests.txt
[ $rc -eq 0 ] || exit $rc
for m in 10 12 13 14 15 16; do
  timeout -k 10 120 python tools/fft_time.py $m 3 check || exit 1
  ZK_FFT_RADIX=1 timeout -k 10 120 python tools/fft_time.py $m 3 || exit 1
done > gpurun_out/r06a_fft_radix_ab.txt 2>&1
rc=$?
cat gpurun_out/r06a_fft_radix_ab.txt
exit $rc
