#!/bin/bash
# round-6 job b: the whole GPU suite on the fast-conversion build, then FFT sizes and Fr vector ops
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b_gpu_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r06b_gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
for m in 12 13 14 15 16; do timeout -k 10 120 python tools/fft_time.py $m 3 || exit 1; done > gpurun_out/r06b_fft_sizes.txt 2>&1 || exit 1
cat gpurun_out/r06b_fft_sizes.txt
( echo "== staged per-op kernels (default)"; timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
  echo "== per-op kernels, per-lane 32-B accesses (ZK_ARR_STAGE=0)"; ZK_ARR_STAGE=0 timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
  echo "== round-5 switch kernel (ZK_ARR_MAP=1)"; ZK_ARR_MAP=1 timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
) > gpurun_out/r06b_arr_time.txt 2>&1 || exit 1
cat gpurun_out/r06b_arr_time.txt
