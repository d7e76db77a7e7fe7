#!/bin/bash
# round-6 job z3: inversion in 60-bit limbs with 2 x 30-step 32-bit divsteps (ZK_INV_DS30, zk_inv.hpp): the
# inversion users' parity (Fr ops, G1 ext, MSM), then the inversion-bound timings and a lane sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_arr.py tests/test_gpu_g1ext.py tests/test_gpu_msm.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r06z3_tests.txt 2>&1
rc=$?; tail -1 gpurun_out/r06z3_tests.txt; [ $rc -eq 0 ] || exit $rc
( for rep in 1 2; do for l in 65536 131072; do
    echo -n "ZK_NORM_LANES=$l  "; ZK_NORM_LANES=$l timeout -k 10 120 python tools/inv_probe.py || exit 1
  done; timeout -k 10 120 python tools/fft_time.py 12 5 || exit 1; done ) > gpurun_out/r06z3_ds30.txt 2>&1 || exit 1
cut -c1-230 gpurun_out/r06z3_ds30.txt
