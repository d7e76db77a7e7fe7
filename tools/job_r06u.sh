#!/bin/bash
# round-6 job u: wave-cooperative Fr batch inversion (ZK_INV_WAVE=K) -- parity for K = 4 / 8 / 16, then A/B vs the chunks
set -o pipefail
mkdir -p gpurun_out
for k in 4 8 16; do
  ZK_INV_WAVE=$k timeout -k 10 400 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r06u_arr_tests_k$k.txt 2>&1
  rc=$?; echo "K=$k: $(tail -1 gpurun_out/r06u_arr_tests_k$k.txt)"; [ $rc -eq 0 ] || exit $rc
done
( for rep in 1 2; do for k in 0 4 8 16; do
    echo -n "ZK_INV_WAVE=$k  "; ZK_INV_WAVE=$k timeout -k 10 120 python tools/inv_probe.py || exit 1
  done; done ) > gpurun_out/r06u_inv_wave_ab.txt 2>&1 || exit 1
cat gpurun_out/r06u_inv_wave_ab.txt
