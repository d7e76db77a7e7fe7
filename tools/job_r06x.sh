#!/bin/bash
# round-6 job x: branch-free batch-affine normalisation (ZK_NORM_BF): g1ext parity, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_g1ext.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06x_g1ext_tests.txt 2>&1
rc=$?; tail -1 gpurun_out/r06x_g1ext_tests.txt; [ $rc -eq 0 ] || exit $rc
( for rep in 1 2; do for v in 0 1; do
    echo "== ZK_NORM_BF=$v"; ZK_NORM_BF=$v timeout -k 10 120 python tools/inv_probe.py || exit 1
    ZK_NORM_BF=$v timeout -k 10 120 python tools/fft_time.py 12 5 || exit 1
  done; done ) > gpurun_out/r06x_norm_bf_ab.txt 2>&1 || exit 1
cut -c1-220 gpurun_out/r06x_norm_bf_ab.txt
