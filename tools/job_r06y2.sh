#!/bin/bash
# round-6 job y2: NTT pass kernel with its load / closing loops unrolled by 4 (variants/nttu) vs the in-tree build
set -o pipefail
mkdir -p gpurun_out
V=$PWD/variants/nttu/libzkalgebra_gpu.so
ZK_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_ntt.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06y2_ntt_tests.txt 2>&1
rc=$?; tail -1 gpurun_out/r06y2_ntt_tests.txt; [ $rc -eq 0 ] || exit $rc
( for rep in 1 2 3; do
    echo -n "base  "; timeout -k 10 120 python tools/ntt_time.py 24 20 || exit 1
    echo -n "unroll  "; ZK_LIB_PATH=$V timeout -k 10 120 python tools/ntt_time.py 24 20 || exit 1
  done ) > gpurun_out/r06y2_ntt_unroll_ab.txt 2>&1 || exit 1
cat gpurun_out/r06y2_ntt_unroll_ab.txt
