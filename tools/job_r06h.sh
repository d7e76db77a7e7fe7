#!/bin/bash
# round-6 job h: software-pipelined Fr op kernel (ZK_ARR_STAGE=4): parity, then A/B against stage 2 and grid caps
set -o pipefail
mkdir -p gpurun_out
ZK_ARR_STAGE=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06h_arr_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06h_arr_tests.txt; [ $rc -eq 0 ] || exit $rc
( for cfg in "2 0" "4 0" "4 1024" "4 2048" "2 0"; do set -- $cfg
    echo "== ZK_ARR_STAGE=$1 ZK_ARR_GRID=$2"; ZK_ARR_STAGE=$1 ZK_ARR_GRID=$2 timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
  done ) > gpurun_out/r06h_arr_pf_ab.txt 2>&1 || exit 1
cat gpurun_out/r06h_arr_pf_ab.txt
