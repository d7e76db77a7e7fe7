#!/bin/bash
# round-6 job v: two interleaved chains per lane in the Fr batch inversion (ZK_INV_ILP): parity, then A/B with the lane count
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06v_arr_tests.txt 2>&1
rc=$?; tail -1 gpurun_out/r06v_arr_tests.txt; [ $rc -eq 0 ] || exit $rc
( for rep in 1 2; do for cfg in "0 131072" "1 131072" "1 65536" "1 262144"; do set -- $cfg
    echo -n "ZK_INV_ILP=$1 ZK_INV_LANES=$2  "; ZK_INV_ILP=$1 ZK_INV_LANES=$2 timeout -k 10 120 python tools/inv_probe.py || exit 1
  done; done ) > gpurun_out/r06v_inv_ilp_ab.txt 2>&1 || exit 1
cut -c1-160 gpurun_out/r06v_inv_ilp_ab.txt
