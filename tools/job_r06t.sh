#!/bin/bash
# round-6 job t: prefetching Fr batch-inversion chains (ZK_INV_PF) -- parity, then A/B with the lane count
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06t_arr_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06t_arr_tests.txt; [ $rc -eq 0 ] || exit $rc
( for rep in 1 2; do for cfg in "0 131072" "1 131072" "1 262144" "1 65536"; do set -- $cfg
    echo -n "ZK_INV_PF=$1 ZK_INV_LANES=$2  "; ZK_INV_PF=$1 ZK_INV_LANES=$2 timeout -k 10 120 python tools/inv_probe.py || exit 1
  done; done ) > gpurun_out/r06t_inv_pf_ab.txt 2>&1 || exit 1
cat gpurun_out/r06t_inv_pf_ab.txt
