#!/bin/bash
# round-6 job i: the software-pipelined Fr op kernel (ZK_ARR_STAGE=4) at larger grids (one workgroup per 256
# elements = loads of all arrays issued up front, no grid-stride loop), against stage 2
set -o pipefail
mkdir -p gpurun_out
( for cfg in "4 65536" "4 8192" "2 8192" "4 0" "2 0"; do set -- $cfg
    echo "== ZK_ARR_STAGE=$1 ZK_ARR_GRID=$2"; ZK_ARR_STAGE=$1 ZK_ARR_GRID=$2 timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
  done ) > gpurun_out/r06i_arr_pf_grid.txt 2>&1 || exit 1
cat gpurun_out/r06i_arr_pf_grid.txt
