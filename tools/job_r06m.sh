#!/bin/bash
# round-6 job m: host-buffer MSM split-weight sweep (ZK_MSM_SPLIT_W), BLS12-381 2^20, twice round robin
set -o pipefail
mkdir -p gpurun_out
( for rep in 1 2; do for w in "2,3,4,4,3" "1,2,3,4,4,2" "2,4,5,5" "1,3,4,4,3,1" "2,3,3,3,3,2" "3,4,5,4" "1,2,4,5,4" "2,3,4,4,2,1"; do
    echo -n "W=$w  "; ZK_MSM_SPLIT_W=$w timeout -k 10 120 python3 tools/e2e_probe.py bls12_381 20 20 || exit 1
  done; done ) > gpurun_out/r06m_split_sweep.txt 2>&1 || exit 1
cat gpurun_out/r06m_split_sweep.txt
