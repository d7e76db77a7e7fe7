#!/bin/bash
# round-6 job n: host-buffer MSM with every split's sort in line on the main stream (ZK_MSM_SORT_INLINE=1) vs the sort stream
set -o pipefail
mkdir -p gpurun_out
( for rep in 1 2 3; do for v in 0 1; do
    echo -n "SORT_INLINE=$v  "; ZK_MSM_SORT_INLINE=$v timeout -k 10 120 python3 tools/e2e_probe.py bls12_381 20 20 || exit 1
    echo -n "SORT_INLINE=$v  "; ZK_MSM_SORT_INLINE=$v timeout -k 10 120 python3 tools/e2e_probe.py bn128 20 20 || exit 1
  done; done ) > gpurun_out/r06n_sort_inline_ab.txt 2>&1 || exit 1
cat gpurun_out/r06n_sort_inline_ab.txt
