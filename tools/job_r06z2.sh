#!/bin/bash
# round-6 job z2: batch_to_affine lane-count sweep on the branch-free normalisation (ZK_NORM_LANES)
set -o pipefail
mkdir -p gpurun_out
( for rep in 1 2; do for l in 32768 65536 131072 196608 262144 524288; do
    echo -n "ZK_NORM_LANES=$l  "; ZK_NORM_LANES=$l timeout -k 10 120 python tools/inv_probe.py || exit 1
  done; done ) > gpurun_out/r06z2_norm_lanes.txt 2>&1 || exit 1
cut -c1-230 gpurun_out/r06z2_norm_lanes.txt
