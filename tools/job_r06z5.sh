#!/bin/bash
# round-6 job z5: lane counts of the Fr batch inversion after the 30-step divsteps (ZK_INV_LANES)
set -o pipefail
mkdir -p gpurun_out
( for rep in 1 2; do for l in 65536 131072 196608 262144; do
    echo -n "ZK_INV_LANES=$l  "; ZK_INV_LANES=$l timeout -k 10 120 python tools/inv_probe.py || exit 1
  done; done ) > gpurun_out/r06z5_inv_lanes.txt 2>&1 || exit 1
cut -c1-200 gpurun_out/r06z5_inv_lanes.txt
