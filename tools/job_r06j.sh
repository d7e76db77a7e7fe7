#!/bin/bash
# round-6 job j: new Fr op defaults (stage 4 for streaming ops, stage 2 at 8192 workgroups for product ops): parity + timing x2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06j_arr_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06j_arr_tests.txt; [ $rc -eq 0 ] || exit $rc
( for i in 1 2; do timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1; done ) > gpurun_out/r06j_arr_time.txt 2>&1 || exit 1
cat gpurun_out/r06j_arr_time.txt
