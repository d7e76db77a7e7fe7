#!/bin/bash
# round-6 job q: fused, LDS-staged division by a vanishing polynomial with the top-down degree scan: parity, then
# bench_ext's 2^22 case against the round-5 kernels (ZK_VANISH_LEGACY=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06q_arr_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06q_arr_tests.txt; [ $rc -eq 0 ] || exit $rc
ZK_VANISH_LEGACY=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q -k vanishing --timeout 120 \
  --timeout-method thread > gpurun_out/r06q_arr_tests_legacy.txt 2>&1
rc=$?; tail -2 gpurun_out/r06q_arr_tests_legacy.txt; [ $rc -eq 0 ] || exit $rc
( for rep in 1 2; do for v in 1 0; do
    ZK_VANISH_LEGACY=$v timeout -k 10 300 python tools/bench_ext.py > gpurun_out/r06q_ext$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r06q_ext$v.json'))['div_by_vanishing']; print('LEGACY=$v', json.dumps(d))"
  done; done ) > gpurun_out/r06q_vanish_ab.txt 2>&1 || exit 1
cat gpurun_out/r06q_vanish_ab.txt
