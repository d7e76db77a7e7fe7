#!/bin/bash
# round-6 job o: operand-scanning REDC in the 381-bit Karatsuba products (variants/rows, -DZK_REDC_ROWS=1)
# against the in-tree build: headline MSM step and k_accum event time, alternating 3x; parity on the variant
set -o pipefail
mkdir -p gpurun_out
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-config4 --no-config5 --no-ntt --no-extras"
ZK_LIB_PATH=$PWD/variants/rows/libzkalgebra_gpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r06o_rows_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06o_rows_tests.txt; [ $rc -eq 0 ] || exit $rc
( for rep in 1 2 3; do for v in base rows; do
    if [ $v = rows ]; then export ZK_LIB_PATH=$PWD/variants/rows/libzkalgebra_gpu.so; else unset ZK_LIB_PATH; fi
    timeout -k 10 200 python $B > gpurun_out/r06o_b.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r06o_b.json')); print('$v', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['parity_vs_reference'])"
  done; done ) > gpurun_out/r06o_redc_rows_ab.txt 2>&1 || exit 1
cat gpurun_out/r06o_redc_rows_ab.txt
