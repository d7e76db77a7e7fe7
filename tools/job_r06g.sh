#!/bin/bash
# round-6 job g: whole GPU suite on the current tree, strided-chunk inversion A/B, Fr ops, then the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06g_gpu_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06g_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
( for v in 1 0; do echo "== ZK_INV_STRIDE=$v"; ZK_INV_STRIDE=$v timeout -k 10 120 python tools/inv_probe.py || exit 1; ZK_INV_STRIDE=$v timeout -k 10 120 python tools/fft_time.py 12 5 || exit 1; done ) > gpurun_out/r06g_inv_stride_ab.txt 2>&1 || exit 1
cat gpurun_out/r06g_inv_stride_ab.txt
timeout -k 10 200 python tools/arr_time.py 24 10 > gpurun_out/r06g_arr_time.txt 2>&1 || exit 1
cat gpurun_out/r06g_arr_time.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r06g_bench.json 2> gpurun_out/r06g_bench.err || { tail gpurun_out/r06g_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r06g_bench.json')); print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))"
