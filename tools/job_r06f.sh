#!/bin/bash
# round-6 job f: tree-summed radix stages (g1ext tests + sizes), G2 Y sums through LDS (tests + A/B
# with kernel trace), Fr vector ops grid A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_g1ext.py tests/test_gpu_arr.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06f_tests.txt; [ $rc -eq 0 ] || exit $rc
ZK_YSUM_G2_LDS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_g2.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f_g2lds_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06f_g2lds_tests.txt; [ $rc -eq 0 ] || exit $rc
for m in 10 12 13 14; do timeout -k 10 120 python tools/fft_time.py $m 5 || exit 1; done > gpurun_out/r06f_fft_sizes.txt 2>&1 || exit 1
cat gpurun_out/r06f_fft_sizes.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 0 1; do
  ZK_YSUM_G2_LDS=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06f_g2lds$v -o g2 --output-format csv -- python3 tools/g2_time.py > gpurun_out/r06f_g2lds$v.txt 2>&1 || { tail gpurun_out/r06f_g2lds$v.txt; exit 1; }
  echo "ZK_YSUM_G2_LDS=$v"; grep "G2 2^" gpurun_out/r06f_g2lds$v.txt
done
( for v in 1 0; do echo "== ZK_INV_SG=$v"; ZK_INV_SG=$v timeout -k 10 120 python tools/inv_probe.py || exit 1; ZK_INV_SG=$v timeout -k 10 120 python tools/fft_time.py 12 5 || exit 1; done
  for l in 131072 262144; do echo "== ZK_NORM_LANES=$l ZK_INV_LANES=$((l*2))"; ZK_NORM_LANES=$l ZK_INV_LANES=$((l*2)) timeout -k 10 120 python tools/inv_probe.py || exit 1; done ) > gpurun_out/r06f_inv_ab.txt 2>&1 || exit 1
cat gpurun_out/r06f_inv_ab.txt
( for g in 2048 65536; do echo "== ZK_ARR_GRID=$g"; ZK_ARR_GRID=$g timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1; done ) > gpurun_out/r06f_arr_grid.txt 2>&1 || exit 1
cat gpurun_out/r06f_arr_grid.txt
