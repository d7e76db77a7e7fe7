#!/bin/bash
# round-6 job r: parity of the prefetching fused kernel, then the per-kernel split of the division by a vanishing polynomial (rocprofv3 stats), new vs legacy
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06r_arr_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06r_arr_tests.txt; [ $rc -eq 0 ] || exit $rc
ZK_VANISH_STAGED=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q -k vanishing --timeout 120 --timeout-method thread > gpurun_out/r06r_arr_tests_pl.txt 2>&1
rc=$?; tail -2 gpurun_out/r06r_arr_tests_pl.txt; [ $rc -eq 0 ] || exit $rc
for v in 0 1 2; do
  [ $v = 2 ] && export ZK_VANISH_STAGED=0
  ZK_VANISH_LEGACY=$((v == 1))  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06r_prof$v -o run --output-format csv -- \
    python3 tools/vanish_probe.py 22 20 > gpurun_out/r06r_probe$v.txt 2> gpurun_out/r06r_prof$v.err || exit 1
  echo "== mode $v (0 fused staged, 1 legacy, 2 fused per-lane)"; cat gpurun_out/r06r_probe$v.txt; cut -d, -f1-4 gpurun_out/r06r_prof$v/run_kernel_stats.csv | cut -c1-160
done > gpurun_out/r06r_vanish_prof.txt
cat gpurun_out/r06r_vanish_prof.txt
