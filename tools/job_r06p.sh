#!/bin/bash
# round-6 job p: G1 Y sums through the LDS-gather k_ysum3<C, 1> (variants/ysumg1, ZK_YSUM_G1_LDS=1) vs k_ysum2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export ZK_LIB_PATH=$PWD/variants/ysumg1/libzkalgebra_gpu.so
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-config4 --no-config5 --no-ntt --no-extras"
ZK_YSUM_G1_LDS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r06p_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06p_tests.txt; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  ZK_YSUM_G1_LDS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06p_prof$v -o run --output-format csv -- \
    python3 $B > gpurun_out/r06p_b$v.json 2> gpurun_out/r06p_prof$v.err || exit 1
done
( for rep in 1 2 3; do for v in 0 1; do
    ZK_YSUM_G1_LDS=$v timeout -k 10 200 python $B > gpurun_out/r06p_b.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r06p_b.json')); print('G1_LDS=$v', round(d['ms_per_step'],4), d['parity_vs_reference'])"
  done; done
  for v in 0 1; do echo "== G1_LDS=$v"; grep -E "k_ysum|k_accum" gpurun_out/r06p_prof$v/run_kernel_stats.csv | cut -c1-200; done
  for v in 0 1; do echo "== G1_LDS=$v bn128 2^20"; ZK_YSUM_G1_LDS=$v timeout -k 10 120 python3 tools/sweep_window.py bn128 20 16 || exit 1; done
) > gpurun_out/r06p_ysum_g1_lds_ab.txt 2>&1 || exit 1
cat gpurun_out/r06p_ysum_g1_lds_ab.txt
