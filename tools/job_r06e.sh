#!/bin/bash
# round-6 job e: Fr vector op tests + A/B (nontemporal staged / staged / per-lane), G2 tests at bench
# sizes, G2 2^18 / 2^20 kernel stats on distinct points
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_arr.py tests/test_gpu_g2.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06e_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r06e_tests.txt; [ $rc -eq 0 ] || exit $rc
( echo "== staged + nontemporal, 1024 workgroups (default)"; timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
  echo "== staged, plain loads/stores (ZK_ARR_STAGE=1)"; ZK_ARR_STAGE=1 timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
  echo "== per-lane 32-B accesses (ZK_ARR_STAGE=0)"; ZK_ARR_STAGE=0 timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
  echo "== staged + nontemporal, 4096 workgroups (ZK_ARR_GRID=4096)"; ZK_ARR_GRID=4096 timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
) > gpurun_out/r06e_arr_ab.txt 2>&1 || exit 1
cat gpurun_out/r06e_arr_ab.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06e_g2prof -o g2 --output-format csv -- python3 tools/g2_time.py > gpurun_out/r06e_g2_time.txt 2>&1 || { tail gpurun_out/r06e_g2_time.txt; exit 1; }
cat gpurun_out/r06e_g2_time.txt | grep -v "^\[" | tail -8
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/r06e_g2pmcsq -o g2 --output-format csv -- python3 tools/g2_time.py > gpurun_out/r06e_g2pmcsq.log 2>&1 || { tail gpurun_out/r06e_g2pmcsq.log; exit 1; }
python3 tools/sq_summary.py gpurun_out/r06e_g2pmcsq --source "r06e: rocprofv3 --pmc SQ_* GRBM_GUI_ACTIVE -- python3 tools/g2_time.py (G2 MSM 2^18 / 2^20, distinct points, both curves; MI355X)" > gpurun_out/r06e_g2_sq_pmc.json
echo done
