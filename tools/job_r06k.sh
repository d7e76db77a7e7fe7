#!/bin/bash
# round-6 job k: product Fr ops held to 64 VGPRs (ZK_ARR_STAGE=6: 8 wavefronts per SIMD) against stage 2
set -o pipefail
mkdir -p gpurun_out
ZK_ARR_STAGE=6 timeout -k 10 300 python -u -m pytest tests/test_gpu_arr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06k_arr_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r06k_arr_tests.txt; [ $rc -eq 0 ] || exit $rc
( for cfg in "6 0" "2 0" "6 4096" "2 4096" "6 0" "2 0"; do set -- $cfg
    echo "== ZK_ARR_STAGE=$1 ZK_ARR_GRID=$2"; ZK_ARR_STAGE=$1 ZK_ARR_GRID=$2 timeout -k 10 200 python tools/arr_time.py 24 10 || exit 1
  done ) > gpurun_out/r06k_arr_w8.txt 2>&1 || exit 1
python - <<'PY'
import json
cur=None
for l in open('gpurun_out/r06k_arr_w8.txt'):
    if l.startswith('=='): cur=l.strip(); continue
    c, m, js = l.split(' ', 2); d=json.loads(js)
    print(cur, c, ' '.join(f"{k}={d[k]['TBps']}" for k in ('mul','sqr','scale','Ax_plus_y','Ax_plus_By')))
PY
