#!/bin/bash
# round-6 job z4: headline MSM step repeated (box-to-box spread check of the final tree)
set -o pipefail
mkdir -p gpurun_out
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-config4 --no-config5 --no-ntt --no-extras"
( for rep in 1 2 3 4; do
    timeout -k 10 200 python $B > gpurun_out/r06z4_b.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r06z4_b.json')); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['parity_vs_reference'])"
  done; nproc; uptime ) > gpurun_out/r06z4_steps.txt 2>&1 || exit 1
cat gpurun_out/r06z4_steps.txt
