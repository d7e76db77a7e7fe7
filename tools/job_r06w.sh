#!/bin/bash
# round-6 job w: per-kernel split of the Fr batch inversion / G1 batch_to_affine probe (rocprofv3 stats)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06w_prof -o run --output-format csv -- python3 tools/inv_probe.py \
  > gpurun_out/r06w_probe.txt 2> gpurun_out/r06w_prof.err || exit 1
python3 - <<'PY' > gpurun_out/r06w_inv_prof.txt
import csv
for r in csv.DictReader(open('gpurun_out/r06w_prof/run_kernel_stats.csv')):
    print(r['Name'][:90], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
cat gpurun_out/r06w_probe.txt gpurun_out/r06w_inv_prof.txt
