#!/bin/bash
# round-6 job l: host-buffer MSM copy / kernel timeline on the current build (rocprofv3 kernel + memory-copy trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/e2e_probe.py bls12_381 20 10 > gpurun_out/r06l_e2e.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r06l_trace -o run --output-format csv -- \
  python3 tools/e2e_probe.py bls12_381 20 3 >> gpurun_out/r06l_e2e.txt 2> gpurun_out/r06l_trace.err || exit 1
python3 tools/trace_timeline.py gpurun_out/r06l_trace > gpurun_out/r06l_timeline.txt || exit 1
cat gpurun_out/r06l_e2e.txt; cat gpurun_out/r06l_timeline.txt
