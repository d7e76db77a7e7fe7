#!/bin/bash
# round-6 job c: streaming ceiling microbenchmark, ext sweep (distinct G2 points, group-FFT plan),
# then SQ counters and kernel stats of the ext quick sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/stream_bw > gpurun_out/r06c_stream_bw.txt 2>&1 || exit 1
cat gpurun_out/r06c_stream_bw.txt
timeout -k 10 600 python tools/bench_ext.py > gpurun_out/r06c_ext.json 2> gpurun_out/r06c_ext.err || { tail gpurun_out/r06c_ext.err; exit 1; }
echo ext done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06c_prof -o ext --output-format csv -- python3 tools/bench_ext.py --quick > gpurun_out/r06c_prof.log 2>&1 || { tail gpurun_out/r06c_prof.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/r06c_pmcsq -o ext --output-format csv -- python3 tools/bench_ext.py --quick > gpurun_out/r06c_pmcsq.log 2>&1 || { tail gpurun_out/r06c_pmcsq.log; exit 1; }
python3 tools/sq_summary.py gpurun_out/r06c_pmcsq --source "r06c: rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 tools/bench_ext.py --quick (MI355X)" > gpurun_out/r06c_ext_sq_pmc.json
echo sq done
