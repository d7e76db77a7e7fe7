#!/bin/bash
# One parameterised GPU-box job (run through gpurun from the repo root):
#   gpurun --timeout 900 -- bash tools/gpu_job.sh TAG step [step ...]
# Steps (each under its own timeout; the job stops at the first failure):
#   tests     pytest -m gpu                       -> gpurun_out/TAG_tests.log
#   testscomm pytest -m gpu beside a live world-1 RCCL communicator (bench.py --gpus N layout) -> TAG_testscomm.log
#   testsel   pytest -m gpu -k "$TESTSEL"         -> gpurun_out/TAG_testsel.log
#   benchcomm bench.py --force-comm (the multi-GPU code path at world 1) -> gpurun_out/TAG_benchcomm.json
#   smoke     __graft_entry__.smoke()             -> gpurun_out/TAG_smoke.log
#   bench     python bench.py (defaults)          -> gpurun_out/TAG_bench.json
#   bench2    bench.py as 2 ranks on the one GPU (gloo exchange) -> gpurun_out/TAG_bench2.json
#   bench2self  bench.py --gpus 2 started WITHOUT torchrun (bench.py's own launcher), gloo exchange
#             -> gpurun_out/TAG_bench2self.json (must print n_gpus 2 and config5 parity true)
#   bench2rccl  bench.py --gpus 2 with the RCCL backend on the one GPU: RCCL refuses two ranks on one
#             device, so the launch MUST exit non-zero (no world-1 line) -> gpurun_out/TAG_bench2rccl.*
#   prof      rocprofv3 --kernel-trace --stats of a short bench -> gpurun_out/TAG_prof/
#   pmcf      rocprofv3 --pmc FETCH_SIZE (own pass) -> gpurun_out/TAG_pmcf/
#   pmcw      rocprofv3 --pmc WRITE_SIZE (own pass) -> gpurun_out/TAG_pmcw/
#   pmcsq     rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU ... (VALU issue, own pass) -> gpurun_out/TAG_pmcsq/
#   calib     rocprofv3 --pmc FETCH_SIZE of tools/microbench/gather_calib (known bytes) -> gpurun_out/TAG_calib/
#   listpmc   rocprofv3 -L (available counters)   -> gpurun_out/TAG_counters.txt
#   ceiling   tools/microbench/valu_ceiling (prebuilt) -> gpurun_out/TAG_ceiling.json
#   ext       tools/bench_ext.py                  -> gpurun_out/TAG_ext.json
#   profext   rocprofv3 --kernel-trace --stats of tools/bench_ext.py -> gpurun_out/TAG_profext/
#   pmcsqext  rocprofv3 --pmc SQ_* GRBM_GUI_ACTIVE over tools/bench_ext.py --quick (VALU busy per kernel)
#   phases    MSM phase profile at several sizes  -> gpurun_out/TAG_phases.txt
#   profsmall rocprofv3 --kernel-trace (per-dispatch timeline) of BLS12-381 2^16 MSMs -> gpurun_out/TAG_profsmall/
#   cmd       bash tools/job_cmd.sh (scratch commands of the current experiment) -> gpurun_out/TAG_cmd.log
set -o pipefail
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/$TAG
BENCH_SHORT="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-config4 --no-config5 --ntt-steps 3 --no-extras"
for step in "$@"; do
  echo "[$(date +%T)] step $step"
  case $step in
    tests) timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 ;;
    testscomm) ZKG_TEST_COMM=1 timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest tests -x -v -m gpu --timeout 120 \
              --timeout-method thread > ${O}_testscomm.log 2>&1 ;;
    testsel) timeout -k 10 ${TESTS_TIMEOUT:-600} python -u -m pytest tests -x -v -m gpu -k "$TESTSEL" --timeout 120 \
              --timeout-method thread > ${O}_testsel.log 2>&1 ;;
    benchcomm) timeout -k 10 300 python -u bench.py --force-comm --steps 10 --warmup 2 --no-e2e --no-cpu-baseline \
              --no-config4 --ntt-steps 2 > ${O}_benchcomm.json 2> ${O}_benchcomm.err ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 ;;
    bench) timeout -k 10 400 python -u bench.py > ${O}_bench.json 2> ${O}_bench.err ;;
    bench2) timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
              --master-port 29517 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > ${O}_bench2.json 2> ${O}_bench2.err ;;
    bench2self) timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --no-extras --no-e2e --no-cpu-baseline \
              --no-config4 --steps 5 --warmup 1 > ${O}_bench2self.json 2> ${O}_bench2self.err ;;
    bench2rccl) timeout -k 10 300 python -u bench.py --gpus 2 --no-extras --no-e2e --no-cpu-baseline --no-config4 \
              --no-config5 --no-ntt --steps 2 --warmup 1 > ${O}_bench2rccl.json 2> ${O}_bench2rccl.err
              rc=$?; echo "bench2rccl rc=$rc (non-zero expected)" >> ${O}_bench2rccl.err
              [ $rc -ne 0 ] && [ $rc -ne 124 ] && [ $rc -ne 137 ] && [ ! -s ${O}_bench2rccl.json ]; (exit $?) ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d ${O}_prof -o run --output-format csv -- python3 $BENCH_SHORT \
              > ${O}_prof_bench.json 2> ${O}_prof.err ;;
    pmcf) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d ${O}_pmcf -o run --output-format csv -- python3 $BENCH_SHORT \
              > /dev/null 2> ${O}_pmcf.err ;;
    pmcw) timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d ${O}_pmcw -o run --output-format csv -- python3 $BENCH_SHORT \
              > /dev/null 2> ${O}_pmcw.err ;;
    pmcsq) timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
              -d ${O}_pmcsq -o run --output-format csv -- python3 $BENCH_SHORT > /dev/null 2> ${O}_pmcsq.err ;;
    calib) timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d ${O}_calib -o run --output-format csv -- tools/microbench/gather_calib \
              > ${O}_calib.log 2>&1 ;;
    listpmc) timeout -k 10 120 rocprofv3 -L > ${O}_counters.txt 2>&1 ;;
    ceiling) timeout -k 10 120 tools/microbench/valu_ceiling > ${O}_ceiling.json 2> ${O}_ceiling.err ;;
    ext) timeout -k 10 400 python -u tools/bench_ext.py > ${O}_ext.json 2> ${O}_ext.err ;;
    profext) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d ${O}_profext -o run --output-format csv -- \
              python3 tools/bench_ext.py > ${O}_profext.json 2> ${O}_profext.err ;;
    pmcsqext) timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
              GRBM_GUI_ACTIVE -d ${O}_pmcsqext -o run --output-format csv -- python3 tools/bench_ext.py --quick \
              > /dev/null 2> ${O}_pmcsqext.err ;;
    phases) timeout -k 10 300 python -u tools/sweep_window.py phases > ${O}_phases.txt 2>&1 ;;
    profsmall) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_profsmall -o run --output-format csv -- \
              python3 tools/sweep_window.py bls12_381 16 > ${O}_profsmall.log 2>&1 ;;
    cmd) TAG=$TAG timeout -k 10 ${JOB_TIMEOUT:-400} bash tools/job_cmd.sh > ${O}_cmd.log 2>&1 ;;
    *) echo "unknown step $step"; false ;;
  esac
  rc=$?
  echo "[$(date +%T)] step $step rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
echo "job $TAG ok"
