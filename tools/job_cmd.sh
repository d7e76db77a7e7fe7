# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
set -e
timeout 200 python -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_g1ext.py tests/test_gpu_arr.py -x -q --timeout 120 --timeout-method thread
for v in base base; do
  timeout 100 python bench.py --steps 2 --warmup 1 --no-e2e --no-cpu-baseline --ntt-steps 5 | python -c "import json,sys; d=json.load(sys.stdin)['ntt']; print({k: (d[k]['ms'], d[k]['kernel_ms']) for k in ('forward','inverse')}, d['parity_vs_reference'])"
done
