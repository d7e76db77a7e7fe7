set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_msm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1 || { echo tests FAILED; tail -30 gpurun_out/t3.log; exit 1; }
echo tests ok; tail -2 gpurun_out/t3.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b3.json 2> gpurun_out/b3.err || { echo bench FAILED; tail gpurun_out/b3.err; exit 1; }
python - <<'P'
import json; d=json.load(open('gpurun_out/b3.json'))
print('msm', d['value'], d['ms_per_step'], d['valu_roofline']['frac'])
n=d['ntt']; print('ntt fwd ms', n['forward']['ms'], 'inv ms', n['inverse']['ms'], n['forward']['valu_roofline']['frac'])
P
