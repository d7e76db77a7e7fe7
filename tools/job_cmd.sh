# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# event spin-wait at the end of the synchronous MSM / NTT calls (in-tree) vs blocking stream sync (variants/prev)
timeout 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_ntt.py tests/test_gpu_concurrency.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -2
for v in prev new prev new; do
  if [ $v = new ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"
  timeout 100 python tools/sweep_window.py bls12_381 20
  timeout 100 python tools/sweep_window.py bls12_381 16
  timeout 100 python tools/sweep_window.py bn128 20
  timeout 100 python tools/ntt_time.py 24 20
done
