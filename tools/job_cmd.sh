# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
set -e
timeout 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread
for v in base nopipe pipe14 base nopipe; do
  if [ $v = base ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"
  timeout 100 python tools/sweep_window.py bls12_381 20
  timeout 100 python tools/sweep_window.py bn128 20
  timeout 100 python tools/sweep_window.py bls12_381 16
  timeout 100 python tools/sweep_window.py bls12_381 18
  timeout 100 python tools/sweep_window.py bls12_381 14
done
