# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# lazy full XYZZ add in the Y sums (variants/lz) vs the in-tree build
ZK_LIB_PATH=$PWD/variants/lz/libzkalgebra_gpu.so timeout 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_dist.py tests/test_gpu_concurrency.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -2
for v in base lz base lz; do
  if [ $v = base ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"
  timeout 100 python tools/sweep_window.py phases2 2>&1 | grep -E "ms/msm|^\[zk msm\]" | awk '/ms\/msm/ || NR%5==4'
done
