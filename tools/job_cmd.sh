# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# NTT: non-last passes store packed, not canonicalised (in-tree) vs canonical (variants/prev)
timeout 400 python -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_arr.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -2
for v in prev new prev new prev new; do
  if [ $v = new ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"; timeout 120 python tools/ntt_time.py 24 20
done
