# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
set -e
for v in base qy8 qy4 qa4 qy8qa4; do
  if [ $v = base ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"
  timeout 100 python tools/sweep_window.py phases2 2>&1
done
