# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
set -e
for v in base chain base chain; do
  if [ $v = base ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"
  timeout 100 python tools/sweep_window.py bls12_381 20
  timeout 100 python tools/sweep_window.py bn128 20
done
