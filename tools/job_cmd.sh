# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# lazy BN128 mixed add in k_accum: variants/bnw4 (4 waves/SIMD, 30 spilled VGPRs), variants/bnw3 (3 waves, 153 VGPRs)
for v in bnw4 bnw3; do
  echo "== tests $v"
  ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so timeout 300 python -u -m pytest tests/test_gpu_msm.py -q -x --timeout 120 --timeout-method thread -k "bn128" 2>&1 | tail -2
done
for v in base bnw4 bnw3 base bnw4 bnw3; do
  if [ $v = base ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"
  timeout 100 python tools/sweep_window.py bn128 20
  timeout 100 python tools/sweep_window.py bn128 16
  timeout 100 python tools/sweep_window.py bn128 22
done
