# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# r04h: Y sums at 2 waves per SIMD (131072 lanes, 8 buckets each; quad fold) vs the default
cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for v in new ysA ysB; do
    if [ $v = new ]; then unset ZK_LIB_PATH; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
    for lg in 20 16; do
      timeout -k 10 120 python -u -c "
import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import sweep_window as s; s.run('bls12_381', $lg, [0], reps=3, profile=True)" 2>&1 | grep -v amdgpu.ids | sed "s/^/[$v] /" | tail -2 || exit 1
    done
  done
done
unset ZK_LIB_PATH
timeout -k 10 200 python -u tools/fft_time.py 16 2 2>&1 | grep -v amdgpu.ids || exit 1
