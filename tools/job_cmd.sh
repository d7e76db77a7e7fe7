# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# A/B/C: new = k_points_int staged through LDS + k_coarse aggregated counters / shuffle scan,
# pts = the points change only, head = committed HEAD; alternating in one job
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_g2.py -x -q -m gpu --timeout 120 --timeout-method thread 2>&1 | tail -3
for rep in 1 2 3; do
for v in new pts head; do
  if [ $v = new ]; then unset ZK_LIB_PATH; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  timeout -k 10 200 python -u -c "
import sys, os, time; sys.path.insert(0, 'zikkurat-algebra_amd'); import zkalgebra as zk
out = []
for curve in ('bls12_381', 'bn128'):
    for lg in (16, 20):
        n = 1 << lg
        ds, dp = zk.DeviceBuffer(zk.gen_fr(curve, 0x5A4B0002, n)), zk.DeviceBuffer(zk.gen_points(curve, 0x5A4B0002, n))
        for _ in range(2): zk.msm_device(curve, n, ds, dp)
        zk.load().zkg_device_synchronize(); t = time.perf_counter()
        for _ in range(20): zk.msm_device(curve, n, ds, dp)
        out.append('%s 2^%d %.3f' % (curve, lg, (time.perf_counter() - t) / 20 * 1e3))
print('$v', ' | '.join(out), flush=True)
" 2>&1 | grep -v amdgpu.ids || exit 1
done
done
for v in new pts head; do
  if [ $v = new ]; then unset ZK_LIB_PATH; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "profile $v"
  timeout -k 10 100 python -u -c "
import sys; sys.path.insert(0, 'zikkurat-algebra_amd'); import zkalgebra as zk
n = 1 << 20
ds, dp = zk.DeviceBuffer(zk.gen_fr('bls12_381', 1, n)), zk.DeviceBuffer(zk.gen_points('bls12_381', 1, n))
import numpy as np; sc = np.zeros((n, 4), dtype=np.uint64); sc[:, 0] = np.random.default_rng(91).integers(0, 2, n).astype(np.uint64); bs = zk.DeviceBuffer(sc)
zk.msm_device('bls12_381', n, ds, dp); zk.msm_device('bls12_381', n, bs, dp, mont=False); zk.msm_profile(True)
for _ in range(2): zk.msm_device('bls12_381', n, ds, dp)
for _ in range(2): zk.msm_device('bls12_381', n, bs, dp, mont=False)
" 2>&1 | grep -v amdgpu.ids || exit 1
done
