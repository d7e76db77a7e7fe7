# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# the library on torch's bundled HIP runtime (what bench.py --gpus N with RCCL now does: torch.cuda first):
# MSM / NTT GPU tests and the headline timings in that process layout
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -c "
import torch; torch.cuda.set_device(0); print('torch runtime first', torch.version.hip, flush=True)
import sys, pytest
sys.exit(pytest.main(['tests/test_gpu_msm.py', 'tests/test_gpu_ntt.py', '-x', '-q', '-m', 'gpu', '-k', 'golden or config2 or config4 or sizes or binary', '--timeout', '300']))
" 2>&1 | grep -v amdgpu.ids | tail -5
timeout -k 10 200 python -u -c "
import torch; torch.cuda.set_device(0)
import sys, os, time; sys.path.insert(0, 'zikkurat-algebra_amd'); import zkalgebra as zk
print(sorted(set(l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l)))
n = 1 << 20
ds, dp = zk.DeviceBuffer(zk.gen_fr('bls12_381', 0x5A4B0002, n)), zk.DeviceBuffer(zk.gen_points('bls12_381', 0x5A4B0002, n))
for _ in range(2): zk.msm_device('bls12_381', n, ds, dp)
zk.load().zkg_device_synchronize(); t = time.perf_counter()
for _ in range(20): zk.msm_device('bls12_381', n, ds, dp)
print('msm 2^20 on torch runtime %.3f ms' % ((time.perf_counter() - t) / 20 * 1e3))
" 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u -c "
import sys, os, time; sys.path.insert(0, 'zikkurat-algebra_amd'); import zkalgebra as zk
n = 1 << 20
ds, dp = zk.DeviceBuffer(zk.gen_fr('bls12_381', 0x5A4B0002, n)), zk.DeviceBuffer(zk.gen_points('bls12_381', 0x5A4B0002, n))
for _ in range(2): zk.msm_device('bls12_381', n, ds, dp)
zk.load().zkg_device_synchronize(); t = time.perf_counter()
for _ in range(20): zk.msm_device('bls12_381', n, ds, dp)
print('msm 2^20 on /opt/rocm runtime %.3f ms' % ((time.perf_counter() - t) / 20 * 1e3))
" 2>&1 | grep -v amdgpu.ids
true
