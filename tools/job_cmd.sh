# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# (1) MADV_POPULATE_WRITE on a fresh 512 MiB array: does it work on this host, how long does it
#     take, and does it remove the first-touch cost of a device-to-host copy?
# (2) host-buffer MSM: in-tree (points in 2 splits, copy thread) vs variants/nosplit (-DZK_MSM_SPLITS=1)
cat > /tmp/pf.py <<'PY'
import ctypes, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "zikkurat-algebra_amd"))
import zkalgebra as zk
libc = ctypes.CDLL(None, use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
N = 512 << 20
print("kernel", os.uname().release)
for trial in range(2):
    a = np.zeros(N // 8, dtype=np.uint64)
    t = time.perf_counter(); r = libc.madvise(ctypes.c_void_p(a.ctypes.data & ~4095), N, 23); dt = time.perf_counter() - t
    print("madvise(POPULATE_WRITE) rc", r, "errno", ctypes.get_errno(), "%.2f ms" % (dt * 1e3))
    t = time.perf_counter(); a[::512] = 1; print("touch after populate %.2f ms" % ((time.perf_counter() - t) * 1e3))
    b = np.zeros(N // 8, dtype=np.uint64)
    t = time.perf_counter(); b[::512] = 1; print("first touch, fresh %.2f ms" % ((time.perf_counter() - t) * 1e3))
d = zk.DeviceBuffer.empty(N)
for label in ("fresh", "fresh+populate", "resident"):
    c = np.zeros(N // 8, dtype=np.uint64)
    if label == "fresh+populate": libc.madvise(ctypes.c_void_p(c.ctypes.data & ~4095), N, 23)
    if label == "resident": c[:] = 1
    t = time.perf_counter(); zk.load().zkg_memcpy_dtoh(c.ctypes.data, d.ptr, N); print("D2H 512 MiB", label, "%.2f ms" % ((time.perf_counter() - t) * 1e3))
m = 24; sg = zk.get_fft_subgroup("bls12_381", m); x = zk.gen_fr("bls12_381", 3, 1 << m)
zk.forward_ntt(sg, x)
for _ in range(3):
    t = time.perf_counter(); y = zk.forward_ntt(sg, x); print("forward_ntt 2^24 fresh output %.2f ms" % ((time.perf_counter() - t) * 1e3))
PY
timeout 120 python /tmp/pf.py || exit 1
cat > /tmp/e2e.py <<'PY'
import sys, time, os
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "zikkurat-algebra_amd"))
import zkalgebra as zk
for curve, logn in (("bls12_381", 20), ("bls12_381", 18), ("bn128", 20), ("bn128", 22)):
    n = 1 << logn
    sc, pts = zk.gen_fr(curve, 0x5A4B0002, n), zk.gen_points(curve, 0x5A4B0002, n)
    ref = zk.msm_affine(curve, sc, pts)
    t = time.perf_counter()
    for _ in range(10): out = zk.msm_affine(curve, sc, pts)
    assert (out == ref).all()
    print(curve, logn, "host-buffer msm %.3f ms" % ((time.perf_counter() - t) / 10 * 1e3), flush=True)
PY
for v in nosplit new nosplit new; do
  if [ $v = new ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"; timeout 120 python /tmp/e2e.py || exit 1
done
unset ZK_LIB_PATH
