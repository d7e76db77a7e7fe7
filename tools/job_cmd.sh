# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# k_fine templated on its width (1024 threads for bins >= 4096 entries, else 256; 4 loads in flight,
# wavefront-aggregated counters; in-tree) vs the committed 256-thread k_fine (variants/fine0): uniform scalars, binary 0/1
# scalars (one bin of ~n/2 entries), c = 17 at 2^22 (carry-only top window); alternating
cat > /tmp/ag.py <<'PY'
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "zikkurat-algebra_amd"))
import zkalgebra as zk
def run(label, curve, n, sc, pts, mont, window=0, reps=10, prof=False):
    ds, dp = zk.DeviceBuffer(sc), zk.DeviceBuffer(pts)
    r0 = zk.msm_device(curve, n, ds, dp, mont=mont, window=window); zk.load().zkg_device_synchronize()
    t = time.perf_counter()
    for _ in range(reps): zk.msm_device(curve, n, ds, dp, mont=mont, window=window)
    import hashlib
    print(label, "%.3f ms" % ((time.perf_counter() - t) / reps * 1e3), hashlib.sha256(r0.tobytes()).hexdigest()[:12], flush=True)
    if prof:
        zk.msm_profile(True); zk.msm_device(curve, n, ds, dp, mont=mont, window=window); zk.msm_profile(False)
for curve in ("bls12_381", "bn128"):
    for lg in (14, 16, 18, 20):
        n = 1 << lg
        pts = zk.gen_points(curve, 0x5A4B0002, n)
        run("%s uniform 2^%d" % (curve, lg), curve, n, zk.gen_fr(curve, 0x5A4B0002, n), pts, True, prof=(lg == 20))
        b = np.zeros((n, 4), dtype=np.uint64); b[:, 0] = np.random.default_rng(5).integers(0, 2, n).astype(np.uint64)
        run("%s binary 2^%d (std)" % (curve, lg), curve, n, b, pts, False, prof=(lg == 20))
n = 1 << 22
pts = zk.gen_points("bls12_381", 0x5A4B0002, n)
sc = zk.gen_fr("bls12_381", 0x5A4B0002, n)
run("bls12_381 2^22 c=16", "bls12_381", n, sc, pts, True, 16, 5, True)
run("bls12_381 2^22 c=17", "bls12_381", n, sc, pts, True, 17, 5, True)
PY
for v in new fine0 new fine0; do
  if [ $v = new ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"; timeout 150 python /tmp/ag.py 2>&1 || exit 1
done
unset ZK_LIB_PATH
