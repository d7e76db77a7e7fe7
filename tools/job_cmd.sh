# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# (1) host-buffer MSM: per-split pipelines (scalars + points per split, own sort, no host sync;
#     up to 4 splits, in-tree) vs 1 split (variants/nosplit) vs at most 2 (variants/split2)
# (2) host-buffer NTT 2^24: staged device-to-host through pinned chunks (in-tree) vs prefault +
#     direct pageable copy (variants/nostage); outputs kept alive (no munmap inside the timing)
cat > /tmp/e2e.py <<'PY'
import sys, time, os
import numpy as np
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
    if logn == 20 and curve == "bls12_381":
        zk.msm_profile(True); zk.msm_affine(curve, sc, pts); zk.msm_affine(curve, sc, pts); zk.msm_profile(False)
m = 24; sg = zk.get_fft_subgroup("bls12_381", m); x = zk.gen_fr("bls12_381", 3, 1 << m)
y0 = zk.forward_ntt(sg, x)
keep = []
for _ in range(3):
    t = time.perf_counter(); y = zk.forward_ntt(sg, x); dt = time.perf_counter() - t
    assert np.array_equal(y, y0)
    keep.append(y)
    print("forward_ntt 2^24 fresh output %.2f ms" % (dt * 1e3), flush=True)
del keep
lib = zk.load(); r = np.ones_like(x)
for _ in range(3):
    t = time.perf_counter(); lib.bls12_381_poly_mont_ntt_forward(m, zk._p(sg.gen_array()), zk._p(x), zk._p(r)); dt = time.perf_counter() - t
    assert np.array_equal(r, y0)
    print("forward_ntt 2^24 resident output %.2f ms" % (dt * 1e3), flush=True)
PY
for v in nosplit new split2 nostage nosplit new split2 nostage; do
  if [ $v = new ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"; timeout 150 python /tmp/e2e.py || exit 1
done
unset ZK_LIB_PATH
