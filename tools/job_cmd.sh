# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# export fused into the job sums (in-tree) vs the separate k_export kernel (variants/prev)
timeout 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread 2>&1 | tail -2
cat > /tmp/ab.py <<'PY'
import sys, time, os
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "zikkurat-algebra_amd"))
import zkalgebra as zk
for curve, logn in (("bls12_381", 20), ("bls12_381", 16), ("bn128", 20)):
    n = 1 << logn
    ds, dp = zk.DeviceBuffer(zk.gen_fr(curve, 0x5A4B0002, n)), zk.DeviceBuffer(zk.gen_points(curve, 0x5A4B0002, n))
    for _ in range(3): zk.msm_device(curve, n, ds, dp)
    t = time.perf_counter()
    for _ in range(20): zk.msm_device(curve, n, ds, dp)
    print(curve, logn, round((time.perf_counter() - t) / 20 * 1e3, 4), "ms", flush=True)
    ds.free(); dp.free()
PY
for v in prev new prev new; do
  if [ $v = new ]; then export ZK_LIB_PATH=; else export ZK_LIB_PATH=$PWD/variants/$v/libzkalgebra_gpu.so; fi
  echo "== $v"; timeout 120 python /tmp/ab.py
done
unset ZK_LIB_PATH
timeout 300 python -u -c "import __graft_entry__ as g; g.smoke()"
