# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# host arithmetic of finish_host on the box's CPU + MSM sizes (device-resident) on the final build
tools/microbench/host_chain
cat > /tmp/sz.py <<'PY'
import sys, time, os
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "zikkurat-algebra_amd"))
import zkalgebra as zk
for curve in ("bls12_381", "bn128"):
    for logn in (12, 14, 16, 18, 20, 22):
        n = 1 << logn
        ds, dp = zk.DeviceBuffer(zk.gen_fr(curve, 0x5A4B0002, n)), zk.DeviceBuffer(zk.gen_points(curve, 0x5A4B0002, n))
        zk.msm_device(curve, n, ds, dp); zk.load().zkg_device_synchronize()
        reps = 20 if logn < 21 else 5
        t = time.perf_counter()
        for _ in range(reps): zk.msm_device(curve, n, ds, dp)
        dt = (time.perf_counter() - t) / reps
        print(curve, logn, "%.4f ms" % (dt * 1e3), "%.3e pairs/s" % (n / dt), flush=True)
        ds.free(); dp.free()
PY
timeout 200 python /tmp/sz.py
