# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# MSM sizes 2^10..2^22 with the round-3 window table and chunk floor (device-resident, 20 reps,
# 2 rounds), phase profiles at 2^14 / 2^16 / 2^20
cat > /tmp/sz.py <<'PY'
import sys, time, os
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "zikkurat-algebra_amd"))
import zkalgebra as zk
data = {}
for curve in ("bls12_381", "bn128"):
    for logn in range(10, 23):
        n = 1 << logn
        sc, pts = zk.gen_fr(curve, 0x5A4B0002, n), zk.gen_points(curve, 0x5A4B0002, n)
        data[(curve, logn)] = (zk.DeviceBuffer(sc), zk.DeviceBuffer(pts))
for rnd in range(2):
    for (curve, logn), (ds, dp) in data.items():
        n = 1 << logn
        zk.msm_device(curve, n, ds, dp); zk.load().zkg_device_synchronize()
        reps = 20 if logn < 21 else 5
        t = time.perf_counter()
        for _ in range(reps): zk.msm_device(curve, n, ds, dp)
        dt = (time.perf_counter() - t) / reps
        print(rnd, curve, logn, "%.4f ms" % (dt * 1e3), "%.3e pairs/s" % (n / dt), flush=True)
for logn in (14, 16, 20):
    ds, dp = data[("bls12_381", logn)]
    zk.msm_profile(True); zk.msm_device("bls12_381", 1 << logn, ds, dp); zk.msm_device("bls12_381", 1 << logn, ds, dp); zk.msm_profile(False)
PY
timeout 300 python /tmp/sz.py
