#!/usr/bin/env python3
"""Time the device-resident MSM for several window sizes (GPU box):
   python tools/sweep_window.py bls12_381 20 13 14 15 16 17"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
import zkalgebra as zk  # noqa: E402

curve, logn = sys.argv[1], int(sys.argv[2])
windows = [int(x) for x in sys.argv[3:]] or [0]
n = 1 << logn
sc = zk.gen_fr(curve, 0x5A4B0002, n)
pts = zk.gen_points(curve, 0x5A4B0002, n)
ds, dp = zk.DeviceBuffer(sc), zk.DeviceBuffer(pts)
ref = None
for c in windows:
    r = zk.msm_device(curve, n, ds, dp, window=c)
    if ref is None:
        ref = r
    assert (r == ref).all(), c
    zk.load().zkg_device_synchronize()
    zk.timer(enable=True, reset=True)
    reps = 5
    t = time.perf_counter()
    for _ in range(reps):
        zk.msm_device(curve, n, ds, dp, window=c)
    dt = (time.perf_counter() - t) / reps
    kms, kn = zk.timer(enable=False)
    print(f"{curve} 2^{logn} c={c or zk.load().zkg_msm_default_window(n)}: {dt*1e3:.3f} ms/msm "
          f"({n/dt:.3e} pairs/s), accum {kms/kn:.3f} ms", flush=True)
