#!/usr/bin/env python3
"""MSM timing helpers for the GPU box.
   python tools/sweep_window.py bls12_381 20 13 14 15 16 17   # device-resident MSM per window size
   python tools/sweep_window.py phases                          # per-phase profile at several sizes
"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
import zkalgebra as zk  # noqa: E402


def run(curve, logn, windows, reps=5, profile=False):
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
        zk.msm_profile(profile)
        zk.timer(enable=True, reset=True)
        t = time.perf_counter()
        for _ in range(reps):
            zk.msm_device(curve, n, ds, dp, window=c)
        dt = (time.perf_counter() - t) / reps
        kms, kn = zk.timer(enable=False)
        zk.msm_profile(False)
        print(f"{curve} 2^{logn} c={c or zk.load().zkg_msm_window(zk.CURVE_ID[curve], n, 4, 1)}: {dt*1e3:.3f} ms/msm "
              f"({n/dt:.3e} pairs/s), accum {kms/kn:.3f} ms, result {hashlib.sha256(r.tobytes()).hexdigest()[:12]}",
              flush=True)
    ds.free()
    dp.free()


if __name__ == "__main__":
    if sys.argv[1] == "phases2":  # last phase line + the timing line per size
        import contextlib, io
        for curve, logn in (("bls12_381", 20), ("bls12_381", 16), ("bn128", 20)):
            run(curve, logn, [0], reps=4, profile=True)
    elif sys.argv[1] == "phases":
        for curve, logn in (("bls12_381", 20), ("bn128", 20), ("bls12_381", 16), ("bls12_381", 14),
                            ("bls12_381", 23)):
            run(curve, logn, [0], reps=4, profile=True)
    else:
        run(sys.argv[1], int(sys.argv[2]), [int(x) for x in sys.argv[3:]] or [0])
