#!/usr/bin/env python3
"""Division by x^n - eta at bench_ext's size (deg 3n - 1, n = 2^m, default m = 22), device-resident,
BLS12-381: wall ms per call (run under rocprofv3 --kernel-trace --stats for the per-kernel split).
python tools/vanish_probe.py [m] [reps]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
import zkalgebra as zk  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 22
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
nv = 1 << m
lib = zk.load()
poly = zk.gen_fr("bls12_381", 4, 3 * nv)
dp, dq, dr = zk.DeviceBuffer(poly), zk.DeviceBuffer.empty(2 * nv * 32), zk.DeviceBuffer.empty(nv * 32)
eta = zk.gen_fr("bls12_381", 5, 1)[0]
f = lib.zkg_poly_div_by_vanishing_device
f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int,
              ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
P = eta.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
call = lambda: f(1, 3 * nv, dp.ptr, nv, P, 2 * nv, dq.ptr, nv, dr.ptr)  # noqa: E731
call()
lib.zkg_device_synchronize()
ts = []
for _ in range(reps):
    t = time.perf_counter()
    call()
    lib.zkg_device_synchronize()
    ts.append((time.perf_counter() - t) * 1e3)
ts.sort()
print(f"div_by_vanishing deg {3 * nv - 1} n 2^{m}: min {ts[0]:.4f} median {ts[len(ts) // 2]:.4f} ms "
      f"({6 * nv * 32 / ts[len(ts) // 2] / 1e9:.2f} TB/s algorithmic)", flush=True)
