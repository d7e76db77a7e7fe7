"""G2 MSM timing, device-resident (GPU box; A/B of variant builds via ZK_LIB_PATH):
    python tools/g2_time.py [curve ...]
2^18 / 2^20 DISTINCT reference-generated G2 points (golden_io.g2_points, as tools/bench_ext.py since
round 6), 3 reps after a warm-up; prints ms and a digest of the projective result."""
import ctypes
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "zikkurat-algebra_amd"), os.path.join(ROOT, "tests"), ROOT):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import zkalgebra as zk  # noqa: E402
from oracle.oracle import Reference  # noqa: E402
import golden_io  # noqa: E402


def main():
    zk.require_gpu()
    lib = zk.load()
    lib.zkg_g2_msm_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    ref = Reference()
    for curve in sys.argv[1:] or ("bn128", "bls12_381"):
        allpts = golden_io.g2_points(ref.lib, curve, 1 << 20)
        for gm in (18, 20):
            ng = 1 << gm
            pts = np.ascontiguousarray(allpts[:ng])
            sc = zk.gen_fr(curve, 8, ng)
            dsc, dpt = zk.DeviceBuffer(sc), zk.DeviceBuffer(pts)
            res = np.zeros(36, np.uint64)
            call = lambda: lib.zkg_g2_msm_device(zk.CURVE_ID[curve], ng, dsc.ptr, 4, 1, dpt.ptr,
                                                 res.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 0)
            call()
            t = time.perf_counter()
            for _ in range(3):
                call()
            ms = (time.perf_counter() - t) / 3 * 1e3
            print(f"{curve} G2 2^{gm}: {ms:7.3f} ms  result {hashlib.sha256(res.tobytes()).hexdigest()[:16]}", flush=True)
            dsc.free()
            dpt.free()


if __name__ == "__main__":
    main()
