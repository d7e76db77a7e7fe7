"""Group FFT (G1 curve FFT, <C>_G1_proj_fft_forward / _inverse) timing at 2^m, device-resident
(zkg_g1_fft_device): python tools/fft_time.py [m] [reps]"""
import sys
import time

sys.path.insert(0, "zikkurat-algebra_amd")
import numpy as np  # noqa: E402
import zkalgebra as zk  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 16
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
lib = zk.load()
import ctypes  # noqa: E402
lib.zkg_g1_fft_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                  ctypes.c_void_p, ctypes.c_void_p]
for curve in ("bls12_381", "bn128"):
    n = 1 << m
    pts = zk.batch_from_affine(curve, zk.gen_points(curve, 0x5A4B0007, n))
    sg = zk.get_fft_subgroup(curve, m)
    g = sg.gen_array()
    d_in = zk.DeviceBuffer(pts)
    d_out = zk.DeviceBuffer.empty(pts.nbytes)
    out = {}
    for name, inv in (("forward", 0), ("inverse", 1)):
        lib.zkg_g1_fft_device(zk.CURVE_ID[curve], inv, m, zk._p(g), d_in.ptr, d_out.ptr)
        lib.zkg_device_synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            lib.zkg_g1_fft_device(zk.CURVE_ID[curve], inv, m, zk._p(g), d_in.ptr, d_out.ptr)
        lib.zkg_device_synchronize()
        out[name] = (time.perf_counter() - t) / reps * 1e3
    glv = zk.g1_fft_last_glv() if hasattr(zk, "g1_fft_last_glv") else "?"
    d_in.free()
    d_out.free()
    rt = ""
    if len(sys.argv) > 3 and sys.argv[3] == "check":  # round trip at this size (host buffers)
        f = zk.forward_fft(sg, pts)
        rt = ", round trip " + ("exact" if np.array_equal(zk.inverse_fft(sg, f), pts) else "MISMATCH")
    print(f"{curve} 2^{m} group FFT: forward {out['forward']:.2f} ms, inverse {out['inverse']:.2f} ms (glv {glv}){rt}",
          flush=True)
