"""Chunked-inversion timings (GPU box): Fr vector inv / div at 2^24 (zkg arr, device-resident) and
G1 batch_to_affine at 2^16 / 2^20 (BLS12-381), 5 reps each after a warm-up:
    ZK_INV_LANES=... ZK_NORM_LANES=... python tools/inv_probe.py"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zikkurat-algebra_amd"))
import numpy as np  # noqa: E402
import zkalgebra as zk  # noqa: E402


def timeit(fn, reps=5):
    fn()
    zk.load().zkg_device_synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    zk.load().zkg_device_synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    zk.require_gpu()
    lib = zk.load()
    env = {k: os.environ.get(k, "default") for k in ("ZK_INV_LANES", "ZK_NORM_LANES")}
    res = {"env": env}
    n = 1 << 24
    a = zk.gen_fr("bls12_381", 11, n)
    b = zk.gen_fr("bls12_381", 12, n)
    da, db, dt = zk.DeviceBuffer(a), zk.DeviceBuffer(b), zk.DeviceBuffer.empty(a.nbytes)
    for op in ("inv", "div"):
        res[op + "_2^24_ms"] = timeit(lambda: zk.arr_op_device("bls12_381", op, n, da, db if op == "div" else None,
                                                               None, d_tgt=dt))
    lib.zkg_g1_batch_to_affine_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    for m in (16, 20):
        np_ = 1 << m
        proj = zk.batch_from_affine("bls12_381", zk.gen_points("bls12_381", 7, np_))
        dp = zk.DeviceBuffer(proj)
        dq = zk.DeviceBuffer.empty(np_ * 2 * 6 * 8)
        res[f"to_affine_2^{m}_ms"] = timeit(lambda: lib.zkg_g1_batch_to_affine_device(1, np_, dp.ptr, dq.ptr))
    print(res, flush=True)


if __name__ == "__main__":
    main()
