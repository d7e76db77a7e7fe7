#!/usr/bin/env python3
"""Fr vector ops at 2^m (default 24), device-resident (zkg_arr_op_device / _dot / _powers): ms and
achieved algorithmic TB/s per op, BLS12-381 and BN128.  python tools/arr_time.py [m] [reps]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
import zkalgebra as zk  # noqa: E402
import numpy as np  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 24
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
n = 1 << m
lib = zk.load()
P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))  # noqa: E731


def timeit(fn):
    fn()
    lib.zkg_device_synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    lib.zkg_device_synchronize()
    return (time.perf_counter() - t) / reps


out = {}
for curve in ("bls12_381", "bn128"):
    cid = zk.CURVE_ID[curve]
    a, b, c = zk.gen_fr(curve, 1, n), zk.gen_fr(curve, 2, n), zk.gen_fr(curve, 6, n)
    da, db, dc, dt = zk.DeviceBuffer(a), zk.DeviceBuffer(b), zk.DeviceBuffer(c), zk.DeviceBuffer.empty(a.nbytes)
    k = zk.gen_fr(curve, 3, 1)[0]
    r = {}
    for op, nread, kw in (("add", 2, {}), ("sub", 2, {}), ("mul", 2, {}), ("sqr", 1, {}), ("scale", 1, {"kA": k}),
                          ("Ax_plus_y", 2, {"kA": k}), ("Ax_plus_By", 2, {"kA": k, "kB": k}),
                          ("mul_add", 3, {}), ("copy", 1, {}), ("inv", 1, {}), ("div", 2, {})):
        d3 = dc if nread == 3 else None
        sec = timeit(lambda: zk.arr_op_device(curve, op, n, da, db if nread >= 2 else None, d3, d_tgt=dt, **kw))
        r[op] = {"ms": round(sec * 1e3, 4), "TBps": round((nread + 1) * 32 * n / sec / 1e12, 3)}
    sec = timeit(lambda: lib.zkg_arr_powers_device(cid, n, P(k), P(k), dt.ptr))
    r["powers"] = {"ms": round(sec * 1e3, 4), "TBps": round(32 * n / sec / 1e12, 3)}
    res = np.zeros(4, np.uint64)
    sec = timeit(lambda: lib.zkg_arr_dot_device(cid, n, da.ptr, db.ptr, P(res)))
    r["dot_prod"] = {"ms": round(sec * 1e3, 4), "TBps": round(64 * n / sec / 1e12, 3)}
    for d in (da, db, dc, dt):
        d.free()
    out[curve] = r
    print(curve, f"2^{m}", json.dumps(r), flush=True)
