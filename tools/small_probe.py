#!/usr/bin/env python3
"""Device-resident MSM calls separated by idle gaps, for a kernel trace of the small-input tail:
   rocprofv3 --kernel-trace --memory-copy-trace -d DIR -- python3 tools/small_probe.py bls12_381 10 [reps]
   python tools/trace_timeline.py DIR idle      # timeline of the last call"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
import zkalgebra as zk  # noqa: E402

curve, logn = sys.argv[1], int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
n = 1 << logn
sc, pts = zk.gen_fr(curve, 0x5A4B0002, n), zk.gen_points(curve, 0x5A4B0002, n)
ds, dp = zk.DeviceBuffer(sc), zk.DeviceBuffer(pts)
ref = zk.msm_device(curve, n, ds, dp)
ts = []
for _ in range(reps):
    time.sleep(0.003)  # idle gap: the trace tool splits the calls on it
    t = time.perf_counter()
    r = zk.msm_device(curve, n, ds, dp)
    ts.append(time.perf_counter() - t)
    assert (r == ref).all()
if os.environ.get("ZK_PROBE_PHASES") == "1":  # per-phase events of three more calls (stderr)
    zk.msm_profile(True)
    for _ in range(3):
        zk.msm_device(curve, n, ds, dp)
    zk.msm_profile(False)
ts.sort()
print(f"{curve} 2^{logn}: median {ts[len(ts) // 2] * 1e3:.3f} ms, min {ts[0] * 1e3:.3f} ms over {reps} calls", flush=True)
