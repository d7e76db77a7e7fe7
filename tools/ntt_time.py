#!/usr/bin/env python3
"""Device-resident NTT timing for A/B runs on the GPU box (ZK_LIB_PATH selects a build):
   python tools/ntt_time.py [log_n] [reps] [max_radix]   (max_radix 12: two-pass schedule, 8: three passes)
Prints forward / inverse ms per transform, the forward output's SHA-256 against the
reference digest at 2^24 (tests/golden/baseline_configs.json) and the round-trip check."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
import numpy as np  # noqa: E402
import zkalgebra as zk  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 24
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
if len(sys.argv) > 3:
    zk.ntt_set_max_radix(int(sys.argv[3]))
curve = "bls12_381"
n = 1 << m
x = zk.gen_fr(curve, 0x5A4B0003, n)
g = zk.get_fft_subgroup(curve, m).gen_array()
d_x, d_f, d_i = zk.DeviceBuffer(x), zk.DeviceBuffer.empty(x.nbytes), zk.DeviceBuffer.empty(x.nbytes)
zk.ntt_device(curve, m, g, d_x, d_f)
zk.ntt_device(curve, m, g, d_f, d_i, inverse=True)
out = {"m": m, "max_radix": int(sys.argv[3]) if len(sys.argv) > 3 else 12}
for name, src, dst, inv in (("fwd", d_x, d_f, False), ("inv", d_f, d_i, True)):
    zk.load().zkg_device_synchronize()
    zk.timer(enable=True, reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        zk.ntt_device(curve, m, g, src, dst, inverse=inv)
    zk.load().zkg_device_synchronize()
    dt = (time.perf_counter() - t0) / reps
    kms, kn = zk.timer(enable=False)
    out[name] = round(dt * 1e3, 4)
    out[name + "_kernel"] = round(kms / kn, 4)
f = d_f.to_host(x)
cfg = json.load(open(os.path.join(ROOT, "tests", "golden", "baseline_configs.json"))).get("config3_bls12_381_ntt_2^24")
out["sha_ok"] = hashlib.sha256(f.tobytes()).hexdigest() == cfg["forward_sha256"] if m == 24 else None
out["roundtrip"] = bool(np.array_equal(d_i.to_host(x), x))
print(json.dumps(out), flush=True)
