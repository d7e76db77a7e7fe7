"""Two host-buffer 2^24 NTTs into fresh (np.empty) outputs and two into a resident one, for a
rocprofv3 --kernel-trace --memory-copy-trace timeline (copies vs passes vs host gaps)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zikkurat-algebra_amd"))
import numpy as np  # noqa: E402
import zkalgebra as zk  # noqa: E402

m = 24
x = zk.gen_fr("bls12_381", 0x5A4B0003, 1 << m)
sg = zk.get_fft_subgroup("bls12_381", m)
g = sg.gen_array()
sym = zk.load().bls12_381_poly_mont_ntt_forward
res = np.ones_like(x)
sym(m, zk._p(g), zk._p(x), zk._p(res))
keep = []
for kind in ("fresh", "fresh", "resident", "resident"):
    b = np.empty_like(x) if kind == "fresh" else res
    keep.append(b)
    t = time.perf_counter()
    sym(m, zk._p(g), zk._p(x), zk._p(b))
    print(f"{kind}: {(time.perf_counter() - t) * 1e3:.2f} ms  t_end={time.perf_counter():.6f}", flush=True)
