"""Tiny group-FFT probe (one call per line, flushed): python tools/fft_probe.py curve m direction"""
import sys
import time

sys.path.insert(0, "zikkurat-algebra_amd")
import zkalgebra as zk  # noqa: E402

curve, m, d = sys.argv[1], int(sys.argv[2]), sys.argv[3]
n = 1 << m
pts = zk.batch_from_affine(curve, zk.gen_points(curve, 0x77, n))
sg = zk.get_fft_subgroup(curve, m)
t = time.perf_counter()
out = zk.forward_fft(sg, pts) if d == "fwd" else zk.inverse_fft(sg, pts)
print(curve, m, d, "%.2f ms" % ((time.perf_counter() - t) * 1e3), int(out[0][0]) & 0xffff, flush=True)
