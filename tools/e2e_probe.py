"""Host-buffer MSM (the reference symbol bls12_381_G1_proj_MSM_mont_coeff_affine_out) at 2^20:
wall time per call and, with --phases, the library's per-phase event profile (stderr).  Run
under rocprofv3 --kernel-trace --memory-copy-trace for the copy / kernel timeline."""
import sys
import time

sys.path.insert(0, "zikkurat-algebra_amd")
import zkalgebra as zk  # noqa: E402

curve = sys.argv[1] if len(sys.argv) > 1 else "bls12_381"
lg = int(sys.argv[2]) if len(sys.argv) > 2 else 20
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
n = 1 << lg
sc = zk.gen_fr(curve, 0x5A4B0002, n)
pts = zk.gen_points(curve, 0x5A4B0002, n)
zk.msm_affine(curve, sc, pts)
ts = []
for _ in range(reps):
    t = time.perf_counter()
    zk.msm_affine(curve, sc, pts)
    ts.append((time.perf_counter() - t) * 1e3)
print(f"{curve} 2^{lg} host-buffer msm_affine ms: min {min(ts):.3f} median {sorted(ts)[len(ts)//2]:.3f}", flush=True)
if "--phases" in sys.argv:
    zk.msm_profile(True)
    for _ in range(3):
        zk.msm_affine(curve, sc, pts)
    zk.msm_profile(False)
