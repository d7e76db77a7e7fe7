#!/usr/bin/env python3
"""Dump G2 MSM outputs for several n (A/B of env-selected code paths; GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import zkalgebra as zk  # noqa: E402
from oracle.oracle import Reference  # noqa: E402
from test_gpu_g2 import g2_points  # noqa: E402

ref = Reference()
out = {}
for curve in ("bn128", "bls12_381"):
    pts_all = g2_points(ref, curve, 300)
    for n in list(range(1, 40)) + [100, 300]:
        sc = zk.gen_fr(curve, 500 + n, n)
        for rep in range(2):
            out[f"{curve}_{n}_{rep}"] = zk.g2_msm(curve, sc, pts_all[:n].copy(), affine=True)
np.savez(sys.argv[1], **out)
