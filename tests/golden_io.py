"""Loading helpers for tests/golden (data only: numpy .npz without pickle, JSON)."""
import json
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def msm_cases(curve):
    z = np.load(os.path.join(GOLD, f"msm_{curve}.npz"), allow_pickle=False)
    for name in z["names"]:
        name = str(name)
        yield (name, z[f"{name}__scalars"], z[f"{name}__points"], bool(z[f"{name}__mont"][0]),
               z[f"{name}__affine"], z[f"{name}__proj_normalized"])


def ntt_cases(curve):
    z = np.load(os.path.join(GOLD, f"ntt_{curve}.npz"), allow_pickle=False)
    ms = sorted({int(k.split("__")[0][1:]) for k in z.files})
    for m in ms:
        yield m, z[f"m{m}__gen"], z[f"m{m}__input"], z[f"m{m}__forward"], z[f"m{m}__inverse"]


def baseline_configs():
    p = os.path.join(GOLD, "baseline_configs.json")
    return json.load(open(p)) if os.path.exists(p) else {}
