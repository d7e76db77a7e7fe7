"""Reentrancy / thread safety of the drop-in boundary (SURVEY.md 8b "Threading": Haskell
`unsafe` ccalls from several capabilities may run concurrently; the reference is reentrant,
bls12_381_G1_proj.c:507-587 keeps only malloc'd locals).  Four host threads call the
reference-named MSM and NTT symbols on both curves at the same time (ctypes releases the
GIL for the foreign call) and every result must equal the reference-generated golden output."""
import threading

import numpy as np
import pytest

from golden_io import msm_cases, ntt_cases

pytestmark = pytest.mark.gpu


def test_concurrent_msm_and_ntt_calls(gpu):
    work = []
    for curve in ("bn128", "bls12_381"):
        for name, sc, pts, mont, aff, _ in msm_cases(curve):
            if sc.shape[0] >= 64:
                work.append(("msm", curve, name, sc, pts, mont, aff))
        for m, gen, x, fwd, inv in ntt_cases(curve):
            if m >= 5:
                work.append(("ntt", curve, m, gen, x, fwd, inv))
    errors = []

    def run(tid):
        try:
            for rep in range(3):
                for k, item in enumerate(work):
                    if (k + tid + rep) % 2:  # threads interleave different calls
                        continue
                    if item[0] == "msm":
                        _, curve, name, sc, pts, mont, aff = item
                        got = gpu.msm_affine(curve, sc, pts, std=not mont)
                        if not np.array_equal(got, aff):
                            errors.append(f"thread {tid}: msm {curve} {name}")
                    else:
                        _, curve, m, gen, x, fwd, inv = item
                        sg = gpu.FFTSubgroup(curve, tuple(int(v) for v in gen), m)
                        if not np.array_equal(gpu.forward_ntt(sg, x), fwd):
                            errors.append(f"thread {tid}: ntt {curve} m={m}")
                        if not np.array_equal(gpu.inverse_ntt(sg, x), inv):
                            errors.append(f"thread {tid}: intt {curve} m={m}")
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(f"thread {tid}: {e!r}")

    gpu.timer(enable=True, reset=True)  # the per-device kernel timer must stay consistent too
    threads = [threading.Thread(target=run, args=(t,)) for t in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    ms, launches = gpu.timer(enable=False)
    assert not any(t.is_alive() for t in threads), "a thread hung"
    assert not errors, errors[:10]
    assert launches > 0 and ms > 0
