#!/usr/bin/env python3
"""Measurement of the SURVEY.md 8f rows (GPU box): Fr vector ops, division by a
vanishing polynomial, G1 batch_to_affine, G1 group FFT, G2 MSM.

Every GPU figure is device-resident (inputs already in HBM, hipDeviceSynchronize around
the timed loop); HBM rooflines use ALGORITHMIC bytes (operands read once + result written
once).  The reference's own C (oracle/_ref, 1 host core) is timed on a bounded sample of
the same workload for scale.  Prints one JSON object.

    python tools/bench_ext.py [--quick]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import zkalgebra as zk  # noqa: E402
from oracle.oracle import Reference  # noqa: E402

HBM = 8000.0  # GB/s, MI355X_MICROARCH.md
CURVE = "bls12_381"
# measured VALU issue ceiling: v_mad_u64_u32 lane-ops/s of the whole chip (profiles/r02_valu_ceiling.json)
VALU_SLOTS = 3.42e13


def isa_slots(key):
    """issue slots of one hot-loop iteration from the newest profiles/*_isa_<key>.json
    (tools/isa_profile.sh; per-lane GLV chain totals: tools/fft_isa.py), or None"""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_isa_{key}.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    return (d.get("hot_loop") or {}).get("issue_slots_per_iteration") or d.get("issue_slots_per_chain")


def timeit(fn, reps):
    fn()
    zk.load().zkg_device_synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    zk.load().zkg_device_synchronize()
    return (time.perf_counter() - t) / reps


def cpu_time(fn):
    t = time.perf_counter()
    fn()
    return time.perf_counter() - t


def hbm(bytes_, sec):
    gbs = bytes_ / sec / 1e9
    return {"bound": "hbm", "achieved": gbs, "peak": HBM, "unit": "GB/s", "frac": gbs / HBM}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    zk.require_gpu()
    ref = Reference() if Reference.available() else None
    out = {"curve": CURVE, "data": "synthetic (zk_gen.cpp generator; G2 points from the reference's generator)"}
    lib = zk.load()
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))

    # ---------------------------------------------------------------- Fr vector ops, 2^24
    m = 22 if args.quick else 24
    n = 1 << m
    a, b = zk.gen_fr(CURVE, 1, n), zk.gen_fr(CURVE, 2, n)
    da, db, dt = zk.DeviceBuffer(a), zk.DeviceBuffer(b), zk.DeviceBuffer.empty(a.nbytes)
    k = zk.gen_fr(CURVE, 3, 1)[0]
    arr = {}
    for op, nread, kw in (("add", 2, {}), ("mul", 2, {}), ("scale", 1, {"kA": k}), ("Ax_plus_y", 2, {"kA": k}),
                          ("inv", 1, {}), ("div", 2, {})):
        sec = timeit(lambda: zk.arr_op_device(CURVE, op, n, da, db if nread == 2 else None, None,
                                              d_tgt=dt, **kw), 5)
        arr[op] = {"n": n, "ms": sec * 1e3, "elems_per_s": n / sec, "roofline": hbm((nread + 1) * 32 * n, sec)}
    sec = timeit(lambda: lib.zkg_arr_powers_device(1, n, P(k), P(k), dt.ptr), 5)
    arr["powers"] = {"n": n, "ms": sec * 1e3, "elems_per_s": n / sec, "roofline": hbm(32 * n, sec)}
    res = np.zeros(4, np.uint64)
    sec = timeit(lambda: lib.zkg_arr_dot_device(1, n, da.ptr, db.ptr, P(res)), 5)
    arr["dot_prod"] = {"n": n, "ms": sec * 1e3, "elems_per_s": n / sec, "roofline": hbm(64 * n, sec)}
    if ref:
        s = 1 << 20
        w = np.zeros((s, 4), np.uint64)
        for op in ("mul", "inv"):
            args_ = (a[:s], b[:s]) if op == "mul" else (a[:s],)
            t = cpu_time(lambda: ref.arr(CURVE, "arr_mont_" + op, s, *args_, w))
            arr[op]["cpu_reference"] = {"elems_per_s": s / t, "cores": 1, "sample": f"2^20 elements, {op}"}
    out["fr_vector_ops"] = arr

    # ---------------------------------------------------------------- div_by_vanishing (PLONK-like)
    nv = 1 << (20 if args.quick else 22)
    poly = zk.gen_fr(CURVE, 4, 3 * nv)
    dp = zk.DeviceBuffer(poly)
    dq = zk.DeviceBuffer.empty(2 * nv * 32)
    dr = zk.DeviceBuffer.empty(nv * 32)
    eta = zk.gen_fr(CURVE, 5, 1)[0]
    lib.zkg_poly_div_by_vanishing_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                                     ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_void_p,
                                                     ctypes.c_int, ctypes.c_void_p]
    sec = timeit(lambda: lib.zkg_poly_div_by_vanishing_device(1, 3 * nv, dp.ptr, nv, P(eta), 2 * nv, dq.ptr, nv,
                                                              dr.ptr), 5)
    out["div_by_vanishing"] = {"deg": 3 * nv - 1, "n": nv, "ms": sec * 1e3,
                               "coeffs_per_s": 3 * nv / sec, "roofline": hbm((3 * nv + 3 * nv) * 32, sec)}
    for d in (dp, dq, dr, da, db, dt):
        d.free()

    # ---------------------------------------------------------------- G1 batch_to_affine, 2^20
    np_ = 1 << 20
    aff = zk.gen_points(CURVE, 6, np_)
    proj = zk.batch_from_affine(CURVE, aff)
    dpj, daf = zk.DeviceBuffer(proj), zk.DeviceBuffer.empty(aff.nbytes)
    lib.zkg_g1_batch_to_affine_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    sec = timeit(lambda: lib.zkg_g1_batch_to_affine_device(1, np_, dpj.ptr, daf.ptr), 5)
    out["g1_batch_to_affine"] = {"n": np_, "ms": sec * 1e3, "points_per_s": np_ / sec,
                                 "roofline": hbm((144 + 96) * np_, sec)}
    if ref:
        s = 1 << 14
        w = np.zeros((s, 12), np.uint64)
        t = cpu_time(lambda: ref.arr(CURVE, "G1_proj_batch_to_affine", s, proj[:s], w))
        out["g1_batch_to_affine"]["cpu_reference"] = {"points_per_s": s / t, "cores": 1, "sample": "2^14 points"}
    dpj.free()
    daf.free()

    # ---------------------------------------------------------------- G1 group FFT, size sweep
    lib.zkg_g1_fft_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.c_void_p, ctypes.c_void_p]
    fft = {}
    sizes = (12, 14) if args.quick else (12, 14, 16, 18, 20)
    for curve in ("bls12_381", "bn128"):
        cid = zk.CURVE_ID[curve]
        for fm in sizes:
            N = 1 << fm
            proj = zk.batch_from_affine(curve, zk.gen_points(curve, 7, N))
            sg = zk.get_fft_subgroup(curve, fm)
            ds, dd = zk.DeviceBuffer(proj), zk.DeviceBuffer.empty(proj.nbytes)
            g = sg.gen_array()
            chain = isa_slots(f"glv_chain_{curve}")
            row = {"plan_bits_per_stage": zk.g1_fft_plan(curve, fm) or [1] * fm}
            for name, inv, smuls in (("forward", 0, N // 2 * fm), ("inverse", 1, N * fm)):
                sec = timeit(lambda: lib.zkg_g1_fft_device(cid, inv, fm, P(g), ds.ptr, dd.ptr), 1 if fm >= 18 else 3)
                row[name] = {"ms": sec * 1e3, "points_per_s": N / sec, "scalar_muls": smuls,
                             "scalar_muls_per_s": smuls / sec, "glv": bool(zk.g1_fft_last_glv())}
                if chain and row[name]["glv"]:
                    pm = zk.g1_fft_glv_products(curve, fm, inverse=bool(inv))
                    iss = pm * 2 * chain / sec  # two lanes (a GLV pair) per product
                    row[name]["valu_roofline"] = {
                        "bound": "valu_issue", "glv_pair_products": pm, "issue_slots_per_lane_chain": chain,
                        "achieved": iss, "peak": VALU_SLOTS, "unit": "issue slots/s", "frac": iss / VALU_SLOTS,
                        "note": "scalar-multiplication chains only (additions, loads, sums, normalisation not "
                                "counted); below 2^15 a stage is latency-bound by construction (fewer lanes than "
                                "one wavefront per SIMD)"}
            fft[f"{curve}_2^{fm}"] = row
            ds.free()
            dd.free()
    if ref:
        cm = 8
        sg8 = zk.get_fft_subgroup(CURVE, cm)
        small = zk.batch_from_affine(CURVE, zk.gen_points(CURVE, 7, 1 << cm))
        w = np.zeros_like(small)
        t = cpu_time(lambda: ref.arr(CURVE, "G1_proj_fft_forward", cm, sg8.gen_array(), small, w))
        fft["cpu_reference"] = {"scalar_muls_per_s": (1 << cm) // 2 * cm / t, "cores": 1,
                                "sample": "BLS12-381 2^8-point forward FFT"}
    out["g1_group_fft"] = fft

    # ---------------------------------------------------------------- G2 MSM, both curves
    # DISTINCT points (verdict r05 item 1): P0 + i H over the reference's own G2 arithmetic
    # (golden_io.g2_points), so the large-window sort and the Y sums see real bucket occupancy
    import golden_io
    lib.zkg_g2_msm_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    out["g2_msm"] = {}
    for curve in ("bls12_381", "bn128"):
        if not ref:
            break
        gms = (16,) if args.quick else (18, 20)
        t0 = time.perf_counter()
        allpts = golden_io.g2_points(ref.lib, curve, 1 << max(gms))
        gen_s = time.perf_counter() - t0
        slots = isa_slots(f"k_accum_{curve}_g2")
        for gm in gms:
            ng = 1 << gm
            pts = np.ascontiguousarray(allpts[:ng])
            sc = zk.gen_fr(curve, 8, ng)
            dsc, dpt = zk.DeviceBuffer(sc), zk.DeviceBuffer(pts)
            res = np.zeros(36, np.uint64)
            sec = timeit(lambda: lib.zkg_g2_msm_device(zk.CURVE_ID[curve], ng, dsc.ptr, 4, 1, dpt.ptr, P(res), 0), 3)
            c = lib.zkg_msm_default_window(ng)
            W = (255 if curve == "bls12_381" else 254) // c + 1
            g2 = {"n": ng, "ms": sec * 1e3, "pairs_per_s": ng / sec, "window": c, "windows": W,
                  "hbm_fraction": hbm((32 + 4 * 8 * zk.NLIMBS_P[curve]) * ng, sec)["frac"],
                  "note": f"{ng} distinct reference-generated G2 points (generated in {gen_s:.0f} s on the host)"}
            if slots:
                madds = W * ng  # one Fp2 mixed add per (window, pair) in the accumulation
                iss = madds * slots / sec
                g2["valu_roofline"] = {"bound": "valu_issue", "madds": madds, "issue_slots_per_madd": slots,
                                       "achieved": iss, "peak": VALU_SLOTS, "unit": "issue slots/s",
                                       "frac": iss / VALU_SLOTS,
                                       "note": "the accumulation's madds x its ISA slot count over the WHOLE "
                                               "MSM time (sort, Y sums and the tail included): a lower bound "
                                               "on the accumulation kernel's own issue fraction"}
            if gm == gms[0]:
                s_ = 1 << 12
                w = np.zeros(4 * zk.NLIMBS_P[curve], np.uint64)
                t = cpu_time(lambda: ref.arr(curve, "G2_proj_MSM_mont_coeff_affine_out", s_, sc[:s_], pts[:s_], w, 4))
                g2["cpu_reference"] = {"pairs_per_s": s_ / t, "cores": 1, "sample": "first 2^12 pairs"}
            out["g2_msm"][f"{curve}_2^{gm}"] = g2
            dsc.free()
            dpt.free()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
