#!/usr/bin/env python3
"""Generate the golden parity fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

The reference ships no golden vectors for MSM/NTT (its tests are
unseeded random properties), so the expected outputs here are produced by running the
reference's own generated C (oracle/_ref/libzkref.so, built in place from
/root/reference/lib/cbits by oracle/Makefile) on deterministic inputs.  Inputs come from
the documented synthetic-input generator (zikkurat-algebra_amd/csrc/zk_gen.cpp; an
independent restatement in oracle/zk_oracle.c is checked equal by the tests).

  python tools/make_golden.py small     # edge-case MSM + NTT vectors (stored in full)  ~1 min
  python tools/make_golden.py large     # BASELINE-config outputs / SHA-256 digests     ~10 min, 8 cores
  python tools/make_golden.py groupfft  # group FFT at KZG SRS sizes (m = 12, 14, both curves, subgroup
                                        # points with random Z; BLS12-381 non-subgroup points at m = 10):
                                        # reference forward / inverse SHA-256 digests
                                        # -> tests/golden/group_fft.json      ~1 min, 8 cores
  python tools/make_golden.py groupfft m16  # only the keys containing "m16" (others kept)
  python tools/make_golden.py g2large   # G2 MSM at 2^16 / 2^18 (distinct points, infinities, zero
                                        # scalars), both curves -> tests/golden/g2_msm.json   ~2 min
  python tools/make_golden.py patterns  # adversarial NTT inputs (tests/golden_io.py NTT_PATTERNS) at
                                        # m = 5, 12, 14, 20 and random 2^20 vectors: reference forward /
                                        # inverse SHA-256 digests -> tests/golden/ntt_patterns.json   ~1 min

Only this script (in this container, where /root/reference exists) runs the reference;
the GPU box only reads the committed .npz/.json files.
"""
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
GOLD = os.path.join(ROOT, "tests", "golden")

from oracle.oracle import Reference, Oracle  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_io  # noqa: E402  (pattern definitions shared with the tests)
import zkalgebra as zk  # noqa: E402  (host-only functions: generator, fft generator)

R_ORDER = {
    "bn128": 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001,
    "bls12_381": 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
}
FLD_FR = {"bn128": 1, "bls12_381": 3}


def limbs(x, n=4):
    return np.array([(x >> (64 * i)) & ((1 << 64) - 1) for i in range(n)], dtype=np.uint64)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ----------------------------------------------------------------------------- small fixtures

def msm_cases(curve):
    """Edge cases the reference's semantics define."""
    o = Oracle()
    NP = zk.NLIMBS_P[curve]
    r = R_ORDER[curve]
    cases = []
    for n in (1, 2, 3, 17, 64, 1000, 4096):
        cases.append((f"random_n{n}", zk.gen_fr(curve, 100 + n, n), zk.gen_points(curve, 200 + n, n), True))
    # std-coefficient variants of the same data (to_std of the Montgomery scalars)
    for n in (17, 1000):
        sc = zk.gen_fr(curve, 100 + n, n)
        cases.append((f"std_n{n}", o.to_std(FLD_FR[curve], sc.copy()), zk.gen_points(curve, 200 + n, n), False))
    n = 64
    pts = zk.gen_points(curve, 7, n)
    sc = zk.gen_fr(curve, 8, n)
    z = sc.copy(); z[::3] = 0
    cases.append(("zero_scalars", z, pts, True))
    cases.append(("all_zero", np.zeros_like(sc), pts, True))
    top = np.tile(limbs(r - 1), (n, 1))
    cases.append(("std_r_minus_1", top.copy(), pts, False))
    full = np.full((n, 4), np.uint64(0xFFFFFFFFFFFFFFFF))
    cases.append(("std_2pow256_minus_1", full, pts, False))
    eq = np.tile(sc[0], (n, 1))
    cases.append(("all_equal_scalars", eq, pts, True))
    dup = np.tile(pts[0], (n, 1))
    cases.append(("duplicate_points", sc.copy(), dup, True))
    # P and -P with equal scalars -> cancels (negate y: p - y)
    neg = pts.copy()
    pfield = {"bn128": 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47,
              "bls12_381": 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB}[curve]
    for i in range(n):
        y = sum(int(neg[i, NP + j]) << (64 * j) for j in range(NP))
        neg[i, NP:] = limbs((pfield - y) % pfield, NP)
    pm = np.concatenate([pts[:32], neg[:32]])
    cs = np.concatenate([sc[:32], sc[:32]])
    cases.append(("p_and_minus_p", cs, pm, True))
    infp = pts.copy(); infp[5:40:4] = np.uint64(0xFFFFFFFFFFFFFFFF)
    cases.append(("infinity_points", sc.copy(), infp, True))
    allinf = np.full_like(pts, np.uint64(0xFFFFFFFFFFFFFFFF))
    cases.append(("all_infinity", sc.copy(), allinf, True))
    small = np.zeros_like(sc); small[:, 0] = np.arange(1, n + 1, dtype=np.uint64)
    cases.append(("std_small_scalars", small, pts, False))
    one_limb = zk.gen_fr(curve, 9, 200)[:, :1].copy()
    cases.append(("std_one_limb", one_limb, zk.gen_points(curve, 10, 200), False))
    return cases


def make_small():
    os.makedirs(GOLD, exist_ok=True)
    ref = Reference()
    for curve in zk.CURVES:
        arrays = {}
        names = []
        t = time.time()
        for name, sc, pts, mont in msm_cases(curve):
            sc = np.ascontiguousarray(sc, dtype=np.uint64)
            pts = np.ascontiguousarray(pts, dtype=np.uint64)
            aff = ref.msm(curve, sc, pts, mont=mont, out="affine")
            proj = ref.msm(curve, sc, pts, mont=mont, out="proj")
            names.append(name)
            arrays[f"{name}__scalars"] = sc
            arrays[f"{name}__points"] = pts
            arrays[f"{name}__mont"] = np.array([1 if mont else 0], dtype=np.uint64)
            arrays[f"{name}__affine"] = aff
            arrays[f"{name}__proj_normalized"] = ref.normalize(curve, proj)
        np.savez_compressed(os.path.join(GOLD, f"msm_{curve}.npz"), names=np.array(names), **arrays)
        print(curve, "msm fixtures", len(names), "%.1fs" % (time.time() - t))
        # NTT
        arrays = {}
        for m in (0, 1, 2, 3, 5, 8, 10, 12):
            g = zk.get_fft_subgroup(curve, m).gen_array()
            x = zk.gen_fr(curve, 300 + m, 1 << m)
            f = ref.ntt(curve, m, g, x)
            i = ref.ntt(curve, m, g, x, inverse=True)
            arrays[f"m{m}__input"] = x
            arrays[f"m{m}__gen"] = g
            arrays[f"m{m}__forward"] = f
            arrays[f"m{m}__inverse"] = i
        np.savez_compressed(os.path.join(GOLD, f"ntt_{curve}.npz"), **arrays)
        print(curve, "ntt fixtures")


# ----------------------------------------------------------------------------- large (BASELINE configs)

def _shard_msm(args):
    curve, seed, lo, hi, mont = args
    sc = zk.gen_fr(curve, seed, hi - lo, start=lo)
    if not mont:
        sc = Oracle().to_std(FLD_FR[curve], sc)
    pts = zk.gen_points(curve, seed, hi - lo, start=lo)
    ref = Reference()
    t = time.time()
    p = ref.msm(curve, sc, pts, mont=mont, out="proj")
    return p, time.time() - t


def large_msm(curve, logn, seed, shards):
    n = 1 << logn
    step = n // shards
    # the reference's Montgomery entry aborts at 2^26 (int overflow, G1_proj.c:631-632): use the
    # std entry on to_std'd scalars there -- same mathematical input.
    mont = logn < 26
    with mp.Pool(min(shards, 8)) as pool:
        parts = pool.map(_shard_msm, [(curve, seed, k * step, (k + 1) * step, mont) for k in range(shards)])
    ref = Reference()
    acc = parts[0][0]
    for p, _ in parts[1:]:
        acc = ref.proj_add(curve, acc, p)
    aff = ref.to_affine(curve, acc)
    cpu_s = sum(t for _, t in parts)
    return {"curve": curve, "log_n": logn, "seed": seed, "affine": [int(x) for x in aff],
            "reference_cpu_seconds_sum_over_shards": cpu_s, "shards": shards,
            "reference_entry": "MSM_mont_coeff_proj_out" if mont else "MSM_std_coeff_proj_out (to_std scalars)"}


def _shard_skew(args):
    curve, seed, kind, n, lo, hi = args
    sc = golden_io.skew_scalars(zk.gen_fr, curve, seed, n, kind)[lo:hi].copy()
    pts = zk.gen_points(curve, seed, hi - lo, start=lo)
    ref = Reference()
    t = time.time()
    p = ref.msm(curve, sc, pts, mont=True, out="proj")
    return p, time.time() - t


def large_skew_msm(curve, logn, seed, kind, shards=8):
    n = 1 << logn
    step = n // shards
    with mp.Pool(min(shards, 8)) as pool:
        parts = pool.map(_shard_skew, [(curve, seed, kind, n, k * step, (k + 1) * step) for k in range(shards)])
    ref = Reference()
    acc = parts[0][0]
    for p, _ in parts[1:]:
        acc = ref.proj_add(curve, acc, p)
    aff = ref.to_affine(curve, acc)
    return {"curve": curve, "log_n": logn, "seed": seed, "kind": kind, "affine": [int(x) for x in aff],
            "reference_cpu_seconds_sum_over_shards": sum(t for _, t in parts), "shards": shards,
            "reference_entry": "MSM_mont_coeff_proj_out (shards added with proj_add)"}


# ----------------------------------------------------------------------------- adversarial NTT patterns

PATTERN_SIZES = (5, 12, 14, 20)
RANDOM_SEED = 0x5A4B0003


def _pattern_job(args):
    curve, name, m, inverse = args
    ref = Reference()
    g = zk.get_fft_subgroup(curve, m).gen_array()
    x = zk.gen_fr(curve, RANDOM_SEED, 1 << m) if name == "random" else golden_io.ntt_pattern(curve, name, m)
    t = time.time()
    y = ref.ntt(curve, m, g, x, inverse=inverse)
    dt = time.time() - t
    closed = None if name == "random" else golden_io.check_pattern_output(curve, name, m, inverse, y)
    return (f"{curve}/{name}/m{m}/{'inverse' if inverse else 'forward'}",
            {"sha256": sha(y), "input_sha256": sha(x), "first": [int(v) for v in y[0]],
             "reference_closed_form_ok": closed, "reference_seconds": dt})


def make_patterns():
    jobs = [(c, nm, m, inv) for c in zk.CURVES for nm in golden_io.NTT_PATTERNS for m in PATTERN_SIZES
            for inv in (False, True)]
    jobs += [(c, "random", 20, inv) for c in zk.CURVES for inv in (False, True)]
    with mp.Pool(8) as pool:
        res = dict(pool.map(_pattern_job, jobs))
    bad = [k for k, v in res.items() if v["reference_closed_form_ok"] is False]
    assert not bad, f"the reference disagrees with the closed forms: {bad}"
    out = {"generator": "tools/make_golden.py patterns (reference lib/cbits, oracle/_ref)",
           "random_seed": RANDOM_SEED, "cases": res}
    json.dump(out, open(os.path.join(GOLD, "ntt_patterns.json"), "w"), indent=1, sort_keys=True)
    print(len(res), "pattern digests;", sum(1 for v in res.values() if v["reference_closed_form_ok"]),
          "also match the closed forms")


def large_ntt(curve, logn, seed):
    ref = Reference()
    g = zk.get_fft_subgroup(curve, logn).gen_array()
    x = zk.gen_fr(curve, seed, 1 << logn)
    t = time.time()
    f = ref.ntt(curve, logn, g, x)
    tf = time.time() - t
    t = time.time()
    i = ref.ntt(curve, logn, g, f, inverse=True)
    ti = time.time() - t
    assert np.array_equal(i, x), "reference NTT round trip failed"
    t = time.time()
    ix = ref.ntt(curve, logn, g, x, inverse=True)  # the inverse applied to the config input itself
    return {"curve": curve, "log_n": logn, "seed": seed, "input_sha256": sha(x), "forward_sha256": sha(f),
            "forward_first": [int(v) for v in f[0]], "forward_last": [int(v) for v in f[-1]],
            "inverse_sha256": sha(ix), "inverse_first": [int(v) for v in ix[0]],
            "roundtrip_ok": True, "reference_forward_seconds": tf, "reference_inverse_seconds": ti}


# ----------------------------------------------------------------------------- group FFT

GFFT_CASES = [  # (key, curve, m, input kind, seed, infinities)
    ("bn128_m12", "bn128", 12, "subgroup_projective", 0x6F0012, 3),
    ("bn128_m14", "bn128", 14, "subgroup_projective", 0x6F0014, 5),
    ("bls12_381_m12", "bls12_381", 12, "subgroup_projective", 0x6F1012, 3),
    ("bls12_381_m14", "bls12_381", 14, "subgroup_projective", 0x6F1014, 5),
    ("bls12_381_nonsubgroup_m10", "bls12_381", 10, "nonsubgroup_affine", 0x6F200A, 0),
    # round 6: the bench size m = 16, and the Jacobian twins <C>_G1_jac_fft_* (bls12_381_G1_jac.c:727-838)
    ("bn128_m16", "bn128", 16, "subgroup_projective", 0x6F0016, 7),
    ("bls12_381_m16", "bls12_381", 16, "subgroup_projective", 0x6F1016, 7),
    ("jac_bn128_m12", "bn128", 12, "subgroup_jacobian", 0x6F3012, 3),
    ("jac_bn128_m14", "bn128", 14, "subgroup_jacobian", 0x6F3014, 5),
    ("jac_bls12_381_m12", "bls12_381", 12, "subgroup_jacobian", 0x6F4012, 3),
    ("jac_bls12_381_m14", "bls12_381", 14, "subgroup_jacobian", 0x6F4014, 5),
    ("jac_bls12_381_nonsubgroup_m10", "bls12_381", 10, "nonsubgroup_jacobian", 0x6F500A, 2),
]


def _gfft_input(case):
    _, curve, m, kind, seed, n_inf = case
    n = 1 << m
    if kind == "subgroup_projective":
        return golden_io.projective_points(zk, Oracle(), curve, n, seed, n_inf=n_inf)
    if kind == "subgroup_jacobian":
        return golden_io.jacobian_points(zk, Oracle(), curve, n, seed, n_inf=n_inf)
    if kind == "nonsubgroup_jacobian":
        return golden_io.jacobian_points(zk, Oracle(), curve, n, seed, n_inf=n_inf,
                                         affine=golden_io.bls_nonsubgroup_points(n, seed))
    aff = golden_io.bls_nonsubgroup_points(n, seed)
    out = np.zeros((n, 3 * zk.NLIMBS_P[curve]), dtype=np.uint64)
    Reference().arr(curve, "G1_proj_batch_from_affine", n, aff, out)
    return out


def _gfft_job(args):
    case, inverse = args
    key, curve, m = case[:3]
    pts = _gfft_input(case)
    g = zk.get_fft_subgroup(curve, m).gen_array()
    out = np.zeros_like(pts)
    t = time.time()
    co = "jac" if "jacobian" in case[3] else "proj"
    Reference().arr(curve, f"G1_{co}_fft_inverse" if inverse else f"G1_{co}_fft_forward", m, g, pts, out)
    return key, inverse, sha(pts), sha(out), time.time() - t


def make_group_fft(only=None):
    """only: comma-separated substring filter on the case keys; other cases keep their stored digests"""
    os.makedirs(GOLD, exist_ok=True)
    cases = [c for c in GFFT_CASES if not only or any(o in c[0] for o in only.split(","))]
    jobs = sorted([(c, inv) for c in cases for inv in (False, True)], key=lambda j: -(j[0][2] + j[1]))
    with mp.Pool(8) as pool:  # longest first
        res = pool.map(_gfft_job, jobs, chunksize=1)
    path = os.path.join(GOLD, "group_fft.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    for case in cases:
        key, curve, m, kind, seed, n_inf = case
        src = ("<C>_G1_jac_fft_forward / _inverse of lib/cbits (bls12_381_G1_jac.c:727-838)" if "jacobian" in kind
               else "<C>_G1_proj_fft_forward / _inverse of lib/cbits (bls12_381_G1_proj.c:679-790)")
        d = {"curve": curve, "log_n": m, "input": kind, "seed": seed, "n_inf": n_inf, "reference": src}
        for k, inv, sin, sout, dt in res:
            if k != key:
                continue
            d["input_sha256"] = sin
            d["inverse_sha256" if inv else "forward_sha256"] = sout
            d["reference_inverse_seconds" if inv else "reference_forward_seconds"] = dt
        data[key] = d
        print(key, "forward %.1fs inverse %.1fs" % (d["reference_forward_seconds"], d["reference_inverse_seconds"]),
              flush=True)
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)


# ----------------------------------------------------------------------------- G2 MSM at bench sizes

G2_CASES = [  # (key, curve, log n, seed): distinct points P0 + i H, 1/4096 of them infinity, 1/1000 zero scalars
    ("bn128_2^16", "bn128", 16, 0x6A0016),
    ("bn128_2^18", "bn128", 18, 0x6A0018),
    ("bls12_381_2^16", "bls12_381", 16, 0x6A1016),
    ("bls12_381_2^18", "bls12_381", 18, 0x6A1018),
]


def _g2_job(case):
    key, curve, logn, seed = case
    ref = Reference()
    sc, pts = golden_io.g2_case_inputs(ref.lib, curve, logn, seed, zk.gen_fr)
    NP = zk.NLIMBS_P[curve]
    out = np.zeros(4 * NP, dtype=np.uint64)
    t = time.time()
    ref.arr(curve, "G2_proj_MSM_mont_coeff_affine_out", sc.shape[0], sc, pts, out, 4)
    dt = time.time() - t
    std = Oracle().to_std(FLD_FR[curve], sc) if logn == 16 else None
    res = {"curve": curve, "log_n": logn, "seed": seed, "scalars_sha256": sha(sc), "points_sha256": sha(pts),
           "mont_affine": [int(x) for x in out], "reference_seconds": dt,
           "reference": f"{curve}_G2_proj_MSM_mont_coeff_affine_out (bls12_381_G2_proj.c:498 ff.)"}
    if std is not None:  # the std entry on to_std'd scalars with a 2^256 - 1 row (used verbatim)
        std[3] = np.uint64(0xFFFFFFFFFFFFFFFF)
        o2 = np.zeros(4 * NP, dtype=np.uint64)
        ref.arr(curve, "G2_proj_MSM_std_coeff_affine_out", std.shape[0], std, pts, o2, 4)
        res["std_affine_row3_all_ones"] = [int(x) for x in o2]
    return key, res


def make_g2_large():
    with mp.Pool(4) as pool:
        res = dict(pool.map(_g2_job, G2_CASES, chunksize=1))
    json.dump(res, open(os.path.join(GOLD, "g2_msm.json"), "w"), indent=1, sort_keys=True)
    for k, v in res.items():
        print(k, "reference %.1fs" % v["reference_seconds"], flush=True)


def make_large(which):
    os.makedirs(GOLD, exist_ok=True)
    path = os.path.join(GOLD, "baseline_configs.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    jobs = {
        "config1_bn128_ntt_2^14": lambda: large_ntt("bn128", 14, 0x5A4B0001),
        "config2_bls12_381_msm_2^20": lambda: large_msm("bls12_381", 20, 0x5A4B0002, 8),
        "config3_bls12_381_ntt_2^24": lambda: large_ntt("bls12_381", 24, 0x5A4B0003),
        "config4_bn128_msm_2^24": lambda: large_msm("bn128", 24, 0x5A4B0004, 8),
        "config5_bls12_381_msm_2^26": lambda: large_msm("bls12_381", 26, 0x5A4B0005, 8),
        # skewed inputs at a size whose sort takes the sub-bin level (k_split)
        "skew_mix3_bls12_381_msm_2^22": lambda: large_skew_msm("bls12_381", 22, 0x5A4B0006, "mix3"),
        "skew_binary_bn128_msm_2^22": lambda: large_skew_msm("bn128", 22, 0x5A4B0007, "binary"),
    }
    for k, fn in jobs.items():
        if which and which not in k:
            continue
        t = time.time()
        data[k] = fn()
        data[k]["wall_seconds"] = time.time() - t
        print(k, "done in %.1fs" % (time.time() - t), flush=True)
        json.dump(data, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in ("small", "large", "patterns", "groupfft", "g2large"):
        print(__doc__)
        sys.exit(2)
    if sys.argv[1] == "small":
        make_small()
    elif sys.argv[1] == "patterns":
        make_patterns()
    elif sys.argv[1] == "groupfft":
        make_group_fft(sys.argv[2] if len(sys.argv) > 2 else None)
    elif sys.argv[1] == "g2large":
        make_g2_large()
    else:
        make_large(sys.argv[2] if len(sys.argv) > 2 else None)
