#!/usr/bin/env python3
"""Issue-slot model of the NTT pass kernel (zk_ntt.hip k_ntt_pass), from the compiler's gfx950
assembly -- the NTT counterpart of the k_accum hot-loop counts (tools/isa_count.py).

    python tools/ntt_isa_model.py TAG     -> profiles/TAG_isa_k_ntt_pass.json   (CPU only)

k_ntt_pass is a sequence of loops whose trip counts follow from the launch shape alone:
  load    G R / NT iterations   (one element: HBM -> LDS, bit-reversed)
  first   G R / 4 / NT          (the first radix-4 round: one product)
  round   G R / 4 / NT per radix-4 round, floor((r - 2) / 2) rounds (four products)
  radix2  G R / 2 / NT          (odd r only: one product)
  store   G R / NT              (closing mode: table twiddle | on-the-fly twiddle | 1/N scale |
                                 product-free reduction)
plus straight-line code once per thread.  The static issue slots of every loop body (CFG loops,
classes and weights of tools/isa_count.py: v_mad_u64_u32, 32-bit multiplies and 64-bit ops one
half-rate slot, other 32-bit VALU half a slot) times those trip counts, summed over the threads
of every pass of a transform (zk_ntt.hip split_digits), give the issue slots per transform;
bench.py divides them by the measured pass-chain time and the measured issue ceiling
(profiles/*valu_ceiling*.json).
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import isa_count  # noqa: E402

LOOP_ORDER = ["load", "first", "round", "radix2", "store_table", "store_otf", "store_scale", "store_reduce"]


def split_digits(m, mode=0):
    """zk_ntt.hip split_digits (default mode)"""
    if m == 0:
        return [0]
    if m <= 11:
        return [m]
    if (mode == 12 and 17 <= m <= 24) or (mode == 0 and m == 20):
        return [(m + 1) // 2, m // 2]
    P = (m + 7) // 8
    base, extra = m // P, m % P
    return [base + (1 if p < extra else 0) for p in range(P)]


def kernel_model(asm, sym):
    lines = open(asm).read().splitlines()
    name, body = isa_count.function_body(lines, sym)
    blocks = isa_count.blocks_of(body)
    loops = isa_count.cfg_loops(blocks)
    slots = {}
    in_loop = set()
    named = []
    for hdr, members in loops.items():
        cls = {}
        for i in members:
            for op, c in blocks[i]["ops"].items():
                k = isa_count.classify(op)
                cls[k] = cls.get(k, 0) + c
        s = cls.get("v_mad_u64_u32", 0) + cls.get("v_mul32", 0) + cls.get("valu_64", 0) + 0.5 * cls.get("valu_other", 0)
        if s < 10:  # address-computation loops outside the data path
            continue
        named.append((hdr, members, s, cls))
        in_loop.update(members)
    if len(named) != len(LOOP_ORDER):
        raise SystemExit(f"{sym}: expected {len(LOOP_ORDER)} data loops, found {len(named)}")
    for key, (hdr, members, s, cls) in zip(LOOP_ORDER, named):
        slots[key] = {"header": hdr, "issue_slots": s, "classes": cls}
    straight = 0.0
    for i, b in enumerate(blocks):
        if i in in_loop:
            continue
        for op, c in b["ops"].items():
            k = isa_count.classify(op)
            straight += {"v_mad_u64_u32": 1, "v_mul32": 1, "valu_64": 1, "valu_other": 0.5}.get(k, 0) * c
    return name, slots, straight


def transform_slots(models, m, inverse, mode=0):
    """issue slots of one 2^m transform: every pass's threads x (straight-line + loops x trips)"""
    dig = split_digits(m, mode)
    N = 1 << m
    P = len(dig)
    total = 0.0
    passes = []
    table_max = 1 << 25
    S = N
    for p, r in enumerate(dig):
        R = 1 << r
        S >>= r
        last = p == P - 1
        big = r > 8
        NT, tile = (1024, 4096) if big else (256, 1024)
        if P == 1:
            G = 1
        elif not last:
            G = min(tile // R, S)
        else:
            G = min(tile // R, 1 << dig[0])
        threads = (N // (R * G)) * NT
        mdl, straight = models[NT]
        per = lambda key: mdl[key]["issue_slots"]
        it = lambda k: -(-k // NT)  # per-thread trip count (ceil: idle lanes still issue)
        t = straight + it(G * R) * per("load")
        if r >= 2:
            t += it(G * R // 4) * per("first")
            t += ((r - 2) // 2) * it(G * R // 4) * per("round")
        if r % 2 == 1:
            t += it(G * R // 2) * per("radix2")
        if not last:
            otf = R * S > table_max
            mode_key = "store_otf" if otf else "store_table"
        else:
            scale = inverse and (P == 1 or N > table_max)  # 1/N rides on pass 0's table when it has one
            mode_key = "store_scale" if scale else "store_reduce"
        t += it(G * R) * per(mode_key)
        passes.append({"radix_log2": r, "G": G, "threads": threads, "slots_per_thread": t, "closing": mode_key})
        total += threads * t
    return total, passes


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "scratch"
    with tempfile.TemporaryDirectory() as d:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                               "--save-temps", "-c", os.path.join(ROOT, "zikkurat-algebra_amd", "csrc", "zk_ntt.hip"),
                               "-o", "zk_ntt.o"], cwd=d)
        asm = os.path.join(d, "zk_ntt-hip-amdgcn-amd-amdhsa-gfx950.s")
        out = {"note": __doc__.strip().splitlines()[0], "curves": {}}
        for curve, F in (("bls12_381", "6BLS_Fr"), ("bn128", "5BN_Fr")):
            models = {}
            kern = {}
            for NT in (256, 1024):
                name, slots, straight = kernel_model(asm, f"k_ntt_passINS_{F}ELi{NT}E")
                models[NT] = (slots, straight)
                kern[str(NT)] = {"function": name, "loops": slots, "straight_line_slots": straight}
            sizes = {}
            for m in (14, 20, 22, 24, 26):
                for inv in (False, True):
                    tot, passes = transform_slots(models, m, inv)
                    sizes[f"m{m}_{'inverse' if inv else 'forward'}"] = {"issue_slots": tot, "passes": passes,
                                                                       "slots_per_element": tot / (1 << m)}
            out["curves"][curve] = {"kernels": kern, "transforms": sizes}
            t24 = sizes["m24_forward"]
            print(f"{curve}: 2^24 forward {t24['issue_slots']:.3e} issue slots ({t24['slots_per_element']:.0f} per element)")
    dst = os.path.join(ROOT, "profiles", f"{tag}_isa_k_ntt_pass.json")
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", os.path.relpath(dst, ROOT))


if __name__ == "__main__":
    main()
