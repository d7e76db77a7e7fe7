#!/usr/bin/env python3
"""Issue slots of ONE lane's GLV scalar-multiplication chain in the group FFT's stage kernels
(zk_g1ext.hip jac_scl130_pair inside k_fft_radix_prod / k_fft_fwd_stage_glv), from the compiler's
gfx950 assembly -- the group-FFT counterpart of the k_accum hot-loop counts:

    bash: hipcc --offload-arch=gfx950 -O3 -std=c++17 --save-temps -c zk_g1ext.hip   (scratch dir)
    python tools/fft_isa.py zk_g1ext-hip-amdgcn-amd-amdhsa-gfx950.s TAG   -> profiles/TAG_isa_glv_chain_<curve>.json

Loop structure of the chain (tools/isa_count.py cfg_loops): a one-block loop = one lazy Jacobian
doubling (rolled, 5 per window), the loop around it = one signed 5-bit window (table lookup, the
phi product, one cached addition), the other large loop = one table step (cached addition + caching,
8 steps, 7 additions).  Blocks with the doubling's mad count inside the addition loops are the
addition's rare P == Q branch and are left out.  Chain = table + 27 windows + 130 doublings + the
straight-line code (conversion in and out, the pair merge; rare branches included: an upper bound).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_count  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def slots(c):
    return c.get("v_mad_u64_u32", 0) + c.get("v_mul32", 0) + c.get("valu_64", 0) + 0.5 * c.get("valu_other", 0)


def chain(asm, sym):
    lines = open(asm).read().splitlines()
    name, body = isa_count.function_body(lines, sym)
    blocks = isa_count.blocks_of(body)
    by = {b["label"]: b for b in blocks}
    cls = {b["label"]: __import__("collections").Counter() for b in blocks}
    for b in blocks:
        for op, c in b["ops"].items():
            cls[b["label"]][isa_count.classify(op)] += c
    loops = isa_count.cfg_loops(blocks)
    lab = lambda i: blocks[i]["label"]  # noqa: E731
    L = {h: [lab(i) for i in m] for h, m in loops.items()}
    dbl = [h for h, m in L.items() if len(m) == 1 and cls[m[0]].get("v_mad_u64_u32", 0) > 500]
    assert len(dbl) == 1, f"{sym}: expected one rolled doubling loop, got {dbl}"
    dbl_lab = L[dbl[0]][0]
    dbl_mads = cls[dbl_lab]["v_mad_u64_u32"]
    win = [h for h, m in L.items() if dbl_lab in m and len(m) > 1]
    assert len(win) == 1
    tab = [h for h, m in L.items() if h not in dbl + win and sum(cls[x].get("v_mad_u64_u32", 0) for x in m) > 1000]
    assert len(tab) == 1, tab

    def common(members, exclude):
        return sum(slots(cls[x]) for x in members if x not in exclude and cls[x].get("v_mad_u64_u32", 0) != dbl_mads)
    s_dbl = slots(cls[dbl_lab])
    s_win = common(L[win[0]], {dbl_lab})
    s_tab = common(L[tab[0]], set())
    in_loops = set(x for m in L.values() for x in m)
    s_straight = sum(slots(cls[b["label"]]) for b in blocks if b["label"] not in in_loops)
    total = 8 * s_tab + 27 * s_win + 130 * s_dbl + s_straight  # table add skipped once: see note
    return {"function": name, "doubling_slots": s_dbl, "window_slots_excl_doublings": s_win,
            "table_step_slots": s_tab, "straight_line_slots": s_straight, "issue_slots_per_chain": total,
            "doubling_mads": dbl_mads}


def main():
    asm, tag = sys.argv[1], sys.argv[2]
    for curve, sym in (("bls12_381", "k_fft_radix_prodINS_6BLS381"), ("bn128", "k_fft_radix_prodINS_5BN254")):
        d = chain(asm, sym)
        d["note"] = ("one lane's GLV chain (|k| < 2^130: 8 table steps, 27 signed 5-bit windows, 130 Jacobian "
                     "doublings) in k_fft_radix_prod (the fused radix-2 stages run the same inlined chain); "
                     "the table's first step has no addition, counted anyway (upper bound, < 1 %)")
        out = os.path.join(ROOT, "profiles", f"{tag}_isa_glv_chain_{curve}.json")
        json.dump(d, open(out, "w"), indent=1)
        print(curve, json.dumps({k: v for k, v in d.items() if k != "note"}))


if __name__ == "__main__":
    main()
