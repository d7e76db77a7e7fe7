#!/usr/bin/env python3
"""Instruction counts of a kernel's hot loop, from the compiler's gfx950 assembly.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --save-temps -c zk_msm.hip   (in a scratch dir)
    python tools/isa_count.py zk_msm-hip-amdgcn-amd-amdhsa-gfx950.s 'k_accumINS_6BLS381' [--json out]

Splits the function into basic blocks, uses LLVM's loop annotations ("in Loop: Header=...
Depth=d") to collect the blocks of every loop, and prints per-block and per-loop opcode
counts.  The VALU roofline in bench.py is priced from these counts: the number of
v_mad_u64_u32 (and of the other VALU instructions) one loop iteration issues, times the
measured per-instruction issue ceiling (tools/microbench/valu_ceiling.hip).
"""
import argparse
import collections
import json
import re
import sys


def function_body(lines, sym):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*%s\S*:" % re.escape(sym), l):
            start = i
            name = l.split(":")[0]
        elif start is not None and l.startswith(".Lfunc_end"):
            return name, lines[start:i]
    raise SystemExit(f"symbol matching {sym!r} not found")


def blocks_of(body):
    blocks = []
    cur = {"label": "entry", "loop": None, "depth": 0, "ops": collections.Counter(), "n": 0, "succ": [],
           "falls": True}
    for l in body[1:]:
        m = re.match(r"^(\.LBB\w+):(.*)$", l)
        if m:
            blocks.append(cur)
            comment = m.group(2)
            hm = re.search(r"Header=(BB\w+) Depth=(\d+)", comment)
            if "Loop Header" in comment:
                dm = re.search(r"Depth=(\d+)", comment)
                loop, depth = m.group(1)[2:], int(dm.group(1)) if dm else 1
            elif hm:
                loop, depth = hm.group(1), int(hm.group(2))
            else:
                loop, depth = None, 0
            cur = {"label": m.group(1), "loop": loop, "depth": depth, "ops": collections.Counter(), "n": 0,
                   "succ": [], "falls": True}
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        cur["ops"][op] += 1
        cur["n"] += 1
        if op.startswith("s_branch") or op.startswith("s_cbranch") or op.startswith("s_setpc"):
            t = re.search(r"(\.LBB\w+)", s)
            if t:
                cur["succ"].append(t.group(1))
            if op.startswith("s_branch") or op.startswith("s_setpc"):
                cur["falls"] = False
        if op.startswith("s_endpgm"):
            cur["falls"] = False
    blocks.append(cur)
    return blocks


def cfg_loops(blocks):
    """natural loops from the control-flow graph (branch targets + fall-through): an edge i -> h
    whose target dominates its source is a back edge; the loop is the header plus every block
    that reaches the back edge's source without passing through the header.  (LLVM's "in Loop"
    comments miss blocks whose label carries another comment.)"""
    idx = {b["label"]: i for i, b in enumerate(blocks)}
    succ = []
    for i, b in enumerate(blocks):
        s = [idx[t] for t in b["succ"] if t in idx]
        if b["falls"] and i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    pred = [[] for _ in blocks]
    for i, ss in enumerate(succ):
        for j in ss:
            pred[j].append(i)
    # dominators (iterative data flow from the entry block)
    n = len(blocks)
    full = set(range(n))
    dom = [full.copy() for _ in range(n)]
    dom[0] = {0}
    changed = True
    while changed:
        changed = False
        for i in range(1, n):
            ps = [dom[p] for p in pred[i]]
            new = (set.intersection(*ps) if ps else set()) | {i}
            if new != dom[i]:
                dom[i] = new
                changed = True
    loops = collections.OrderedDict()
    for i, ss in enumerate(succ):
        for h in ss:
            if h in dom[i]:  # back edge i -> h (h dominates i)
                body = loops.setdefault(blocks[h]["label"], {h})
                stack = [i]
                while stack:
                    x = stack.pop()
                    if x in body:
                        continue
                    body.add(x)
                    stack.extend(pred[x])
    # keep innermost-first order by header position
    return collections.OrderedDict((k, sorted(v)) for k, v in sorted(loops.items(), key=lambda kv: idx[kv[0]]))


def classify(op):
    if op.startswith("v_mad_u64_u32"):
        return "v_mad_u64_u32"
    if op.startswith(("v_mul_lo", "v_mul_hi", "v_mul_u32", "v_mad_u32")):
        return "v_mul32"
    if op.startswith(("v_lshrrev_b64", "v_lshlrev_b64", "v_lshl_add_u64")) or op.endswith("_b64"):
        return "valu_64"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_"):
        return "salu/smem/branch"
    if op.startswith("v_"):
        return "valu_other"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    ap.add_argument("--json")
    ap.add_argument("--note", default="", help="what one iteration of the hot loop is")
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines()
    name, body = function_body(lines, a.symbol)
    blocks = blocks_of(body)
    total = collections.Counter()
    for b in blocks:
        total.update(b["ops"])
    print(f"{name}: {sum(total.values())} instructions, {total['v_mad_u64_u32']} v_mad_u64_u32 (static)")
    # loops as LLVM annotates them ("in Loop: Header=..." on the block labels): for k_accum these
    # are exactly the blocks of one mixed add (its rare branches -- doubling, flush, infinity --
    # carry other comments), which is what the VALU roofline prices
    loops = collections.OrderedDict()
    for b in blocks:
        if b["loop"]:
            loops.setdefault(b["loop"], []).append(b)
    # natural loops of the control-flow graph: every block of each loop (tools/ntt_isa_model.py)
    out_cfg = collections.OrderedDict()
    for hdr, members in cfg_loops(blocks).items():
        cls = collections.Counter()
        for i in members:
            for op, c in blocks[i]["ops"].items():
                cls[classify(op)] += c
        out_cfg[hdr[2:] if hdr.startswith(".L") else hdr] = {
            "blocks": [blocks[i]["label"] for i in members], "classes": dict(cls),
            "issue_slots": cls.get("v_mad_u64_u32", 0) + cls.get("v_mul32", 0) + cls.get("valu_64", 0) +
            0.5 * cls.get("valu_other", 0)}
    out = {"function": name, "note": a.note, "static_total": dict(total), "blocks": [], "loops": {},
           "cfg_loops": out_cfg}
    print(f"{'block':<14}{'loop':<12}{'d':>2}{'instr':>7}{'mad64':>7}{'valu':>7}{'vmem':>6}{'lds':>6}")
    for b in blocks:
        cls = collections.Counter()
        for op, c in b["ops"].items():
            cls[classify(op)] += c
        valu = sum(v for k, v in cls.items() if k.startswith("v"))
        print(f"{b['label']:<14}{str(b['loop']):<12}{b['depth']:>2}{b['n']:>7}{cls['v_mad_u64_u32']:>7}"
              f"{cls['v_mad_u64_u32'] + cls['v_mul32'] + cls['valu_64'] + cls['valu_other']:>7}{cls['vmem']:>6}{cls['lds']:>6}")
        out["blocks"].append({"label": b["label"], "loop": b["loop"], "depth": b["depth"], "instr": b["n"],
                              "classes": dict(cls)})
    for hdr, d in out_cfg.items():
        print(f"cfg loop {hdr}: {len(d['blocks'])} blocks, {d['issue_slots']:.1f} issue slots, "
              + ", ".join(f"{k}={v}" for k, v in sorted(d["classes"].items())))
    for lp, bl in loops.items():
        cls = collections.Counter()
        for b in bl:
            for op, c in b["ops"].items():
                cls[classify(op)] += c
        out["loops"][lp] = {"blocks": [b["label"] for b in bl], "classes": dict(cls)}
        print(f"loop {lp}: {len(bl)} blocks, " + ", ".join(f"{k}={v}" for k, v in sorted(cls.items())))
    if out["loops"]:
        hot = max(out["loops"], key=lambda k: out["loops"][k]["classes"].get("v_mad_u64_u32", 0))
        cls = out["loops"][hot]["classes"]
        # issue-slot model (tools/microbench/valu_ceiling.hip, profiles/*valu_ceiling*.json):
        # v_mad_u64_u32, v_mul_lo/hi_u32 and 64-bit shifts issue at half rate (1 slot),
        # plain 32-bit VALU at full rate (1/2 slot); the chip's slot ceiling is the measured
        # v_mad_u64_u32 rate
        slots = cls.get("v_mad_u64_u32", 0) + cls.get("v_mul32", 0) + cls.get("valu_64", 0) + \
            0.5 * cls.get("valu_other", 0)
        out["hot_loop"] = {"label": hot, "per_iteration": cls, "issue_slots_per_iteration": slots}
        print(f"hot loop {hot}: {slots:.1f} half-rate issue slots per iteration")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
