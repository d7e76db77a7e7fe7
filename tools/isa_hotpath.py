#!/usr/bin/env python3
"""Issue slots of one iteration of a loop whose hot path is a SUBSET of its blocks -- for loops
where LLVM's loop annotation does not cover the body (the G2 k_accum: the Fp2 mixed add's blocks
sit outside the annotated loop, and the loop also holds the rare doubling path and the bucket-run
flush).  Blocks are named by their hot-path role after inspecting tools/isa_count.py's output:

    python tools/isa_hotpath.py ASM SYMBOL --hot .LBB134_16,... --json out.json --note "..."

Slots: v_mad_u64_u32 / 32-bit multiplies / 64-bit VALU (v_mad_i64_i32 included) 1, other VALU 1/2
(tools/isa_count.py's classes and its measured issue ceiling)."""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_count  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    ap.add_argument("--hot", required=True, help="comma-separated block labels of the common path")
    ap.add_argument("--cold", default="", help="blocks of the loop left out (documentation)")
    ap.add_argument("--json")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines()
    name, body = isa_count.function_body(lines, a.symbol)
    blocks = {b["label"]: b for b in isa_count.blocks_of(body)}
    hot = a.hot.split(",")
    cls = collections.Counter()
    for lab in hot:
        for op, c in blocks[lab]["ops"].items():
            cls[isa_count.classify(op)] += c
    slots = cls.get("v_mad_u64_u32", 0) + cls.get("v_mul32", 0) + cls.get("valu_64", 0) + 0.5 * cls.get("valu_other", 0)
    out = {"function": name, "note": a.note, "hot_blocks": hot, "cold_blocks": [c for c in a.cold.split(",") if c],
           "hot_loop": {"per_iteration": dict(cls), "issue_slots_per_iteration": slots}}
    print(f"{name}: {slots:.1f} issue slots per iteration over {len(hot)} blocks; {dict(cls)}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
