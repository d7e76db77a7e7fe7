#!/usr/bin/env python3
"""Per-kernel SQ / GRBM counters (mean per dispatch) from a rocprofv3 --pmc pass:

    python tools/sq_summary.py gpurun_out/TAG_pmcsq --source "..." > profiles/TAG_valu_pmc.json

Counters: SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
(tools/gpu_job.sh step pmcsq).  valu_busy_est = SQ_INSTS_VALU x 3.5 issue cycles per wave
instruction (4 for the half-rate v_mad_u64_u32 class, ~2 for full-rate 32-bit ops) /
(GRBM_GUI_ACTIVE / 8 XCDs) / 1024 SIMDs -- an estimate; the ISA-count issue-slot model
(tools/isa_count.py, bench.py valu_roofline) is the reference.
"""
import argparse
import csv
import glob
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{a.dir}/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = (r.get("Kernel_Name") or "").split("(")[0].replace("void ", "").strip()
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"source": a.source,
           "note": "valu_busy_est = SQ_INSTS_VALU x 3.5 / (GRBM_GUI_ACTIVE / 8 XCDs) / 1024 SIMDs -- an estimate; "
                   "the ISA-count model (bench.py valu_roofline) is the reference"}
    for name, cs in vals.items():
        m = {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())}
        if m.get("GRBM_GUI_ACTIVE"):
            m["valu_busy_est"] = round(m.get("SQ_INSTS_VALU", 0) * 3.5 / (m["GRBM_GUI_ACTIVE"] / 8) / 1024, 3)
        out[name] = m
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
