#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (mean per dispatch).
    python tools/pmc_summary.py <dir_with_FETCH_SIZE_run> <dir_with_WRITE_SIZE_run> [calib_dir]
FETCH_SIZE / WRITE_SIZE are in KiB.  The gfx950 FETCH_SIZE scale for a given access
pattern is calibrated with tools/microbench/gather_calib (known byte count) when given."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            short = name.split("(")[0].split("<")[0].replace("void ", "").strip()
            vals[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


fetch = load(sys.argv[1])
write = load(sys.argv[2])
calib = load(sys.argv[3]) if len(sys.argv) > 3 else {}
out = {}
scale = None
if calib:
    kib, _ = calib.get(("k_gather", "FETCH_SIZE"), (None, 0))
    if kib:
        known = (1 << 24) * 128 + (1 << 24) * 4
        scale = known / (kib * 1024)
        out["gather_calibration"] = {"known_bytes": known, "fetch_size_bytes": kib * 1024, "scale": scale}
for (k, c), (v, n) in sorted(fetch.items()):
    if c != "FETCH_SIZE" or not k.startswith("zk::"):
        continue
    w = write.get((k, "WRITE_SIZE"), (0.0, 0))[0]
    out[k] = {"fetch_bytes_raw": v * 1024, "write_bytes": w * 1024, "dispatches": n}
print(json.dumps(out, indent=1))
