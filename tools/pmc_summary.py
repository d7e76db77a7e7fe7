#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 --pmc counter_collection CSVs (mean per dispatch).

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR CALIB_DIR [--tag r02] > profiles/<tag>_pmc.json

FETCH_DIR / WRITE_DIR: separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes over
the same bench command.  CALIB_DIR: `rocprofv3 --pmc FETCH_SIZE -- tools/microbench/gather_calib`
(known byte count READS * 128 + READS * 4 per launch).  Counter values are KiB.

Corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reports 1/2 of the bytes of wide
coalesced 16-B/lane streaming reads, so streaming kernels get x2; other access widths are
uncalibrated in the guide, so the random 128-B row gathers of k_accum are calibrated here
on a known byte count, for plain global_load (k_gather) and global_load_lds (k_gather_lds),
and k_accum's fetch is scaled by the glds factor (its row gathers dominate its reads).
WRITE_SIZE is exact for 16-B/lane stores.  Infinity-Cache hits are counted, not excluded.
"""
import argparse
import csv
import glob
import json
from collections import defaultdict

STREAMING_X2 = ("k_ntt_pass", "k_points_int", "k_digits", "k_coarse", "k_fine", "k_export", "k_arr", "k_ysum")
GATHER_GLDS = ("k_accum",)
READS = 1 << 24


def load(d):
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            short = name.split("(")[0].replace("void ", "").strip()
            short = short.split("<")[0].split("::")[-1] + ("<" + short.split("<", 1)[1] if "<" in short else "")
            vals[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("calib")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    fetch, write, calib = load(a.fetch), load(a.write), load(a.calib)
    known = READS * 128 + READS * 4
    out = {"source": a.source, "note": __doc__.split("\n\n")[2].replace("\n", " "), "calibration": {}}
    scales = {}
    for k in ("k_gather", "k_gather_lds"):
        kib, _ = calib.get((k, "FETCH_SIZE"), (None, 0))
        if kib:
            scales[k] = known / (kib * 1024)
            out["calibration"][k] = {"known_bytes": known, "fetch_size_bytes": kib * 1024, "scale": scales[k]}
    for (k, c), (v, n) in sorted(fetch.items()):
        if c != "FETCH_SIZE" or not (k.startswith("k_") or k.startswith("zk")):
            continue
        base = k.split("<")[0]
        w = write.get((k, "WRITE_SIZE"), (0.0, 0))[0] * 1024
        raw = v * 1024
        if base in GATHER_GLDS and "k_gather_lds" in scales:
            corr, how = raw * scales["k_gather_lds"], f"x{scales['k_gather_lds']:.3f} (glds row-gather calibration)"
        elif base.startswith(STREAMING_X2):
            corr, how = raw * 2, "x2 (16-B/lane streaming reads, guide)"
        else:
            corr, how = raw, "uncorrected"
        out[k] = {"fetch_bytes_raw": raw, "fetch_bytes_corrected": corr, "fetch_correction": how,
                  "write_bytes": w, "hbm_bytes_per_launch": corr + w, "dispatches": n}
        # bench.py looks kernels up by their base name
        if base not in out or out[base].get("hbm_bytes_per_launch", 0) < corr + w:
            out[base] = out[k]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
