#!/usr/bin/env python3
"""VGPR / AGPR / spill counts and the resulting waves per SIMD of every kernel in a gfx950
assembly file (the amdhsa.kernels metadata), e.g.
    python tools/kernel_regs.py zk_msm-hip-amdgcn-amd-amdhsa-gfx950.s k_ysum2 k_accum"""
import re
import sys


def kernels(path):
    txt = open(path).read()
    meta = txt[txt.index("amdhsa.kernels:"):]
    out = {}
    for block in re.split(r"\n  - ", meta)[1:]:
        name = re.search(r"\.name:\s+(\S+)", block)
        if not name:
            continue
        get = lambda k: int(re.search(r"\.%s:\s+(\d+)" % k, block).group(1)) if re.search(r"\.%s:\s+(\d+)" % k, block) else 0
        v, a = get("vgpr_count"), get("agpr_count")
        out[name.group(1)] = {"vgpr": v, "agpr": a, "vgpr_spill": get("vgpr_spill_count"),
                              "sgpr_spill": get("sgpr_spill_count"), "lds": get("group_segment_fixed_size"),
                              "waves_per_simd": 512 // max(1, ((v + a + 7) // 8) * 8)}
    return out


if __name__ == "__main__":
    ks = kernels(sys.argv[1])
    for name, d in ks.items():
        if len(sys.argv) > 2 and not any(p in name for p in sys.argv[2:]):
            continue
        print(f"{name[:70]:70s} vgpr {d['vgpr']:3d} agpr {d['agpr']:3d} spill {d['vgpr_spill']:3d} "
              f"lds {d['lds']:6d} waves/SIMD {d['waves_per_simd']}")
