#!/usr/bin/env python3
"""Print VGPR / occupancy / spill for our kernels: python tools/kres.py csrc/zk_msm.hip"""
import re, subprocess, sys
src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o", "/dev/null",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+): (\S+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if "zk" not in k:
        continue
    d = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    print(f"{d[:70]:70s} vgpr={v.get('VGPRs')} occ={v.get('Occupancy [waves/SIMD]')} spill={v.get('VGPRs Spill')} scratch={v.get('ScratchSize [bytes/lane]')} lds={v.get('LDS Size [bytes/block]')}")
