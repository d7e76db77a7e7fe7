"""Print the kernel / copy timeline of the LAST call in a rocprofv3 --kernel-trace
--memory-copy-trace directory (one line per dispatch or copy, microseconds from the call's first
host-to-device copy): python tools/trace_timeline.py gpurun_out/<tag>_trace"""
import csv
import os
import sys

d = sys.argv[1]
ks = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
mp = os.path.join(d, "run_memory_copy_trace.csv")
ms = list(csv.DictReader(open(mp))) if os.path.exists(mp) else []
ev = []
for k in ks:
    name = k["Kernel_Name"].split("(")[0].replace("void ", "").replace("zk::", "")[:40]
    ev.append((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K", name, k.get("Stream_Id", "")))
for m in ms:
    ev.append((int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "C", m["Direction"].replace("MEMORY_COPY_", ""),
               m.get("Stream_Id", "")))
ev.sort()
starts, prev = [], None
idle = len(sys.argv) > 2 and sys.argv[2] == "idle"  # calls separated by >= 1 ms with nothing running
for i, e in enumerate(ev):
    if idle:
        if prev is None or e[0] - prev > 1_000_000:
            starts.append(i)
        prev = e[1] if prev is None else max(prev, e[1])
    elif e[2] == "C" and e[3].startswith("HOST_TO_DEVICE"):
        if prev is None or e[0] - prev > 1_000_000:
            starts.append(i)
        prev = e[1]
s = starts[-1] if starts else 0
t0 = ev[s][0]
for e in ev[s:]:
    print(f"{(e[0] - t0) / 1e3:8.1f} {(e[1] - t0) / 1e3:8.1f} {(e[1] - e[0]) / 1e3:7.1f} {e[2]} s{e[4]} {e[3]}")
