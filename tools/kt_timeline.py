#!/usr/bin/env python3
"""Timeline of consecutive dispatches from a rocprofv3 --kernel-trace run: start offset / duration / gap
(us) of the last N dispatches:  tools/kt_timeline.py gpurun_out/<dir> [N]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ptgs::", "")[:34]
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:7.1f}  gap {gap:6.1f}  grid {r.get('Grid_Size', '?'):>9} {name}")
    prev_end = e
