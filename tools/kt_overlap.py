#!/usr/bin/env python3
"""Two-queue timeline of a rocprofv3 --kernel-trace run (frames in flight): per dispatch its start / end
relative to the window's first, duration, queue, and for each blend the gap since the previous blend ended
and how much of the front end of the next frame ran inside it.
   tools/kt_overlap.py gpurun_out/<dir> [first] [count]   (default: 30 dispatches from 40% into the trace)"""
import csv
import glob
import os
import sys

d = sys.argv[1]
f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "gs_" in r["Kernel_Name"]]
first = int(sys.argv[2]) if len(sys.argv) > 2 else int(len(rows) * 0.4)
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 30
sub = rows[first:first + cnt]
t0 = int(sub[0]["Start_Timestamp"])
prev_blend_end = None
for r in sub:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ptgs::", "")[:30]
    extra = ""
    if "blend" in name:
        if prev_blend_end is not None:
            extra = f"  gap since previous blend {(s - prev_blend_end) / 1e3:5.1f}"
        prev_blend_end = e
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  dur {(e - s) / 1e3:6.1f}  q{r['Queue_Id']}  {name}{extra}")
