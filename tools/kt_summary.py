#!/usr/bin/env python3
"""Per-kernel average durations (us) of rocprofv3 --stats runs: tools/kt_summary.py gpurun_out/gs_kt_*"""
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        parts = []
        tot = 0.0
        for r in rows:
            name = r["Name"].split("(")[0].replace("void ", "").replace("ptgs::", "")
            if name.startswith("at::") or name.startswith("__amd"):
                continue
            us = float(r["AverageNs"]) / 1e3
            tot += us
            parts.append(f"{name} {us:.1f}")
        print(f"{os.path.basename(d):28s} sum {tot:7.1f} us | " + " | ".join(parts))
