#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy of one HIP source (gfx950), from the compiler's
kernel-resource-usage remarks:  python3 tools/kres.py <file.hip> [-Dflags ...]"""
import os
import re
import subprocess
import sys

src = sys.argv[1]
d = os.path.dirname(os.path.abspath(src))
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(d, "..", "..", "include"),
       "-I", d, "--offload-arch=gfx950", *sys.argv[2:], "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
if not rows:
    print(out[-3000:])
keys = [("VGPRs", "VGPR"), ("AGPRs", "AGPR"), ("TotalSGPRs", "SGPR"), ("ScratchSize [bytes/lane]", "scratch"),
        ("VGPRs Spill", "Vspill"), ("SGPRs Spill", "Sspill"), ("Occupancy [waves/SIMD]", "occ"),
        ("LDS Size [bytes/block]", "LDS")]
for r in rows:
    print(f"{r['name'][:72]:72s} " + " ".join(f"{short} {r.get(k, '?'):>5}" for k, short in keys))
