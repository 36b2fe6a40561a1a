#!/bin/bash
# Per-kernel register / scratch / occupancy of one HIP source (gfx950), from the compiler's
# kernel-resource-usage remarks:  tools/kres.sh pathtracer_gaussiansplatting_amd/csrc/pt_kernels.hip [-Dflags]
SRC=$1; shift
D=$(cd "$(dirname "$SRC")" && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -I "$D/../../include" -I "$D" --offload-arch=gfx950 "$@" \
  -c "$SRC" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    print(f"{r[\"name\"][:70]:70s} VGPR {r.get(\"VGPRs\",\"?\"):>4} AGPR {r.get(\"AGPRs\",\"?\"):>3} SGPR {r.get(\"TotalSGPRs\",\"?\"):>4} "
          f"scratch {r.get(\"ScratchSize [bytes/lane]\",\"?\"):>4} VGPRspill {r.get(\"VGPRs Spill\",\"?\"):>3} SGPRspill {r.get(\"SGPRs Spill\",\"?\"):>3} "
          f"occ {r.get(\"Occupancy [waves/SIMD]\",\"?\"):>2} LDS {r.get(\"LDS Size [bytes/block]\",\"?\")}")
'
