#!/bin/bash
# Kernel traces of tools/gs_bands.py: the full frame and bands 0 / 3 / 7 of 8 (with and without chunk
# bounds) at the given configs (default c2 10m); per-kernel averages under gpurun_out/gsb_<cfg>_<band>_<bounds>/
# (summarise: tools/kt_summary.py).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in ${GS_CFGS:-c2 10m}; do
  for spec in full:1 0:1 3:1 7:1 3:0; do
    band=${spec%%:*}; b=${spec##*:}
    GS_CFG=$cfg GS_BAND=$band GS_BOUNDS=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      -d gpurun_out/gsb_${cfg}_${band}_${b} -o run --output-format csv -- python3 tools/gs_bands.py \
      > gpurun_out/gsb_${cfg}_${band}_${b}.log 2>&1
    grep "ms/frame" gpurun_out/gsb_${cfg}_${band}_${b}.log
  done
done
