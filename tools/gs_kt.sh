#!/bin/bash
# Kernel-trace the 3DGS forward at GS_N Gaussians (default 100k and 1M) with the given library
# variants: per-kernel averages under gpurun_out/gs_kt_<n>_<variant>/ (summarise: tools/kt_summary.py).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for n in ${GS_NS:-100000 1000000}; do
  for v in "$@"; do
    GS_N=$n GS_STAGES=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/gs_kt_${n}_${v} -o run \
      --output-format csv -- python3 tools/gs_probe.py $v > gpurun_out/gs_kt_${n}_${v}.log 2>&1
  done
done
