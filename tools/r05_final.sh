#!/bin/bash
# round-5 final: rocprofv3 passes of the final library (profiles/profile.sh), their summary (written into
# this box's profiles/ so the bench below reads the matching traffic_latest.json), then the driver's
# round-end tiers (tools/gpu_check.sh); the profile outputs are copied to gpurun_out/final/
set -uo pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 bash profiles/profile.sh r05 > gpurun_out/final/profile.log 2>&1 || exit 1
python3 profiles/parse_rocprof.py r05 > gpurun_out/final/parse.log 2>&1 || exit 1
cp profiles/r05_summary.md profiles/r05_kernel_stats.csv profiles/traffic_latest.json gpurun_out/final/ || exit 1
bash tools/gpu_check.sh r05b
