#!/bin/bash
# round-5 GPU step: BVH build variants (64 SAH bins, node cost 0.25) on C3; then the round-end rehearsal
set -uo pipefail
mkdir -p gpurun_out/r05m
AB_SPP=16 AB_ROUNDS=3 timeout -k 10 240 python3 tools/ab_pt.py base b64 ct25 > gpurun_out/r05m/ab.log 2>&1 || exit 1
bash tools/gpu_check.sh r05a
