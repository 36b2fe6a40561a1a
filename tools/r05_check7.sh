#!/bin/bash
# round-5 GPU step: tile-order workgroup stamps at C2; BVH shape A/B on C5's mesh (api.cpp PTGS_BVH_TRIES)
set -uo pipefail
O=gpurun_out/r05i; mkdir -p $O
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_stamps.py > $O/stamps.log 2>&1 || exit 1
PTGS_BVH_LOG=1 AB_SPP=16 AB_ROUNDS=3 timeout -k 10 400 python3 tools/ab_tree.py default 4:4:38 3:4:34 3:4:30 3:4:26 > $O/tree.log 2>&1 || exit 1
exit 0
