#!/bin/bash
# round-5 GPU step: moving-camera A/B of position-indexed rows (posrows orders are one frame staler)
set -uo pipefail
O=gpurun_out/r05n; mkdir -p $O
AB_ROUNDS=4 timeout -k 10 300 python3 tools/gs_orbit_ab.py base pr0 > $O/orbit_ab.log 2>&1 || exit 1
GS_AB_ROUNDS=3 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_pr0.so" > $O/ab.log 2>&1 || exit 1
exit 0
