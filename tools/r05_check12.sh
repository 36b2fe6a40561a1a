#!/bin/bash
# round-5 GPU step: position-indexed rows, moving camera: orders one frame staler (pr1, default) vs the
# in-launch order (pr2) vs rows by tile (pr0); static C2 likewise; pr2 bit-exactness
set -uo pipefail
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 120 python3 tools/gs_ab_check.py pr2 > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py pr2 >> $O/check.log 2>&1 || exit 1
AB_ROUNDS=4 timeout -k 10 300 python3 tools/gs_orbit_ab.py base pr0 pr2 > $O/orbit_ab.log 2>&1 || exit 1
GS_AB_ROUNDS=3 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_pr0.so" "GS_LIB=libptgs_pr2.so" > $O/ab.log 2>&1 || exit 1
exit 0
