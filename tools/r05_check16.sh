#!/bin/bash
# round-5 GPU step: the blend's evaluation two list entries per unrolled step (55 VGPRs: 9 workgroups
# per CU) vs four (64 VGPRs: 8)
set -uo pipefail
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 120 python3 tools/gs_ab_check.py u2 > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py u2 >> $O/check.log 2>&1 || exit 1
GS_AB_ROUNDS=4 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_u2.so" > $O/ab.log 2>&1 || exit 1
AB_ROUNDS=3 timeout -k 10 300 python3 tools/gs_orbit_ab.py base u2 > $O/orbit_ab.log 2>&1 || exit 1
exit 0
