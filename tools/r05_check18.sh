#!/bin/bash
# round-5 GPU step: the blend evaluation's all-done test interval (GS_DONE_EVERY 4 / 8 / 16)
set -uo pipefail
O=gpurun_out/r05ac; mkdir -p $O
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py de8 > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py de16 >> $O/check.log 2>&1 || exit 1
GS_AB_ROUNDS=3 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_de8.so" "GS_LIB=libptgs_de16.so" > $O/ab.log 2>&1 || exit 1
exit 0
