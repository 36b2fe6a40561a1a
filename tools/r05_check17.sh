#!/bin/bash
# round-5 GPU step: the small-tile counting / merge-ranking crossover (GS_MERGE_MIN 64 / 96 / 128)
set -uo pipefail
O=gpurun_out/r05ab; mkdir -p $O
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py mm64 > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py mm128 >> $O/check.log 2>&1 || exit 1
GS_AB_ROUNDS=3 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_mm64.so" "GS_LIB=libptgs_mm128.so" > $O/ab.log 2>&1 || exit 1
exit 0
