#!/bin/bash
# round-5 GPU step: 4x4 sub-block lists (bit-exact vs the quadrant-list library, C2 / 1M A/B), tests
set -uo pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 120 python3 tools/gs_ab_check.py quad > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py quad >> $O/check.log 2>&1 || exit 1
GS_N=1000000 timeout -k 10 120 python3 tools/gs_ab_check.py quad >> $O/check.log 2>&1 || exit 1
GS_AB_ROUNDS=3 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_quad.so" "GS_LIB=libptgs_base.so" > $O/ab.log 2>&1 || exit 1
GS_N=1000000 GS_FRAMES=60 GS_AB_ROUNDS=2 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_base.so" > $O/ab_1m.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
exit 0
