#!/bin/bash
# round-5 GPU step: tile order from per-tile bucket bytes (one load round trip), row prefetch behind the
# count walk; posrows modes 0 / 1 / 2 static + moving; stamps; splat tests
set -uo pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 120 python3 tools/gs_ab_check.py pr0 > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py pr2 >> $O/check.log 2>&1 || exit 1
GS_AB_ROUNDS=3 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_pr0.so" "GS_LIB=libptgs_pr2.so" > $O/ab.log 2>&1 || exit 1
AB_ROUNDS=4 timeout -k 10 300 python3 tools/gs_orbit_ab.py base pr0 pr2 > $O/orbit_ab.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_stamps.py > $O/stamps.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -k "gaussian or splat or tight or raster or hybrid or c4 or c5 or dist" > $O/pytest.log 2>&1 || exit 1
exit 0
