#!/bin/bash
# round-5 GPU step: DPP / permlane exchanges + lockstep run searches vs the committed library
set -uo pipefail
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 120 python3 tools/gs_ab_check.py c38 > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py c38 >> $O/check.log 2>&1 || exit 1
GS_AB_ROUNDS=3 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_dpp.so" "GS_LIB=libptgs_c38.so" > $O/ab.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -k "gaussian or splat or tight or raster or hybrid or c4 or c5" > $O/pytest.log 2>&1 || exit 1
exit 0
