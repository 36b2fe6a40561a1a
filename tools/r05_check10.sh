#!/bin/bash
# round-5 GPU step: position-indexed key rows (GS_POSROWS) vs rows by tile; parity; asm-min PT parity
set -uo pipefail
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 120 python3 tools/gs_ab_check.py pr0 > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py pr0 >> $O/check.log 2>&1 || exit 1
GS_AB_ROUNDS=4 timeout -k 10 400 bash tools/gs_ab.sh "" "GS_LIB=libptgs_pr0.so" > $O/ab.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -k "gaussian or splat or tight or raster or hybrid or c4 or c5 or pt or dist" > $O/pytest.log 2>&1 || exit 1
exit 0
