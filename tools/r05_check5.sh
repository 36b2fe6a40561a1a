#!/bin/bash
# round-5 GPU step: tests, C2 / 1M vs round 4, band front ends
set -uo pipefail
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
GS_AB_ROUNDS=2 timeout -k 10 200 bash tools/gs_ab.sh "" "GS_LIB=libptgs_base.so" > $O/ab.log 2>&1 || exit 1
GS_N=1000000 GS_FRAMES=60 GS_AB_ROUNDS=2 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_base.so" > $O/ab_1m.log 2>&1 || exit 1
GS_CFGS="10m c2" timeout -k 10 600 bash tools/gs_bands.sh > $O/bands.log 2>&1 || exit 1
for d in gpurun_out/gsb_*; do python3 tools/kt_summary.py $d; done > $O/bands_kt.txt 2>&1
mv gpurun_out/gsb_* $O/ 2>/dev/null
exit 0
