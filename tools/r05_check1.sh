#!/bin/bash
# round-5 GPU step: stripped library bit-exact vs the round-4 library, GPU tests, write-through A/B, C2 timeline
set -uo pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 120 python3 tools/gs_ab_check.py base > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py base wt7 >> $O/check.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
GS_AB_ROUNDS=2 timeout -k 10 400 bash tools/gs_ab.sh "" "GS_LIB=libptgs_wt1.so" "GS_LIB=libptgs_wt2.so" "GS_LIB=libptgs_wt4.so" "GS_LIB=libptgs_wt6.so" "GS_LIB=libptgs_wt7.so" > $O/ab.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
GS_SORTED=2 GS_N=100000 GS_STAGES=0 timeout -k 10 120 rocprofv3 --kernel-trace -d $O/kt_base -o run --output-format csv -- python3 tools/gs_probe.py base > $O/kt_base.log 2>&1 || exit 1
python3 tools/kt_timeline.py $O/kt_base 24 > $O/timeline_base.txt 2>&1
GS_SORTED=2 GS_N=100000 GS_STAGES=0 timeout -k 10 120 rocprofv3 --kernel-trace -d $O/kt_wt7 -o run --output-format csv -- python3 tools/gs_probe.py wt7 > $O/kt_wt7.log 2>&1 || exit 1
python3 tools/kt_timeline.py $O/kt_wt7 24 > $O/timeline_wt7.txt 2>&1
