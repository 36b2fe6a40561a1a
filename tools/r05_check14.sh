#!/bin/bash
# round-5 GPU step: the box test without the far-distance slack (PTGS_PT_SLACK=0, padding only): A/B on C3
# (megakernel + wavefront), then every path-tracer parity test against that library (copied over
# libptgs.so in this box's scratch copy of the tree)
set -uo pipefail
O=gpurun_out/r05s; mkdir -p $O
AB_SPP=16 AB_ROUNDS=4 timeout -k 10 200 python3 tools/ab_pt.py base ns > $O/ab.log 2>&1 || exit 1
AB_WF=1 AB_SPP=16 AB_ROUNDS=3 timeout -k 10 200 python3 tools/ab_pt.py base ns >> $O/ab.log 2>&1 || exit 1
cp pathtracer_gaussiansplatting_amd/libptgs_ns.so pathtracer_gaussiansplatting_amd/libptgs.so || exit 1
timeout -k 10 900 python -u -m pytest tests/test_pt_gpu.py tests/test_configs_gpu.py tests/test_hybrid_gpu.py tests/test_capture_gpu.py -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/pytest.log
exit 0
