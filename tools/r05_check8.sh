#!/bin/bash
# round-5 GPU step: near/far plane box test (PTGS_PT_NEARFAR) vs min/max, C3 megakernel + wavefront; PT parity tests
set -uo pipefail
O=gpurun_out/r05j; mkdir -p $O
AB_SPP=16 AB_ROUNDS=4 timeout -k 10 200 python3 tools/ab_pt.py base nf0 > $O/ab.log 2>&1 || exit 1
AB_WF=1 AB_SPP=16 AB_ROUNDS=3 timeout -k 10 200 python3 tools/ab_pt.py base nf0 >> $O/ab.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_pt_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
exit 0
