#!/bin/bash
# round-5 GPU step: traversal tweaks A/B (sorted-hit count, asm min) on C3; then the bench
set -uo pipefail
O=gpurun_out/r05k; mkdir -p $O
AB_SPP=16 AB_ROUNDS=4 timeout -k 10 200 python3 tools/ab_pt.py base sh am sham > $O/ab.log 2>&1 || exit 1
timeout -k 10 640 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || exit 1
exit 0
