#!/bin/bash
# The blend's phase split: for each library variant (probe builds, splat_probe.h: base,
# p8 = no exact quadrant test, p1 = no evaluation, p9 = + no exact test, p13 = + identity ranks, p15 = +
# no record gather), over the C2 loop in the timed mode (tools/gs_probe.py, device Morton order with ids):
# a kernel trace and three --pmc passes (SQ instruction counts, waits, VMEM / SMEM / branch counts).
#   tools/gs_phase.sh <out-dir> base p8 p1 ...      summarise: tools/gs_phase.py <out-dir>
set -euo pipefail
OUT=${1:?out dir}
shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P1="SQ_BUSY_CU_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_LDS_DATA_FIFO_FULL SQ_BUSY_CYCLES"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_FLAT"
for v in "$@"; do
  mkdir -p "$OUT/$v"
  GS_SORTED=2 GS_STAGES=0 GS_ITERS=${GS_ITERS:-60} timeout -k 10 90 rocprofv3 --kernel-trace --stats -d "$OUT/$v/kt" -o run \
    --output-format csv -- python3 tools/gs_probe.py "$v" > "$OUT/$v/kt.log" 2>&1
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    GS_SORTED=2 GS_STAGES=0 GS_ITERS=${GS_ITERS:-30} timeout -s KILL 90 rocprofv3 --pmc $P -d "$OUT/$v/p$i" -o run \
      --output-format csv -- python3 tools/gs_probe.py "$v" > "$OUT/$v/p$i.log" 2>&1
  done
done
