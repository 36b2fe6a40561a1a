#!/bin/bash
# PMC passes over the C2 3DGS loop (tools/gs_probe.py, device Morton order with ids = the bench's timed
# mode) for the given library variant: LDS / VALU / wait counters, one rocprofv3 run per pass.
#   tools/gs_pmc.sh [variant] -> gpurun_out/gs_pmc_<variant>/p{1,2}; summarise with tools/pmc_kernels.py
set -euo pipefail
V=${1:-base}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/gs_pmc_$V
mkdir -p $OUT
P1="SQ_BUSY_CU_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_LDS_DATA_FIFO_FULL SQ_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  GS_SORTED=2 GS_STAGES=0 GS_ITERS=${GS_ITERS:-30} timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv \
    -- python3 tools/gs_probe.py $V > $OUT/p$i.log 2>&1
done
python3 tools/pmc_kernels.py $OUT/p1 $OUT/p2 --match gs_
