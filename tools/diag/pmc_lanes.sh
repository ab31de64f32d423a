#!/bin/bash
# PMC passes (issue / wait / LDS / memory pipeline) over the lane decoder.
# Usage: OUT=gpurun_out/r03/pmc CFGS="3 2" tools/diag/pmc_lanes.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/pmclanes}
for CFG in ${CFGS:-3 2}; do
  D=$O/c$CFG; rm -rf $D; mkdir -p $D
  i=0
  for SET in \
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
    "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
    "SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_SCA TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" ; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $SET -d $D/p$i -o run --output-format csv -- python3 tools/diag/dec_lanes.py $CFG 5 > $D/p$i.log 2>&1 || { tail -5 $D/p$i.log; exit 1; }
  done
  echo "== config $CFG"; python3 tools/diag/pmc_sum.py $D k_decode_lanes | tee $D/summary.txt
done
