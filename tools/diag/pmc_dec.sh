#!/bin/bash
# PMC passes over the decode-only driver (one counter group per run,
# --kernel-trace only).  Usage: pmc_dec.sh <config>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
CFG=${1:-2}
OUT=gpurun_out/pmc${DRIVER:-dec_only}$CFG
rm -rf $OUT; mkdir -p $OUT
G=("SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES"
   "SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS"
   "SQ_LDS_BANK_CONFLICT,SQ_LDS_ADDR_CONFLICT,SQ_LDS_UNALIGNED_STALL,SQ_LDS_IDX_ACTIVE,SQ_LDS_CMD_FIFO_FULL,SQ_LDS_DATA_FIFO_FULL"
   "SQ_IFETCH,SQ_IFETCH_LEVEL,SQ_INST_LEVEL_LDS,SQ_INSTS_BRANCH,SQ_INST_CYCLES_SALU,SQ_INSTS_SMEM")
i=0
for g in "${G[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc ${g//,/ } -d $OUT/p$i -o run --output-format csv \
      -- python3 tools/diag/${DRIVER:-dec_only}.py $CFG 5 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
