#!/bin/bash
# Two PMC passes (issue / wait breakdown) over the encode-only driver, per
# kernel (k_enc_count, k_encode).  Usage: OUT=gpurun_out/pmcenc CFGS="3" tools/diag/pmc_enc2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/pmcenc}
for CFG in ${CFGS:-3}; do
  D=$O/c$CFG; rm -rf $D; mkdir -p $D
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INST_LEVEL_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
     -d $D/p1 -o run --output-format csv -- python3 tools/diag/enc_only.py $CFG 5 > $D/p1.log 2>&1 || { tail -5 $D/p1.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_BRANCH \
     -d $D/p2 -o run --output-format csv -- python3 tools/diag/enc_only.py $CFG 5 > $D/p2.log 2>&1 || { tail -5 $D/p2.log; exit 1; }
  for k in k_enc_count k_encode; do echo "== config $CFG $k"; python3 tools/diag/pmc_sum.py $D "$k<" | tee $D/summary_$k.txt; done
done
