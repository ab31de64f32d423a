#!/bin/bash
# One PMC pass (LDS / VALU utilisation) over the decode-only driver per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for CFG in ${CFGS:-2 3}; do
  OUT=gpurun_out/pmclds$CFG; rm -rf $OUT; mkdir -p $OUT
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INST_LEVEL_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
     -d $OUT/p1 -o run --output-format csv -- python3 tools/diag/dec_only.py $CFG 5 > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
  echo "== config $CFG"; python3 tools/diag/pmc_sum.py $OUT k_decode
done
