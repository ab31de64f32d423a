#!/bin/bash
# PMC passes (issue / wait / LDS latency and conflicts) over the decode-only
# driver, per config; one rocprofv3 run per pass, each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
K=${KERNEL:-k_decode_items}
DRV=${DRIVER:-tools/diag/dec_only.py}
for CFG in ${CFGS:-3 2}; do
  OUT=gpurun_out/pmcdd$CFG; rm -rf $OUT; mkdir -p $OUT
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
     -d $OUT/p1 -o run --output-format csv -- python3 $DRV $CFG 5 > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH \
     -d $OUT/p2 -o run --output-format csv -- python3 $DRV $CFG 5 > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
  echo "== config $CFG ($K)"; for k in $K; do python3 tools/diag/pmc_sum.py $OUT $k; done
done
