#!/bin/bash
# PMC passes for configs 2 and 3 over bench.py (one counter group per run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
G="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES;SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum,TCC_MISS_sum,GRBM_GUI_ACTIVE"
for c in ${CFGS:-2 3}; do
  PMC_OUT=gpurun_out/pmc_c$c GROUPS_LIST="${GROUPS_LIST:-$G}" BENCH_ARGS="--no-cpu-baseline --steps 5 --warmup 2 --config $c" bash tools/pmc.sh || exit $?
done
