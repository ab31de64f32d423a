#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only, as
# MI355X_MICROARCH.md prescribes) over a short bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${PMC_OUT:-gpurun_out/pmc}; rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---no-cpu-baseline --steps 5 --warmup 2}"
i=0
for grp in "${PMC_GROUPS[@]:-}" ; do :; done
GROUPS_LIST=${GROUPS_LIST:-"SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES;SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_INST_CYCLES_VMEM;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum,TCC_MISS_sum,GRBM_GUI_ACTIVE"}
IFS=';' read -ra G <<< "$GROUPS_LIST"
for g in "${G[@]}"; do
  i=$((i+1))
  echo "== pmc pass $i: $g"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${g//,/ } -d $OUT/p$i -o run \
      --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 2 $OUT/p$i.log
  if [ $rc -ne 0 ]; then echo "stopping after pass $i"; exit $rc; fi
done
