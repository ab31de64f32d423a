#!/bin/bash
# Instruction mix and waits of the three hot kernels on config 3 (one stream):
# two PMC passes, each its own run and limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=${OUT:-gpurun_out/r7pmc}; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-secondary --streams 1 --steps 5 --warmup 2 --config 3"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- $B > $O/p1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/p2 -o run --output-format csv -- $B > $O/p2.log 2>&1 || exit 1
for k in k_decode_items k_encode k_enc_count; do echo "== $k"; python3 tools/diag/pmc_sum.py $O $k; done > $O/summary.txt
