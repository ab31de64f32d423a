#!/bin/bash
# GPU parity suite on the current build, then the one-process decode A/B
# (tools/diag/ab_decode.py) against the tools/diag/lib_*.so variants.
# Usage: OUT=gpurun_out/ab1 CFGS="3 2 5" tools/diag/ab_run.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/ab}; mkdir -p $O
if [ "${NOTEST:-0}" = 0 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 400 python -u tools/diag/ab_decode.py ${CFGS:-3 2 5} > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
