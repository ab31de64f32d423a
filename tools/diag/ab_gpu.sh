#!/bin/bash
# GPU: parity suite on the in-tree build (NOTEST=1 skips it), then the
# one-process A/B of tools/diag/lib_*.so (ab_libs.py) on CFGS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=${OUT:-gpurun_out/ab}; mkdir -p $O
if [ "${NOTEST:-0}" = 0 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 400 python -u tools/diag/ab_libs.py ${CFGS:-3 2 5} > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
