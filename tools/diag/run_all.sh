#!/bin/bash
# GPU box: parity tests, phase stamps, variant timing (configs 2 and 3) and
# the decode PMC passes; each GPU step under its own time limit, stopping at
# the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/diag
timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/diag/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/diag/pytest.log
[ $rc -le 1 ] || exit $rc
for c in 2 3; do
  timeout -k 10 200 python tools/diag/time_variants.py $c > gpurun_out/diag/tv$c.json 2>&1 || exit $?
done
[ -n "${NO_PMC:-}" ] || bash tools/diag/pmc_dec.sh 2
