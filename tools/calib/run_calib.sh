#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/calib; export TMPDIR=/tmp
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/calib/$c -o run --output-format csv -- ./tools/calib/calib > gpurun_out/calib/$c.log 2>&1 || exit $?
done
echo calib ok
